#!/bin/bash
# r05e: split-sampler granularity / grid sweep at the per-rank row counts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_sampler_splits.py > gpurun_out/r05e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_tests.log; [ $rc -eq 0 ] || exit $rc
ROWS=64,128 SETTINGS=256:2048,1024:1024:8192,1024:960:2048,1024:1024:2048,1024:768:2048,1024:512:2048,1024:1536:2048,1024:2048:2048,1024:1024:4096,1024:768:4096 \
  timeout -k 10 300 python -u scripts/probe/sampler_rows_probe.py > gpurun_out/r05e_rows.json 2> gpurun_out/r05e_rows.err
rc=$?; cat gpurun_out/r05e_rows.json; exit $rc
