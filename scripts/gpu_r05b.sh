#!/bin/bash
# r05b: sampler at per-rank row counts (eager vs graph, rocprof), the per-parameter AdamW and the
# trainer's in-flight weight wait.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/probe/sampler_rows_probe.py > gpurun_out/r05b_rows.json 2> gpurun_out/r05b_rows.err
rc=$?; cat gpurun_out/r05b_rows.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05b_rows.err; exit $rc; }
ROWS=64,256 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b_prof -o rows -- \
  python3 scripts/probe/sampler_rows_probe.py > gpurun_out/r05b_rows_prof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05b_rows_prof.log; exit $rc; }
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_optim.py tests/test_gpu_trainer_e2e.py > gpurun_out/r05b_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r05b_tests.log; exit $rc
