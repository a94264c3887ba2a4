#!/bin/bash
# r05p: sampler A/B (lazy workgroup bar) + the sampler suites
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05p_ab.json 2>&1
rc=$?; tail -1 gpurun_out/r05p_ab.json; [ $rc -eq 0 ] || exit $rc
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_sampler_splits.py tests/test_gpu_sampler_stats.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_parity.py > gpurun_out/r05p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05p_tests.log; [ $rc -eq 0 ] || exit $rc
