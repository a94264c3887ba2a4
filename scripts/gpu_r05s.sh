#!/bin/bash
# r05s: row-mode sampler with waves drawing chunks from an LDS counter: A/B + the sampler suites
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_DEFINE=SKYRL_DYN_WAVES timeout -k 10 200 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05s_ab_dyn.json 2>&1
rc=$?; tail -1 gpurun_out/r05s_ab_dyn.json; [ $rc -eq 0 ] || exit $rc
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_sampler_splits.py tests/test_gpu_sampler_stats.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_sampler_topp_fast.py tests/test_gpu_parity.py > gpurun_out/r05s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05s_tests.log; [ $rc -eq 0 ] || exit $rc
