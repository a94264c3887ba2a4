#!/bin/bash
# r05h: top_p pass 1 records per wave, pass-2 slots, cut timing probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_sampler_topp_fast.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_sampler_splits.py tests/test_gpu_sampler_stats.py \
  > gpurun_out/r05h_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05h_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/topp_variants.py run > gpurun_out/r05h_topp_variants.json 2>&1
rc=$?; tail -1 gpurun_out/r05h_topp_variants.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/probe/topp_probe.py > gpurun_out/r05h_topp_probe.json 2>&1
rc=$?; tail -c 3000 gpurun_out/r05h_topp_probe.json; echo; [ $rc -eq 0 ] || exit $rc
