#!/bin/bash
# r05j: top_p pass 2 inside the pass-1 launch (piece queue)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_sampler_topp_fast.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_sampler_splits.py \
  > gpurun_out/r05j_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05j_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/topp_variants.py run > gpurun_out/r05j_topp_variants.json 2>&1
rc=$?; tail -1 gpurun_out/r05j_topp_variants.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/probe/topp_probe.py > gpurun_out/r05j_topp_probe.json 2>&1
rc=$?; tail -c 3000 gpurun_out/r05j_topp_probe.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $T tests/test_gpu_policy_train_step.py tests/test_gpu_policy_train_split.py tests/test_gpu_grpo_loss_fused.py tests/test_gpu_parity.py tests/test_gpu_vocabs.py > gpurun_out/r05j_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/r05j_tests2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/adamw_probe.py > gpurun_out/r05j_adamw_probe.json 2>&1
rc=$?; tail -2 gpurun_out/r05j_adamw_probe.json; [ $rc -eq 0 ] || exit $rc
