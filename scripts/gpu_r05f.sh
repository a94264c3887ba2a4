#!/bin/bash
# r05f: wide step plan (+GRPO) / fold, sampler default grid, bench N=1 and per-rank shares
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_gpu_policy_train_step.py tests/test_gpu_policy_train_split.py tests/test_gpu_sampler_splits.py \
  tests/test_gpu_parity.py tests/test_gpu_worker.py tests/test_gpu_trainer.py tests/test_gpu_grpo_loss_fused.py \
  > gpurun_out/r05f_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || exit $rc
NOLEGS="--no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs --no-filtered-leg"
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > gpurun_out/r05f_$name.json 2> gpurun_out/r05f_$name.err
  local rc=$?
  tail -c 300 gpurun_out/r05f_$name.json; echo
  [ $rc -eq 0 ] || { tail -20 gpurun_out/r05f_$name.err; exit $rc; }
}
run n1 300 --steps 3 --warmup 1 $NOLEGS
for W in 2 4 8; do run emu$W 240 --steps 3 --warmup 1 --emulate-world $W $NOLEGS; done
