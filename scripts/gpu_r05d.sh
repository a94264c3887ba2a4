#!/bin/bash
# r05d: split training pass (partner states computed in place, contention test), split-sampler phases,
# bench N=1 and one 8-rank share.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_policy_train_split.py tests/test_gpu_policy_train_step.py tests/test_gpu_vocabs.py \
  > gpurun_out/r05d_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05d_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/probe/sampler_split_phase.py run > gpurun_out/r05d_split_phase.json 2> gpurun_out/r05d_split_phase.err
rc=$?; cat gpurun_out/r05d_split_phase.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05d_split_phase.err; exit $rc; }
NOLEGS="--no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs --no-filtered-leg"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $NOLEGS > gpurun_out/r05d_n1.json 2> gpurun_out/r05d_n1.err
rc=$?; tail -c 300 gpurun_out/r05d_n1.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05d_n1.err; exit $rc; }
timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --emulate-world 8 $NOLEGS > gpurun_out/r05d_emu8.json 2> gpurun_out/r05d_emu8.err
rc=$?; tail -c 300 gpurun_out/r05d_emu8.json; exit $rc
