#!/bin/bash
# r05t: rocprofv3 kernel stats of the per-rank (N = 8) step emulation: is the 64-row training launch slower itself?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
NOLEGS="--no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs --no-filtered-leg"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05t/emu8 -o run -- python3 bench.py --steps 2 --warmup 1 --emulate-world 8 $NOLEGS > gpurun_out/r05t/emu8.log 2>&1
rc=$?; echo "emu8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05t/n1 -o run -- python3 bench.py --steps 2 --warmup 1 $NOLEGS > gpurun_out/r05t/n1.log 2>&1
rc=$?; echo "n1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
