#!/bin/bash
# r05 final tree (after the bar-publish change): the whole GPU suite + smoke, bench N=1 (default), per-rank emulation at N=8,
# rocprofv3 kernel stats of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05final2_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r05final2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05final2_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r05final2_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r05final2_bench.json 2> gpurun_out/r05final2_bench.err
rc=$?; tail -c 300 gpurun_out/r05final2_bench.json; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05final2_bench.err; exit $rc; }
timeout -k 10 400 python -u bench.py --emulate-world 8 --no-cpu-baseline --no-e2e --no-adv-loss-leg --no-attention-leg \
  --no-lmhead-leg --no-vocab-legs --no-filtered-leg > gpurun_out/r05final2_emu8.json 2> gpurun_out/r05final2_emu8.err
rc=$?; tail -c 300 gpurun_out/r05final2_emu8.json; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05final2_emu8.err; exit $rc; }
OUT=gpurun_out/r05final2_prof
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py \
  --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/trace.log 2>&1
echo "trace rc=$?"
