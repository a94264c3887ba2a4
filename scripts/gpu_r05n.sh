#!/bin/bash
# r05n: the whole GPU suite + smoke, then rocprofv3 stats and FETCH/WRITE PMC of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05n_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r05n_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05n_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r05n_smoke.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r05n_prof
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
ARGS2="--steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "logprob|grpo|sample|pack|policy_train|train_plan|train_fold|adamw|sumsq" --output-format csv -d $OUT/pmc_$c -o run -- python3 bench.py $ARGS2 > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
