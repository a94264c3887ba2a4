#!/bin/bash
# r05g: plan from pack row sums + fold loads; bench N=1 (all legs); rocprofv3 stats + FETCH/WRITE PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_policy_train_step.py tests/test_gpu_trainer.py \
  > gpurun_out/r05g_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r05g_bench.json 2> gpurun_out/r05g_bench.err
rc=$?; tail -c 400 gpurun_out/r05g_bench.json; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05g_bench.err; exit $rc; }
OUT=gpurun_out/r05g_prof
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
ARGS2="--steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs --no-filtered-leg"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "logprob|grpo|sample_kernel|pack|policy_train|train_plan|train_fold|adamw|sumsq" --output-format csv -d $OUT/pmc_$c -o run -- python3 bench.py $ARGS2 > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find $OUT -name "*.csv"
