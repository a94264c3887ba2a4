#!/bin/bash
# rocprofv3 passes for bench.py: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950). No sys/runtime trace with PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-e2e}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ "${PMC:-1}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "${PMC_REGEX:-logprob|grpo|ppo_loss|sample_kernel|pack|policy_train|paged_decode|lmhead_gemm}" --output-format csv -d $OUT/pmc_$c -o run -- python3 bench.py $ARGS > $OUT/pmc_$c.log 2>&1
    rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
find $OUT -name "*.csv" | head -50
