#!/bin/bash
# One GPU session: gpu tests -> smoke -> bench. Each step has its own time limit; any
# fault/abort/timeout (exit >= 124 or signal) stops the session before the next GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_if_fatal() {  # $1 = rc, $2 = step
  if [ "$1" -ge 124 ] || [ "$1" -lt 0 ]; then echo "FATAL rc=$1 in $2: stopping" | tee -a $OUT/session.log; exit "$1"; fi
}
echo "start $(date)" > $OUT/session.log
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a $OUT/session.log; tail -5 $OUT/pytest_gpu.log; stop_if_fatal $rc pytest
fi
if [ "${RUN_SMOKE:-1}" = 1 ]; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc" | tee -a $OUT/session.log; tail -3 $OUT/smoke.log; stop_if_fatal $rc smoke
fi
if [ "${RUN_BENCH:-1}" = 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 2 --warmup 1} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc" | tee -a $OUT/session.log; cat $OUT/bench.json; tail -5 $OUT/bench.err; stop_if_fatal $rc bench
fi
echo "done $(date)" >> $OUT/session.log
