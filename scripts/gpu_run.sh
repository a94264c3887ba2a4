#!/bin/bash
# One parameterised GPU session (run on the box through gpurun): each step writes under
# gpurun_out/<tag>_*, runs under its own time limit, and the first failing step ends the call.
#
#   gpurun --timeout 1200 -- bash scripts/gpu_run.sh <tag> <step> [<step> ...]
#
# steps:
#   tests[:EXPR]   pytest -m gpu (optionally -k EXPR), -x, per-test 120 s limit
#   files:F1,F2    pytest -m gpu on the given test files only
#   smoke          __graft_entry__.smoke()
#   bench          python bench.py (the driver's default run)
#   emu8           bench.py --emulate-world 8 (one rank's share of an 8-GPU job), no side legs
#   prof           rocprofv3 --kernel-trace --stats of a short bench run (N = 1)
#   prof_emu8      the same for the emu8 run
#   pmc_emu8:CTRS  one rocprofv3 --pmc pass (counters CTRS, comma-separated) over the emu8 run
#   pmc:CTRS       the same over the N = 1 run
#   py:SCRIPT      python SCRIPT (a probe; its own output)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
NOLEGS="--no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs --no-filtered-leg"
step_rc() {  # name rc log
  echo "[$TAG] $1 rc=$2"
  if [ "$2" -ne 0 ]; then
    [ -n "$3" ] && tail -30 "$3"
    exit "$2"
  fi
}
for S in "$@"; do
  name=${S%%:*}
  arg=${S#*:}
  [ "$arg" = "$S" ] && arg=""
  O=gpurun_out/${TAG}_${name}
  case $name in
    tests)
      K=()
      [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider "${K[@]}" > $O.log 2>&1
      rc=$?; tail -3 $O.log; step_rc tests $rc $O.log ;;
    files)
      timeout -k 10 1100 python -u -m pytest ${arg//,/ } -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > $O.log 2>&1
      rc=$?; tail -3 $O.log; step_rc files $rc $O.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O.log 2>&1
      rc=$?; tail -2 $O.log; step_rc smoke $rc $O.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > $O.json 2> $O.err
      rc=$?; tail -c 400 $O.json; echo; step_rc bench $rc $O.err ;;
    emu8)
      timeout -k 10 400 python -u bench.py --emulate-world 8 $NOLEGS > $O.json 2> $O.err
      rc=$?; tail -c 400 $O.json; echo; step_rc emu8 $rc $O.err ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 bench.py \
        --steps 2 --warmup 1 $NOLEGS > $O.log 2>&1
      rc=$?; step_rc prof $rc $O.log ;;
    prof_emu8)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 bench.py \
        --steps 2 --warmup 1 --emulate-world 8 $NOLEGS > $O.log 2>&1
      rc=$?; step_rc prof_emu8 $rc $O.log ;;
    pmc_emu8|pmc)
      EXTRA=""
      [ $name = pmc_emu8 ] && EXTRA="--emulate-world 8"
      timeout -s KILL 400 rocprofv3 --pmc ${arg//,/ } --kernel-trace --kernel-include-regex "${PMC_REGEX:-policy_train|sample_kernel|logprob}" --output-format csv -d $O -o run -- python3 bench.py \
        --steps 1 --warmup 1 $EXTRA $NOLEGS > $O.log 2>&1
      rc=$?; step_rc $name $rc $O.log ;;
    py)
      timeout -k 10 600 python -u $arg > $O.log 2>&1
      rc=$?; tail -5 $O.log; step_rc py $rc $O.log ;;
    *)
      echo "unknown step $S"; exit 2 ;;
  esac
done
