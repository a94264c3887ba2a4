#!/bin/bash
# r05l: the whole GPU suite, smoke, bench N=1 (default legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05l_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r05l_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05l_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r05l_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/probe/split_wpe.py run > gpurun_out/r05l_split_wpe.json 2>&1
rc=$?; tail -1 gpurun_out/r05l_split_wpe.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err
rc=$?; tail -c 300 gpurun_out/r05l_bench.json; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05l_bench.err; exit $rc; }
