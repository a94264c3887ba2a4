#!/bin/bash
# r05 final tree (after the top_p bar forms): the whole GPU suite + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05final3_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r05final3_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05final3_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r05final3_smoke.log; [ $rc -eq 0 ] || exit $rc
