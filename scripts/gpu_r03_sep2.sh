set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -p no:cacheprovider tests/test_gpu_separated.py > gpurun_out/r03_separated.log 2>&1; rc=$?; tail -30 gpurun_out/r03_separated.log; exit $rc
