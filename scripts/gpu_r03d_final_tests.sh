set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_pytest_gpu_final.log 2>&1; rc=$?
tail -3 gpurun_out/r03d_pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke_final.log 2>&1; rc=$?; tail -1 gpurun_out/r03d_smoke_final.log; exit $rc
