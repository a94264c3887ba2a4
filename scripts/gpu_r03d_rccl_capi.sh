set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_capi.py tests/test_capi.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_rccl_capi_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r03d_rccl_capi_tests.log; exit $rc
