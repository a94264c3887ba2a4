set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_e2e.py -v --timeout 240 --timeout-method thread > gpurun_out/r02_t7.log 2>&1; echo "tests rc=$?" >> gpurun_out/r02_t7.log
