set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler_stats.py -v --timeout 200 --timeout-method thread > gpurun_out/r02_t10.log 2>&1; echo "tests rc=$?" >> gpurun_out/r02_t10.log
