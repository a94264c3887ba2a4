set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_gpt2_grpo.py -v --timeout 300 --timeout-method thread > gpurun_out/r02_t9.log 2>&1; echo "tests rc=$?" >> gpurun_out/r02_t9.log
