set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_vocabs.py tests/test_gpu_parity.py tests/test_gpu_worker.py tests/test_gpu_trainer.py -q --timeout 240 --timeout-method thread > gpurun_out/r02_t8.log 2>&1; echo "tests rc=$?" >> gpurun_out/r02_t8.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-attention-leg > gpurun_out/r02_b8.json 2> gpurun_out/r02_b8.err
