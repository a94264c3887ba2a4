set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocabs.py -q --timeout 200 --timeout-method thread -k "persistent or policy_train" > gpurun_out/r02_t11.log 2>&1; echo "tests rc=$?" >> gpurun_out/r02_t11.log
timeout -k 10 300 python scripts/kbench.py --only fused --rounds 5 > gpurun_out/r02_kb11.json 2> gpurun_out/r02_kb11.err
