set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_agent_e2e.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_agent_test.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r02_agent_test.log
