set -o pipefail
mkdir -p gpurun_out
bash scripts/rehearse_multirank.sh > gpurun_out/r02_rehearse.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_multirank_test.log 2>&1; echo "tests rc=$?" >> gpurun_out/r02_multirank_test.log
