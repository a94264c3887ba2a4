set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "n_samples" > gpurun_out/r02_eng_test.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r02_eng_test.log
