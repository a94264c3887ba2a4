set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lmhead_sample.py -k "grouped" -x -q --timeout 120 --timeout-method thread > gpurun_out/grouped_tests.log 2>&1 || { tail -30 gpurun_out/grouped_tests.log; exit 1; }
tail -2 gpurun_out/grouped_tests.log
