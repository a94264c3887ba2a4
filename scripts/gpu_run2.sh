set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lmhead_sample.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_lms_test.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r02_lms_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/probe/lmhead_sample_bench.py --T 1.0 0.7 0.0 --M 512 256 64 8 --pipes 4 4 --iters 40 > gpurun_out/r02_lms_bench4.json 2> gpurun_out/r02_lms_bench4.err
