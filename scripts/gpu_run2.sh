set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lmhead_sample.py -x -q --timeout 200 --timeout-method thread -k "pipeline or exact or sample_equals" > gpurun_out/r02_lms_test.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r02_lms_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python scripts/probe/lmhead_sample_bench.py --gemm-sweep > gpurun_out/r02_gemm_sweep.json 2> gpurun_out/r02_gemm_sweep.err
