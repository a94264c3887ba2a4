set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lmhead_sample.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02_lms_test.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r02_lms_test.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python scripts/probe/lmhead_sample_bench.py --T 1.0 0.0 > gpurun_out/r02_lms_bench.json 2> gpurun_out/r02_lms_bench.err || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-vocab-legs > gpurun_out/r02_bench_coherent.json 2> gpurun_out/r02_bench_coherent.err
