set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_lmhead_sample.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lm_bar_tests.log 2>&1 || { tail -30 gpurun_out/lm_bar_tests.log; exit 1; }
tail -1 gpurun_out/lm_bar_tests.log
timeout -k 10 200 python -u scripts/probe/lmhead_phase_probe.py run > gpurun_out/lmhead_phase3.json 2> gpurun_out/lmhead_phase3.err
timeout -k 10 300 python -u scripts/probe/lmhead_sample_bench.py --T 1.0 0.7 0.0 --M 512 256 64 8 > gpurun_out/lms_bench_bar.json 2> gpurun_out/lms_bench_bar.err
cat gpurun_out/lms_bench_bar.json
