set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -v --timeout 180 --timeout-method thread > gpurun_out/eng_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/eng_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/probe/engine_bench.py --max-tokens 128 > gpurun_out/engine_bench.json 2> gpurun_out/engine_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/engine_bench.json; tail -5 gpurun_out/engine_bench.err
