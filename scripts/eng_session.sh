set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -v --timeout 300 --timeout-method thread > gpurun_out/eng_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -${TAILN:-30} gpurun_out/eng_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
if [ "${RUN_BENCH:-1}" = 1 ]; then
timeout -k 10 400 python -u scripts/probe/engine_bench.py --max-tokens 128 ${BENCH_ARGS:-} > gpurun_out/engine_bench.json 2> gpurun_out/engine_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/engine_bench.json; tail -5 gpurun_out/engine_bench.err
fi
