set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_agent_e2e.py tests/test_gpu_trainer_e2e.py tests/test_gpu_pause_continue.py -x -q --timeout 240 --timeout-method thread > gpurun_out/engine_auto_tests.log 2>&1 || { tail -30 gpurun_out/engine_auto_tests.log; exit 1; }
tail -1 gpurun_out/engine_auto_tests.log
