set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lmhead_sample.py -k "pipeline_variants" -x -q --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -1 gpurun_out/pp_tests.log
timeout -k 10 400 python -u scripts/probe/gemm_noload.py run > gpurun_out/pipe14.json 2> gpurun_out/pipe14.err
cat gpurun_out/pipe14.json
