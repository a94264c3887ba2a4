set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocabs.py -k "prologue or sampler_bit_exact" -x -q --timeout 120 --timeout-method thread > gpurun_out/sampler_pre_tests.log 2>&1 || { tail -30 gpurun_out/sampler_pre_tests.log; exit 1; }
echo "tests ok"
timeout -k 10 240 python -u scripts/probe/sampler_row_probe.py > gpurun_out/sampler_pre_probe.json 2> gpurun_out/sampler_pre_probe.err
cat gpurun_out/sampler_pre_probe.json
