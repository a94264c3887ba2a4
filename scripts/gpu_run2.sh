set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocabs.py tests/test_gpu_parity.py tests/test_gpu_sampler_stats.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sampler_tests.log 2>&1 || { tail -30 gpurun_out/sampler_tests.log; exit 1; }
tail -1 gpurun_out/sampler_tests.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-e2e > gpurun_out/bench_prio.json 2> gpurun_out/bench_prio.err
python3 -c "import json;d=json.load(open('gpurun_out/bench_prio.json'));print(d['value'], d['ms_per_step'], {k:(v['avg_launch_ms'],v['ms_per_step']) for k,v in d['kernels'].items()})"
