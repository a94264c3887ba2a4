set -eu
mkdir -p gpurun_out/gemm12
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probe/lmhead_sample_bench.py --T 1.0 0.0 --M 512 256 64 8 > gpurun_out/lms_bench.json 2> gpurun_out/lms_bench.err
cat gpurun_out/lms_bench.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gemm12/t512 -o run -- python3 scripts/probe/gemm_once.py 512 > gpurun_out/gemm12/t512.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gemm12/t8192 -o run -- python3 scripts/probe/gemm_once.py 8192 > gpurun_out/gemm12/t8192.log 2>&1
echo prof ok
