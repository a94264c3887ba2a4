set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/probe/gemm_noload.py run > gpurun_out/noload_hw.json 2> gpurun_out/noload_hw.err
cat gpurun_out/noload_hw.json
