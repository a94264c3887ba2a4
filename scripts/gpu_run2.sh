set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/kbench.py --only fused_mb --rounds 5 > gpurun_out/kbench_mb.json 2> gpurun_out/kbench_mb.err
cat gpurun_out/kbench_mb.json
