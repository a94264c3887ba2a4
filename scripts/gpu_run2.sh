set -eu
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/probe/ws_reuse_check.py > gpurun_out/ws_reuse_old.log 2>&1 || true
grep -v amdgpu.ids gpurun_out/ws_reuse_old.log | tail -8
