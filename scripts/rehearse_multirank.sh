#!/bin/bash
# Rehearse bench.py's N>1 path (sharded optimizer, reduce-scatter / all-gather on the comm
# stream, metric all-reduce, barrier + max-over-ranks timing) with 2 ranks on ONE GPU over
# gloo: RCCL refuses two ranks on the same device, the 8-GPU RCCL run is the driver's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --logits-rows 16384 \
  --params 10000000 --bucket-mb 8 > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err
rc=$?
cat gpurun_out/rehearse_n2.json
exit $rc
