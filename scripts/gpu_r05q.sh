#!/bin/bash
# r05q: the N > 1 bench path -- 2 gloo ranks on one GPU (strong scaling, in-flight weight sync) and
# one RCCL rank with every exchange forced to a collective
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --logits-rows 16384 \
  --params 10000000 --bucket-mb 8 --no-e2e --no-cpu-baseline > gpurun_out/r05q_gloo_n2.json 2> gpurun_out/r05q_gloo_n2.err
rc=$?; tail -c 600 gpurun_out/r05q_gloo_n2.json; echo; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05q_gloo_n2.err; exit $rc; }
SKYRL_FORCE_COLLECTIVES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 1 --steps 2 --warmup 1 --weight-sync inflight \
  --no-e2e --no-cpu-baseline > gpurun_out/r05q_rccl_solo.json 2> gpurun_out/r05q_rccl_solo.err
rc=$?; tail -c 600 gpurun_out/r05q_rccl_solo.json; echo; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05q_rccl_solo.err; exit $rc; }
AB_DEFINE=SKYRL_SEED_BARRIER timeout -k 10 200 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05q_ab_seedbar.json 2>&1
rc=$?; tail -1 gpurun_out/r05q_ab_seedbar.json; [ $rc -eq 0 ] || exit $rc
