#!/bin/bash
# r05a: strong-scaling bench: N=1 unchanged, one rank's share of a 2/4/8-rank job on one GPU,
# and the 2-rank gloo rehearsal of the in-flight comm chain.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NOLEGS="--no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs --no-filtered-leg"
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > gpurun_out/r05a_$name.json 2> gpurun_out/r05a_$name.err
  local rc=$?
  tail -c 400 gpurun_out/r05a_$name.json; echo
  [ $rc -eq 0 ] || { tail -20 gpurun_out/r05a_$name.err; exit $rc; }
}
run n1 300 --steps 3 --warmup 1 $NOLEGS
for W in 2 4 8; do
  run emu$W 240 --steps 3 --warmup 1 --emulate-world $W $NOLEGS
done
run emu8_inflight 240 --steps 3 --warmup 1 --emulate-world 8 --weight-sync inflight $NOLEGS
run n1_inflight 300 --steps 3 --warmup 1 --weight-sync inflight $NOLEGS
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --logits-rows 16384 \
  --params 10000000 --bucket-mb 8 $NOLEGS > gpurun_out/r05a_rehearse_n2.json 2> gpurun_out/r05a_rehearse_n2.err
rc=$?; tail -c 600 gpurun_out/r05a_rehearse_n2.json; exit $rc
