#!/bin/bash
# r05m: the empty-last-micro-batch rehearsal (full logs), split-sampler occupancy probe, bench N=1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
REHEARSE_EMPTY_LAST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 scripts/rehearse_trainer_optim.py > gpurun_out/r05m_empty.log 2>&1
echo "empty-last rc=$?"; grep -n "Error\|error\|ok\"" gpurun_out/r05m_empty.log | head -20
timeout -k 10 200 python -u scripts/probe/split_wpe.py run > gpurun_out/r05m_split_wpe.json 2>&1
rc=$?; tail -1 gpurun_out/r05m_split_wpe.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r05m_bench.json 2> gpurun_out/r05m_bench.err
rc=$?; tail -c 300 gpurun_out/r05m_bench.json; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05m_bench.err; exit $rc; }
