set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u scripts/rehearse_trainer_optim.py > gpurun_out/r03_optim_w1.log 2>&1; echo "w1 rc=$?"; tail -3 gpurun_out/r03_optim_w1.log | cut -c1-1500
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/rehearse_trainer_optim.py > gpurun_out/r03_optim_w2.log 2>&1; echo "w2 rc=$?"; tail -3 gpurun_out/r03_optim_w2.log | cut -c1-1500
