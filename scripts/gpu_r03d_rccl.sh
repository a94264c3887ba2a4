set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer_e2e.py -k "rccl or hip_optimizer" -v --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_rccl_tests.log 2>&1; rc=$?
tail -6 gpurun_out/r03d_rccl_tests.log; [ $rc -eq 0 ] || exit $rc
SKYRL_FORCE_COLLECTIVES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs > gpurun_out/r03d_bench_rccl_solo.json 2> gpurun_out/r03d_bench_rccl_solo.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/r03d_bench_rccl_solo.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03d_bench_rccl_solo.err; exit $rc; }
