set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_sampler_topp_fast.py tests/test_gpu_policy_train_step.py > gpurun_out/r04a_tests1.log 2>&1; rc=$?
tail -15 gpurun_out/r04a_tests1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 $T tests/test_gpu_optim.py tests/test_gpu_policy_train_split.py tests/test_gpu_sampler_topk_fast.py \
  tests/test_gpu_trainer_e2e.py tests/test_gpu_trainer.py tests/test_gpu_gpt2_grpo.py tests/test_gpu_ppo_critic_e2e.py \
  tests/test_gpu_multirank.py tests/test_gpu_e2e.py > gpurun_out/r04a_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r04a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04a_bench.err; exit $rc; }
python -c "import json;d=json.loads(open('gpurun_out/r04a_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['advantage_loss_product'],d['sampler_filtered'],d.get('end_to_end',{}).get('value'))"
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 --logits-rows 16384 --params 10000000 \
  --bucket-mb 8 --no-e2e --no-cpu-baseline --no-adv-loss-leg --no-attention-leg --no-lmhead-leg --no-vocab-legs \
  --no-filtered-leg > gpurun_out/r04a_spawn_n2.json 2> gpurun_out/r04a_spawn_n2.err; rc=$?
echo "spawn n2 rc=$rc"; tail -c 600 gpurun_out/r04a_spawn_n2.json; exit $rc
