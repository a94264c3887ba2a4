"""A real-model GRPO loop through every layer of the build (SURVEY §8(f)2 + (f)3, single node):
AMDInferenceEngine rollout (paged decode loop + HIP sampler) -> pack kernel -> lm_head-fused
HIP logprobs (old, ref) on a HF Qwen2 learner -> GRPO -> fused PPO/KL loss -> AdamW ->
weight sync into the engine (update_named_weights), repeated.

Properties checked (parity unpinned against the reference: its loop needs Ray + vLLM):
  * the engine's rollout log-probs equal the learner's recomputed old log-probs of the same
    tokens (mean |diff| < 0.02): engine numerics and the weight sync both hold, every step;
  * the task is learnable and the loop learns it: mean reward rises well above its start.
"""

import pytest
import torch

from skyrl_amd.config import AlgorithmConfig
from skyrl_amd.inference_engines.client import InferenceEngineClient
from skyrl_amd.inference_engines.engine import AMDInferenceEngine
from skyrl_amd.inference_engines.model import PagedDecoder
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TARGET = 64  # reward: fraction of response tokens with id < TARGET (1/8 of the vocabulary)


def reward(prompt, response, extra):
    return sum(t < TARGET for t in response) / max(1, len(response))


def test_grpo_loop_with_engine_learns_and_stays_in_sync():
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    ref = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    ref.load_state_dict(policy.state_dict())
    engine_model = PagedDecoder(cfg, DEV, seed=None, max_model_len=256)
    engine_model.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    client = InferenceEngineClient([AMDInferenceEngine(engine_model, num_blocks=512, max_num_seqs=64, seed=3)])
    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=16, micro_train_batch_size_per_gpu=16,
                         micro_forward_batch_size_per_gpu=32, lr=5e-3, weight_decay=0.0,
                         sampling_params={"max_tokens": 12, "min_tokens": 1, "ignore_eos": True},
                         algorithm=AlgorithmConfig(use_kl_loss=True))
    trainer = GRPOTrainer(tcfg, policy, client, reward, pad_token_id=0, ref=ref)
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(2, 512, (int(torch.randint(3, 9, (1,), generator=g)),), generator=g).tolist()
               for _ in range(16)]
    hist = []
    for step in range(16):
        m = trainer.step(prompts)
        hist.append(m)
        assert m["logprobs_diff_mean"] < 0.02, (step, m["logprobs_diff_mean"])
        assert all(torch.isfinite(torch.tensor(v)) for v in m.values())
    first = hist[0]["avg_final_rewards"]
    last = sum(h["avg_final_rewards"] for h in hist[-3:]) / 3
    assert first < 0.3 and last > first + 0.2, [h["avg_final_rewards"] for h in hist]
    assert hist[-1]["policy_kl"] > 0


def test_data_parallel_trainer_two_ranks_one_gpu():
    """scripts/rehearse_trainer_dp.py under torch.distributed.run (2 ranks, gloo, one GPU):
    after every step both ranks hold identical policy weights although their rollouts differ."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "scripts", "rehearse_trainer_dp.py")]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["world"] == 2 and all(s["weights_identical_across_ranks"] for s in res["steps"])
    assert all(s["logprobs_diff_mean"] < 0.02 for s in res["steps"])


def _run_optim_rehearsal(nproc, rccl_solo=False, extra_env=None):
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = os.path.join(root, "scripts", "rehearse_trainer_optim.py")
    env = dict(os.environ)
    env.update(extra_env or {})
    if rccl_solo:
        env.update(SKYRL_FORCE_COLLECTIVES="1", REHEARSE_BACKEND="nccl")
    if nproc == 1 and not rccl_solo:
        cmd = [sys.executable, script]
    else:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(port), script]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stderr[-3000:]
    res = json.loads(lines[-1])
    assert p.returncode == 0 and res["ok"], json.dumps(res)[:3000] + p.stderr[-2000:]
    return res


@pytest.mark.parametrize("nproc", [1, 2])
def test_hip_optimizer_trainer_matches_torch_adamw(nproc):
    """GRPOTrainer(optimizer="hip") -- flat fp32 master, reduce-scatter fired from the backward
    hooks, one HIP clip + AdamW pass that writes the engine's bf16 copy -- against
    GRPOTrainer(optimizer="torch") (torch AdamW + clip_grad_norm_ on the rank-mean gradient,
    fsdp_strategy.py:155-191, worker.py:902-924) on the same fixed rollouts: parameters within
    1e-6, grad norms within rel 1e-5, ranks identical, and the engine's weights after the sync
    equal the learner's bf16 cast bit for bit. 1 rank, and 2 ranks on one GPU over gloo."""
    res = _run_optim_rehearsal(nproc)
    assert res["world"] == nproc and len(res["steps"]) == 3


def test_hip_optimizer_trainer_over_rccl_one_rank():
    """The same check with the trainer's exchanges forced through RCCL on a one-rank group
    (torchrun, nccl backend, SKYRL_FORCE_COLLECTIVES=1): the bucket reduce-scatters fired from
    the backward hooks, the grad-norm all-reduce and the fp32 / bf16 all-gathers all run as
    RCCL collectives on the comm stream, as at N > 1 (RCCL refuses two ranks on one GPU)."""
    res = _run_optim_rehearsal(1, rccl_solo=True)
    assert res["world"] == 1 and res["backend"] == "nccl" and res["collective_path"]
    assert res["reduce_scatters_from_backward"] > 0 and len(res["steps"]) == 3


def test_trainer_passes_wait_for_the_in_flight_weight_gather():
    """the optimizer's fp32 re-assembly of the master is left in flight on the
    comm stream, and the trainer's passes read the weights through base_model and the lm_head
    weight, not the module's forward. With the comm stream held back ~40 ms before each gather
    and 2 mini-batches (2 optimizer steps) per train_on, every weight read of the trainer's passes
    must see the updated master (checked on the reading stream), over one-rank RCCL."""
    res = _run_optim_rehearsal(1, rccl_solo=True, extra_env={"REHEARSE_DELAY_GATHER": "1"})
    assert res["weight_reads"]["checked"] >= 12 and res["weight_reads"]["stale"] == 0, res["weight_reads"]


def test_fused_policy_pass_matches_chunked_lmhead_path():
    """GRPOTrainer's policy micro-batch through the fused pass (lm_head GEMM -> ONE pass for
    logprob + entropy + PPO/KL/entropy loss + dL/dz -> the lm_head backward GEMMs) against the
    chunked lm_head logprob + HIP loss path, on the same fixed rollouts: the loss metrics agree
    and so does the gradient the optimizer receives (bf16 dlogits either way)."""
    import copy

    from transformers import AutoModelForCausalLM, Qwen2Config

    from skyrl_amd import comm

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)
    base = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    ref = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    ref.load_state_dict(base.state_dict())
    g = torch.Generator().manual_seed(5)
    gen = {"prompt_token_ids": [], "response_ids": [], "rewards": [], "rollout_logprobs": [], "loss_masks": [],
           "stop_reasons": []}
    for i in range(4):
        p = torch.randint(2, 512, (int(torch.randint(3, 9, (1,), generator=g)),), generator=g).tolist()
        for _ in range(4):
            r = torch.randint(2, 512, (int(torch.randint(1, 13, (1,), generator=g)),), generator=g).tolist()
            gen["prompt_token_ids"].append(p)
            gen["response_ids"].append(r)
            gen["rewards"].append(float(torch.rand(1, generator=g) < 0.5))
            gen["rollout_logprobs"].append((-2.0 + 0.1 * torch.randn(len(r), generator=g)).tolist())
            gen["loss_masks"].append([1] * len(r))
            gen["stop_reasons"].append("length")
    out = {}
    for fused in (True, False):
        policy = copy.deepcopy(base)
        tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=4, micro_train_batch_size_per_gpu=8,
                             micro_forward_batch_size_per_gpu=16, lr=1e-3, temperature=0.8, fused_policy_pass=fused,
                             algorithm=AlgorithmConfig(use_kl_loss=True, use_entropy_loss=True, entropy_loss_coef=0.01,
                                                       policy_loss_type="dual_clip"))
        tr = GRPOTrainer(tcfg, policy, None, None, pad_token_id=0, ref=ref)
        grads = []
        step0 = tr.optim.step

        def capture(n_micro=1, lr=None, tr=tr, grads=grads, step0=step0):
            grads.append(tr.optim.reducer.grad[: tr.optim.reducer.layout.numel].clone())
            return step0(n_micro, lr)

        tr.optim.step = capture
        m = tr.train_on(copy.deepcopy(gen))
        out[fused] = (m, grads[0])
    (mf, gf), (mc, gc) = out[True], out[False]
    for k in ("final_loss", "policy_loss", "policy_entropy", "policy_kl", "ppo_clip_ratio"):
        assert abs(mf[k] - mc[k]) <= 1e-4 * max(1.0, abs(mc[k])), (k, mf[k], mc[k])
    rel = float((gf - gc).norm() / gc.norm())
    assert rel < 2e-2, rel


def test_empty_last_micro_batch_on_one_rank():
    """scripts/rehearse_empty_micro.py under torch.distributed.run
    (2 ranks, gloo, one GPU) runs GRPOTrainer._fused_policy_pass directly on a mini-batch whose
    last micro-batch has no response token on rank 1 only (the generator check rejects such
    output, so it is made empty after packing). Its loss is 0, both ranks fire the same
    bucket reduce-scatter sequence from the backward hooks, and the weights stay bit-identical."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "scripts", "rehearse_empty_micro.py")]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stderr[-3000:]
    res = json.loads(lines[-1])
    assert p.returncode == 0 and res["ok"], json.dumps(res) + p.stderr[-2000:]
    assert res["launch_sequences_equal"] and res["empty_micro_loss"] == 0.0
    assert res["weights_identical_across_ranks"]
