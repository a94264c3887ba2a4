"""BASELINE config 1 -- GPT-2-small GRPO on 16 gsm8k-style prompts, group 4, world_size 1 gloo --
through GRPOTrainer on the GPU.

GPT-2 is not served by the paged engine (PagedDecoder covers Qwen2/Llama), so the rollout is
HFGenerateEngine: the reference's HF fallback (HFModelWrapper.generate,
model_wrapper.py:185-218) with the HIP sampler choosing every token. The learner is HF GPT-2
(random init, the real 124 M architecture, V = 50,257: odd, so its logits rows are not 16-B
aligned) with the lm_head-fused HIP logprob kernels, the HIP pack, GRPO and fused PPO/KL loss,
AdamW, and the weight sync back into the engine. A world_size-1 gloo group is the DP group,
as in config 1.

Checked: every micro-batch's loss from the fused pass equals oracle/cpu_ref's loss assembly
(PPO clip + k3 KL to ref, token mean) on the same log-probs within 1e-4; the engine's rollout
logprobs equal the learner's recomputed old logprobs of the same tokens (the sampler, the
weight sync and the fused logprob agree), every metric is finite, the policy moves away from
the reference (KL > 0), with sample packing off and on.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist

from skyrl_amd.config import AlgorithmConfig
from skyrl_amd.inference_engines.client import InferenceEngineClient
from skyrl_amd.inference_engines.hf_engine import HFGenerateEngine
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _reward(prompt, response, extra):  # gsm8k-style strict-answer stand-in: answer token parity
    return float(len(response) > 0 and response[-1] % 2 == 0)


@pytest.fixture
def gloo_world1():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.mark.parametrize("packing", [False, True])
def test_gpt2_small_grpo_steps(gloo_world1, packing, monkeypatch):
    from transformers import AutoModelForCausalLM, GPT2Config

    from oracle import cpu_ref
    from skyrl_amd import ops

    # every micro-batch's fused pass against the oracle's loss assembly on the same log-probs
    # (workers/worker.py:801-876: PPO clip + k3 KL to ref, token-mean; cpu_ref.policy_loss_assembly)
    checked = []
    orig = ops.policy_train_ragged

    def checked_pass(logits, labels, pos, old, adv, mask, params, **kw):
        loss, met, lp, ent = orig(logits, labels, pos, old, adv, mask, params, **kw)
        exp, _ = cpu_ref.policy_loss_assembly(lp.detach().float().cpu(), old.float().cpu(), adv.float().cpu(),
                                              mask.float().cpu(), kw["ref_log_probs"].float().cpu(),
                                              ent.detach().float().cpu())
        got = float(met[0])
        checked.append(abs(got - float(exp)) <= 1e-5 + 1e-4 * abs(float(exp)))
        return loss, met, lp, ent

    monkeypatch.setattr(ops, "policy_train_ragged", checked_pass)

    # ... and the GRPO advantages against the oracle (utils/ppo_utils.py:1132-1182), every step
    from skyrl_amd import trainer_utils

    adv_checked = []
    orig_adv = trainer_utils.compute_advantages_and_returns

    def checked_adv(data, alg):
        out = orig_adv(data, alg)
        exp = cpu_ref.grpo_advantage(out["rewards"].float().cpu(), out["response_mask"].cpu(),
                                     out.metadata["uids"])
        adv_checked.append(torch.allclose(out["advantages"].float().cpu(), exp, atol=1e-5, rtol=1e-5))
        return out

    monkeypatch.setattr(trainer_utils, "compute_advantages_and_returns", checked_adv)

    cfg = GPT2Config()  # GPT-2-small: 12 layers, 768 wide, 12 heads, V = 50,257
    assert cfg.vocab_size == 50257 and cfg.n_layer == 12
    torch.manual_seed(0)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    ref = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    ref.load_state_dict(policy.state_dict())
    rollout = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV)
    rollout.load_state_dict(policy.state_dict())
    client = InferenceEngineClient([HFGenerateEngine(rollout, pad_token_id=0, seed=5)])
    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=16, micro_train_batch_size_per_gpu=16,
                         micro_forward_batch_size_per_gpu=32, lr=1e-5, weight_decay=0.01,
                         use_sample_packing=packing,
                         sampling_params={"max_tokens": 24, "min_tokens": 1, "temperature": 1.0},
                         algorithm=AlgorithmConfig(use_kl_loss=True))
    trainer = GRPOTrainer(tcfg, policy, client, _reward, pad_token_id=0, ref=ref, dp_group=gloo_world1)
    assert trainer.grad_sync is None  # world_size 1: nothing to reduce
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(1, 50256, (int(torch.randint(8, 33, (1,), generator=g)),), generator=g).tolist()
               for _ in range(16)]
    w0 = policy.transformer.h[0].attn.c_attn.weight.detach().clone()
    hist = []
    for step in range(3):
        m = trainer.step(prompts)
        hist.append(m)
        assert all(torch.isfinite(torch.tensor(float(v))) for v in m.values()), m
        assert m["logprobs_diff_mean"] < 0.03, (step, m["logprobs_diff_mean"])
    assert checked and all(checked), checked  # 3 steps x 4 micro-batches, each within 1e-4 of the oracle
    assert len(adv_checked) == 3 and all(adv_checked), adv_checked
    assert not torch.equal(policy.transformer.h[0].attn.c_attn.weight.detach(), w0)
    assert hist[-1]["policy_kl"] > 0
    # the engine holds the learner's weights (bf16) after the sync
    assert torch.equal(rollout.transformer.h[0].attn.c_attn.weight,
                       policy.transformer.h[0].attn.c_attn.weight.detach().to(torch.bfloat16))
