"""BASELINE config 1 -- GPT-2-small GRPO on 16 gsm8k-style prompts, group 4, world_size 1 gloo --
through GRPOTrainer on the GPU.

GPT-2 is not served by the paged engine (PagedDecoder covers Qwen2/Llama), so the rollout is
HFGenerateEngine: the reference's HF fallback (HFModelWrapper.generate,
model_wrapper.py:185-218) with the HIP sampler choosing every token. The learner is HF GPT-2
(random init, the real 124 M architecture, V = 50,257: odd, so its logits rows are not 16-B
aligned) with the lm_head-fused HIP logprob kernels, the HIP pack, GRPO and fused PPO/KL loss,
AdamW, and the weight sync back into the engine. A world_size-1 gloo group is the DP group,
as in config 1.

Rewards: skyrl-gym's strict gsm8k scorer (skyrl_amd/envs/gsm8k.py, utils.py:17-63) on the
responses through a fixture detokenizer, against answers the test plants per prompt.
Checked: every micro-batch's fused-pass logprobs and entropies equal oracle/cpu_ref's on the
micro-batch's own lm_head logits within 1e-4, and its loss equals oracle/cpu_ref's loss assembly
(PPO clip + k3 KL to ref, token mean) on those oracle log-probs within 1e-4; the engine's rollout
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


def _detok(ids):
    """Fixture detokenizer (GPT-2's vocabulary files are not in the image): every 16th token id is
    the gsm8k answer marker, the others a digit, so the strict scorer sees `#### <digit>` often."""
    return "".join("#### " if t % 16 == 0 else f"{t % 10} " for t in ids)


def _reward_fn(log):
    from skyrl_amd.envs.gsm8k import compute_score

    def reward(prompt, response, extra):  # skyrl-gym gsm8k strict scorer (utils.py:17-63) on the planted answer
        r = float(compute_score(_detok(response), extra["ground_truth"]))
        log.append(r)
        return r
    return reward


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

    # every micro-batch's fused pass against the oracle: its logprobs / entropies against
    # cpu_ref.logprobs_from_logits / entropy_from_logits on the micro-batch's own lm_head logits
    # (1e-4), and its loss against the oracle's loss assembly (workers/worker.py:801-876: PPO clip +
    # k3 KL to ref, token mean; cpu_ref.policy_loss_assembly) on those ORACLE log-probs (1e-4)
    checked, lp_checked = [], []
    orig_micro, orig_fold = ops.PolicyTrainStep.micro, ops.PolicyTrainStep.fold

    def micro(self, k, logits, labels, token_pos=None):
        if not hasattr(self, "_cap"):
            self._cap = {}
        self._cap[k] = (logits.detach().cpu(), labels.detach().cpu(), token_pos.detach().cpu().long())
        return orig_micro(self, k, logits, labels, token_pos)

    def fold(self):
        loss, met = orig_fold(self)
        for k, (z, lab, pos) in self._cap.items():
            i, j = self.rows(k)
            R = self.R
            lp_o = cpu_ref.logprobs_from_logits(z, lab)
            ent_o = cpu_ref.entropy_from_logits(z)
            lp_k = self.logp[i:j].cpu().reshape(-1)[pos]
            ent_k = self.entropy[i:j].cpu().reshape(-1)[pos]
            lp_checked.append(torch.allclose(lp_k, lp_o, atol=1e-4, rtol=1e-4)
                              and torch.allclose(ent_k, ent_o, atol=1e-4, rtol=1e-4))
            lp_full = torch.zeros((j - i) * R)
            ent_full = torch.zeros((j - i) * R)
            lp_full[pos], ent_full[pos] = lp_o, ent_o
            exp, _ = cpu_ref.policy_loss_assembly(lp_full.view(j - i, R), self.old[i:j].cpu(), self.adv[i:j].cpu(),
                                                  self.mask[i:j].cpu(), self.ref[i:j].cpu(), ent_full.view(j - i, R))
            checked.append(abs(float(met[k][0]) - float(exp)) <= 1e-5 + 1e-4 * abs(float(exp)))
        return loss, met

    monkeypatch.setattr(ops.PolicyTrainStep, "micro", micro)
    monkeypatch.setattr(ops.PolicyTrainStep, "fold", fold)

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
    # with the built-in GRPO estimator the advantages come from the step plan's launch
    # (skyrl_policy_train_plan_grpo) and are complete when the metrics are taken after training
    orig_metrics = trainer_utils.advantage_metrics

    def checked_metrics(data, step_wise=False):
        exp = cpu_ref.grpo_advantage(data["rewards"].float().cpu(), data["response_mask"].cpu(),
                                     data.metadata["uids"])
        adv_checked.append(torch.allclose(data["advantages"].float().cpu(), exp, atol=1e-5, rtol=1e-5))
        return orig_metrics(data, step_wise)

    monkeypatch.setattr(trainer_utils, "advantage_metrics", checked_metrics)

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
    rewards = []
    trainer = GRPOTrainer(tcfg, policy, client, _reward_fn(rewards), pad_token_id=0, ref=ref, dp_group=gloo_world1)
    assert trainer.grad_sync is None  # world_size 1: nothing to reduce
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(1, 50256, (int(torch.randint(8, 33, (1,), generator=g)),), generator=g).tolist()
               for _ in range(16)]
    w0 = policy.transformer.h[0].attn.c_attn.weight.detach().clone()
    hist = []
    extras = [{"ground_truth": str(i % 10)} for i in range(16)]  # planted gsm8k answers
    for step in range(3):
        m = trainer.step(prompts, extras)
        hist.append(m)
        assert all(torch.isfinite(torch.tensor(float(v))) for v in m.values()), m
        assert m["logprobs_diff_mean"] < 0.03, (step, m["logprobs_diff_mean"])
    assert len(checked) == 12 and all(checked), checked  # 3 steps x 4 micro-batches, each within 1e-4 of the oracle
    assert len(lp_checked) == 12 and all(lp_checked), lp_checked
    assert 0 < sum(rewards) < len(rewards), rewards  # the strict scorer's rewards are not degenerate
    assert len(adv_checked) == 3 and all(adv_checked), adv_checked
    assert not torch.equal(policy.transformer.h[0].attn.c_attn.weight.detach(), w0)
    assert hist[-1]["policy_kl"] > 0
    # the engine holds the learner's weights (bf16) after the sync
    assert torch.equal(rollout.transformer.h[0].attn.c_attn.weight,
                       policy.transformer.h[0].attn.c_attn.weight.detach().to(torch.bfloat16))
