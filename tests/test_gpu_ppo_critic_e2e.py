"""PPO with a critic through the whole build (config 4's algorithm shape, tiny model): engine
rollout -> values from a CriticModel (HF base + value_head) -> GAE (lambda 0.95) + whitening on
the HIP kernel -> HIP clipped value loss update -> HIP PPO policy loss update -> weight sync.

Every step's GAE advantages / returns and every critic micro-batch's value loss are checked
against the oracle on the step's own batch. Properties: the critic regresses onto the returns
(its loss falls), advantages are whitened (masked mean 0,
variance 1 — checked through the GAE registry entry on the step's own batch), rollout and
learner logprobs agree, and nothing goes non-finite.
"""

import pytest
import torch

from skyrl_amd.config import AlgorithmConfig
from skyrl_amd.inference_engines.engine import AMDInferenceEngine
from skyrl_amd.inference_engines.model import PagedDecoder
from skyrl_amd.trainer import CriticModel, GRPOTrainer, TrainerConfig

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_ppo_with_critic_and_gae(monkeypatch):
    from transformers import AutoModelForCausalLM, Qwen2Config

    from oracle import cpu_ref
    from skyrl_amd import ppo_utils, trainer_utils

    # each step's GAE (+ whitening) and each critic micro-batch's clipped value loss against the
    # oracle on the same inputs (utils/ppo_utils.py:1101-1129, 148-172, 175-193)
    checks = {"gae": [], "critic": []}
    orig_adv, orig_vl = trainer_utils.compute_advantages_and_returns, ppo_utils.ppo_critic_loss

    def checked_adv(data, alg_cfg):
        out = orig_adv(data, alg_cfg)
        adv, ret = cpu_ref.gae(out["rewards"].float().cpu(), out["values"].float().cpu(),
                               out["response_mask"].float().cpu(), alg_cfg.gamma, alg_cfg.lambd)
        checks["gae"].append(torch.allclose(out["advantages"].cpu(), adv, atol=1e-4, rtol=1e-4)
                             and torch.allclose(out["returns"].cpu(), ret, atol=1e-5, rtol=1e-5))
        return out

    def checked_vl(values, old_values, returns, config, loss_mask=None):
        loss, clipfrac = orig_vl(values, old_values, returns, config, loss_mask=loss_mask)
        exp, _ = cpu_ref.critic_loss(values.detach().float().cpu(), old_values.float().cpu(), returns.float().cpu(),
                                     loss_mask.float().cpu(), config.value_clip)
        checks["critic"].append(abs(float(loss.detach()) - float(exp)) <= 1e-6 + 1e-5 * abs(float(exp)))
        return loss, clipfrac

    monkeypatch.setattr(trainer_utils, "compute_advantages_and_returns", checked_adv)
    monkeypatch.setattr(ppo_utils, "ppo_critic_loss", checked_vl)

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    critic = CriticModel(cfg).to(DEV)
    em = PagedDecoder(cfg, DEV, seed=None, max_model_len=256)
    em.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(em, num_blocks=256, max_num_seqs=64, seed=5)
    alg = AlgorithmConfig(advantage_estimator="gae", lambd=0.95, gamma=1.0, use_kl_loss=False, value_clip=0.2)
    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=8, micro_train_batch_size_per_gpu=16,
                         micro_forward_batch_size_per_gpu=32, lr=1e-3, critic_lr=3e-3, weight_decay=0.0,
                         sampling_params={"max_tokens": 10, "min_tokens": 1, "ignore_eos": True}, algorithm=alg)
    trainer = GRPOTrainer(tcfg, policy, engine, lambda p, r, e: sum(t < 64 for t in r) / len(r), pad_token_id=0,
                          critic=critic)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(2, 512, (int(torch.randint(3, 9, (1,), generator=g)),), generator=g).tolist()
               for _ in range(8)]
    hist = [trainer.step(prompts) for _ in range(8)]
    for h in hist:
        assert h["logprobs_diff_mean"] < 0.02
        assert all(torch.isfinite(torch.tensor(v)) for v in h.values())
        assert abs(h["avg_advantages"]) < 0.2  # whitened over the masked tokens
    # the critic tracks the returns: the policy's learning moves them (the loss spikes once the
    # reward starts to rise), and by the end of the run the critic has caught up to a tenth of the
    # peak (the first step's loss is not a fixed reference: it depends on the initial rewards)
    cl = [h["critic_loss"] for h in hist]
    assert cl[-1] < 0.1 * max(cl) and min(cl[-3:]) < cl[0], cl
    assert "values_clipfrac" in hist[0] and "critic_grad_norm" in hist[0]
    assert len(checks["gae"]) == 8 and all(checks["gae"]), checks["gae"]
    assert checks["critic"] and all(checks["critic"]), checks["critic"]
