"""PolicyMicroStep / CriticMicroStep: the reference's _forward_backward_micro status dict and
logits gradient (workers/worker.py:731-900, 1062-1114), fused kernel vs the registry
composition vs the oracle (torch-CPU autograd of the restated loss assembly).
Tolerances: loss/metrics 1e-4; logits gradient compared in bf16 (the kernel writes bf16).
"""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import worker as W
from skyrl_amd.config import AlgorithmConfig
from skyrl_amd.trainer_utils import Experience

pytestmark = pytest.mark.gpu


def _exp(dev, n=3, P=5, R=37, V=1000, seed=0):
    g = torch.Generator().manual_seed(seed)
    S = P + R
    seq = torch.randint(0, V, (n, S), generator=g)
    lp = -2 + 0.1 * torch.randn(n, R, generator=g)
    mask = (torch.arange(R)[None] < torch.tensor([R, R // 2, 1])[:, None]).float()
    e = Experience(sequences=seq.to(dev), action_log_probs=(lp + 0.05 * torch.randn(n, R, generator=g)).to(dev),
                   base_action_log_probs=(lp + 0.05 * torch.randn(n, R, generator=g)).to(dev), values=None,
                   returns=None, advantages=torch.randn(n, R, generator=g).to(dev), attention_mask=None,
                   loss_mask=mask.to(dev), action_mask=mask.to(dev), rollout_logprobs=None, num_actions=R, info={})
    logits = (3 * torch.randn(n, S, V, generator=g)).to(torch.bfloat16)
    return e, logits


@pytest.mark.parametrize("loss_type", ["regular", "dual_clip"])
def test_policy_micro_step_fused_vs_composed_vs_oracle(dev, loss_type):
    cfg = AlgorithmConfig()
    cfg.policy_loss_type = loss_type
    cfg.use_kl_loss = True
    e, logits_cpu = _exp(dev)
    outs = []
    for fused in (True, False):
        step = W.PolicyMicroStep(cfg)
        if not fused:
            step._fused_ok = lambda name: False
        logits = logits_cpu.to(dev).requires_grad_(True)
        st = step(logits, e)
        outs.append((st, logits.grad.float().cpu()))
    (sf, gf), (sc, gc) = outs
    assert set(sf) == set(sc) == {"final_loss", "policy_loss", "policy_entropy", "response_length", "policy_lr",
                                  "loss_metrics/clip_ratio", "policy_kl"}
    for k in sf:
        assert sf[k] == pytest.approx(sc[k], abs=1e-4), k
    assert torch.allclose(gf, gc, atol=2e-6, rtol=1e-2)
    # oracle: torch-CPU fp32 autograd of the reference formulas
    R = e.num_actions
    x = logits_cpu[:, -R - 1:-1].float().requires_grad_(True)
    lab = e.sequences[:, -R:].cpu()
    lp = cpu_ref.logprobs_from_logits(x, lab)
    ent = cpu_ref.entropy_from_logits(x.detach())
    loss, m = cpu_ref.policy_loss_assembly(lp, e.action_log_probs.cpu(), e.advantages.cpu(), e.loss_mask.cpu(),
                                           e.base_action_log_probs.cpu(), ent, dual_clip=loss_type == "dual_clip")
    loss.backward()
    assert sf["final_loss"] == pytest.approx(float(loss.detach()), abs=1e-4)
    ref_grad = torch.zeros_like(gf)
    ref_grad[:, -R - 1:-1] = x.grad.to(torch.bfloat16).float()
    assert torch.allclose(gf, ref_grad, atol=2e-6, rtol=2e-2)


def test_critic_micro_step(dev):
    cfg = AlgorithmConfig()
    g = torch.Generator().manual_seed(1)
    n, R = 4, 33
    vals = torch.randn(n, R, generator=g).to(dev).requires_grad_(True)
    mask = (torch.rand(n, R, generator=g) > 0.3).float()
    e = Experience(sequences=None, action_log_probs=None, base_action_log_probs=None,
                   values=torch.randn(n, R, generator=g).to(dev), returns=torch.randn(n, R, generator=g).to(dev),
                   advantages=None, attention_mask=None, loss_mask=mask.to(dev), action_mask=None,
                   rollout_logprobs=None, num_actions=R, info={})
    st = W.CriticMicroStep(cfg)(vals, e)
    v = vals.detach().cpu().requires_grad_(True)
    ref_loss, ref_clip = cpu_ref.critic_loss(v, e.values.cpu(), e.returns.cpu(), mask, cfg.value_clip)
    ref_loss.backward()
    assert st["critic_loss"] == pytest.approx(float(ref_loss), abs=1e-5)
    assert st["values_clipfrac"] == pytest.approx(float(ref_clip), abs=1e-5)
    assert torch.allclose(vals.grad.cpu(), v.grad, atol=1e-6)
