"""Secondary registry entries (skyrl_amd/secondary.py) against the reference.

tests/golden/secondary.npz was written by tools/gen_golden.py from the imported reference
(ppo_utils.py:589-981 losses, :1013-1098 estimators): the reference's own KAT inputs
(tests/cpu/algorithms/test_losses.py:85-137 CISPO, :291-402 GSPO, :442-502 clip_cov,
:504-561 kl_cov, :564-618 SAPO; tests/cpu/utils/test_ppo_utils.py:65-129 REINFORCE++ / RLOO)
plus seeded ragged batches under every reduction and, for the losses that apply it, off-policy
correction. Each case is replayed through the registry by name: loss, metrics and dL/dlog_probs
(autograd) within 1e-6, advantages/returns within 1e-6. clip_cov's randperm is reproduced by
seeding the global generator exactly as the generator did. The hand-computed constants of the
reference tests are asserted as well.

CPU tensors here; the same cases on device tensors under `-m gpu` (the restatements run as
torch ops on whatever device their inputs live on).
"""

import json

import numpy as np
import pytest
import torch

from skyrl_amd import ppo_utils
from skyrl_amd.config import AlgorithmConfig

from conftest import load_golden

G = load_golden("secondary")
LOSS_TAGS = [str(t) for t in G["loss_tags"]]
EST_TAGS = [str(t) for t in G["est_tags"]]


def _close(a, b, tol=1e-6):
    torch.testing.assert_close(torch.as_tensor(a).detach().double().cpu(), torch.as_tensor(b).detach().double().cpu(),
                               atol=tol, rtol=tol)


def _run_loss(tag, device):
    cfgd = json.loads(str(G[f"cfg_{tag}"]))
    name = cfgd["policy_loss_type"]
    cfg = AlgorithmConfig.from_dict(cfgd)
    to = lambda k: G[k].to(device) if k in G else None  # noqa: E731
    x = G[f"lp_{tag}"].clone().to(device).requires_grad_(True)
    torch.manual_seed(int(G[f"seed_{tag}"]))
    fn = ppo_utils.PolicyLossRegistry.get(name)
    loss, met = fn(x, to(f"old_{tag}"), to(f"adv_{tag}"), cfg, loss_mask=to(f"mask_{tag}"),
                   rollout_logprobs=to(f"rollout_{tag}"))
    if loss.requires_grad:
        loss.backward()
    grad = x.grad if x.grad is not None else torch.zeros_like(x)
    return loss, met, grad


def _check_loss(tag, device):
    loss, met, grad = _run_loss(tag, device)
    assert loss.device.type == torch.device(device).type
    _close(loss, G[f"loss_{tag}"])
    _close(grad, G[f"grad_{tag}"])
    keys = [str(k) for k in G[f"mkeys_{tag}"]]
    assert sorted(met) == keys, (tag, sorted(met), keys)
    for k, v in zip(keys, G[f"mvals_{tag}"].tolist()):
        assert met[k] == pytest.approx(v, abs=1e-6, rel=1e-6), (tag, k)


def _check_est(tag, device):
    name = "rloo" if "rloo" in tag else "reinforce++"
    fn = ppo_utils.AdvantageEstimatorRegistry.get(name)
    idx = G.get(f"index_{tag}")
    idx = None if idx is None else np.asarray(idx)
    a, r = fn(token_level_rewards=G[f"rew_{tag}"].clone().to(device), response_mask=G[f"rmask_{tag}"].to(device),
              index=idx, gamma=float(G[f"gamma_{tag}"]))
    _close(a, G[f"eadv_{tag}"])
    _close(r, G[f"eret_{tag}"])


@pytest.mark.parametrize("tag", LOSS_TAGS)
def test_secondary_loss_matches_reference(tag):
    _check_loss(tag, "cpu")


@pytest.mark.parametrize("tag", EST_TAGS)
def test_secondary_estimator_matches_reference(tag):
    _check_est(tag, "cpu")


def test_reference_hand_computed_constants():
    """The literal expectations of the reference's tests."""
    loss, _, _ = _run_loss("kat_cispo", "cpu")
    assert loss.item() == pytest.approx(-0.99768266666, abs=1e-4)  # test_losses.py:137
    loss, met, _ = _run_loss("kat_sapo", "cpu")
    assert met["clip_ratio"] == 0.0  # test_losses.py:618
    _, met, _ = _run_loss("kat_kl_cov", "cpu")
    assert met["clip_ratio"] == 0.0  # test_losses.py:542
    _, met, _ = _run_loss("kat_clip_cov", "cpu")
    assert 0.0 <= met["clip_ratio"] <= 1.0  # test_losses.py:483
    fn = ppo_utils.AdvantageEstimatorRegistry.get("reinforce++")
    _, ret = fn(token_level_rewards=torch.tensor([[1.0, 2.0, 3.0]]), response_mask=torch.tensor([[1.0, 1.0, 0.0]]),
                gamma=1.0)
    _close(ret, torch.tensor([[3.0, 2.0, 3.0]]), 1e-5)  # test_ppo_utils.py:76
    _, ret = fn(token_level_rewards=torch.tensor([[1.0, 2.0, 3.0]]), response_mask=torch.ones(1, 3), gamma=0.5)
    _close(ret, torch.tensor([[2.75, 3.5, 3.0]]), 1e-5)  # test_ppo_utils.py:96
    fn = ppo_utils.AdvantageEstimatorRegistry.get("rloo")
    rew = torch.tensor([[0.0, 0.0, 6.0], [0.0, 0.0, 3.0], [0.0, 0.0, 9.0], [0.0, 0.0, 12.0], [0.0, 0.0, 1.0]])
    adv, ret = fn(token_level_rewards=rew, response_mask=torch.ones_like(rew), index=np.array([0, 0, 1, 1, 2]))
    _close(adv, torch.tensor([3.0, -3.0, -3.0, 3.0, 0.0]).unsqueeze(-1) * torch.ones_like(rew), 1e-5)
    assert torch.equal(adv, ret)


def test_registry_names_match_reference():
    """ppo_utils.py:451-456, 495-504: the same registered name sets."""
    assert set(ppo_utils.PolicyLossRegistry.list_available()) >= {
        "regular", "dual_clip", "gspo", "clip_cov", "kl_cov", "sapo", "cross_entropy", "importance_sampling", "cispo"}
    assert set(ppo_utils.AdvantageEstimatorRegistry.list_available()) >= {"grpo", "gae", "rloo", "reinforce++"}


@pytest.mark.gpu
@pytest.mark.parametrize("tag", LOSS_TAGS)
def test_gpu_secondary_loss_matches_reference(dev, tag):
    _check_loss(tag, dev)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", EST_TAGS)
def test_gpu_secondary_estimator_matches_reference(dev, tag):
    _check_est(tag, dev)
