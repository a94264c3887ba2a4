"""The step form of the fused policy pass (ABI 8: skyrl_policy_train_plan / _micro_fwd / _fold,
ops.PolicyTrainStep): one plan and one fold launch per mini-batch instead of a scales and an
epilogue launch per micro-batch. Per micro-batch the loss, metrics, logp / entropy and dlogits
must be the per-call form's bits (ops.policy_train_ragged / ops.policy_train on that
micro-batch), for packed and dense micro-batches, every loss reduction, a short last
micro-batch, temperature != 1 and GPT-2's odd V; and the oracle's loss assembly
(workers/worker.py:801-876 restated in oracle/cpu_ref.py) on the same inputs."""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import ops, ppo_utils
from skyrl_amd.config import AlgorithmConfig

pytestmark = pytest.mark.gpu

RED = ("token_mean", "sequence_mean", "seq_mean_token_sum_norm")


def _batch(dev, n, R, V, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(1, R + 1, (n,), generator=g)
    live = torch.arange(R)[None] < lens[:, None]
    logits = (torch.randn(n, R, V, generator=g) * 3).to(torch.bfloat16).to(dev)
    labels = torch.randint(0, V, (n, R), generator=g).to(dev)
    old = (-6 + torch.randn(n, R, generator=g)).to(dev)
    adv = torch.randn(n, R, generator=g).to(dev)
    ref = (-6 + torch.randn(n, R, generator=g)).to(dev)
    mask = (live & (torch.rand(n, R, generator=g) < 0.9)).float().to(dev)
    return live.to(dev), logits, labels, old, adv, ref, mask


def _params(red, R, kl=True, ent=True):
    cfg = AlgorithmConfig(use_entropy_loss=ent, policy_loss_type="dual_clip", loss_reduction=RED[red], max_seq_len=R)
    return ppo_utils.ppo_params_from_config(cfg, use_kl_loss=kl, use_entropy_loss=ent, has_entropy=True)


@pytest.mark.parametrize("V,red,temp", [(151936, 0, 1.0), (151936, 1, 1.0), (151936, 2, 1.0), (512, 0, 0.7),
                                        (50264, 1, 1.0), (50257, 0, 1.0)])
def test_step_matches_per_call_packed(dev, V, red, temp):
    n, R, mb = 7, 40, 3  # micro-batches of 3, 3, 1 rows
    live, logits, labels, old, adv, ref, mask = _batch(dev, n, R, V, V + red)
    params = _params(red, R)
    step = ops.PolicyTrainStep(old, adv, mask, params, mb, ref_log_probs=ref, temperature=temp)
    assert step.n_micro == 3
    grads, ref_out = [], []
    for k in range(step.n_micro):
        i, j = step.rows(k)
        lv = live[i:j]
        pos = torch.nonzero(lv.reshape(-1)).reshape(-1).to(torch.int32)
        z = logits[i:j][lv].contiguous().requires_grad_(True)
        loss = step.micro(k, z, labels[i:j][lv], pos)
        loss.backward()
        grads.append(z.grad)
        zc = logits[i:j][lv].contiguous().requires_grad_(True)
        l_c, m_c, lp_c, ent_c = ops.policy_train_ragged(zc, labels[i:j][lv], pos, old[i:j], adv[i:j], mask[i:j],
                                                        params, ref_log_probs=ref[i:j], temperature=temp)
        l_c.backward()
        ref_out.append((l_c.detach().clone(), m_c.clone(), lp_c, ent_c, zc.grad))
    losses, mets = step.fold()
    for k, (l_c, m_c, lp_c, ent_c, g_c) in enumerate(ref_out):
        i, j = step.rows(k)
        assert torch.equal(losses[k], l_c), (k, losses[k], l_c)
        assert torch.equal(mets[k][:7], m_c[:7]), (k, mets[k], m_c)
        assert torch.equal(step.logp[i:j], lp_c) and torch.equal(step.entropy[i:j], ent_c)
        assert torch.equal(grads[k], g_c)
    assert float(mets[:, 6].abs().sum()) == 0.0
    ops.check_loss_metrics(mets)


def test_step_dense_matches_per_call_dense(dev):
    """The dense form (the bench's: a micro-batch's [rows, R, V] rows of one matrix) against
    skyrl_policy_train_fwd per micro-batch; two mini-batches in a row on the same workspace (the
    exchange tags advance), and the step after a per-call launch on its own workspace."""
    n, R, V, mb = 8, 32, 151936, 4
    params = _params(0, R)
    for seed in (1, 2):
        live, logits, labels, old, adv, ref, mask = _batch(dev, n, R, V, seed)
        step = ops.PolicyTrainStep(old, adv, mask, params, mb, ref_log_probs=ref)
        outs = []
        for k in range(step.n_micro):
            i, j = step.rows(k)
            x = logits[i:j].clone().requires_grad_(True)
            step.micro(k, x, labels[i:j]).backward()
            xc = logits[i:j].clone().requires_grad_(True)
            l_c, m_c, lp_c, ent_c = ops.policy_train(xc, labels[i:j], old[i:j], adv[i:j], mask[i:j], params,
                                                     ref_log_probs=ref[i:j])
            l_c.backward()
            outs.append((x.grad, l_c.detach().clone(), m_c.clone(), lp_c, ent_c, xc.grad))
        losses, mets = step.fold()
        for k, (gx, l_c, m_c, lp_c, ent_c, g_c) in enumerate(outs):
            i, j = step.rows(k)
            assert torch.equal(losses[k], l_c) and torch.equal(mets[k][:7], m_c[:7])
            assert torch.equal(step.logp[i:j], lp_c) and torch.equal(step.entropy[i:j], ent_c)
            assert torch.equal(gx, g_c)


@pytest.mark.parametrize("red", [0, 1])
def test_step_matches_oracle_loss_assembly(dev, red):
    """Every micro-batch's final_loss / policy_loss / kl / entropy against the oracle's
    restatement of _forward_backward_micro on the kernel-independent fp32 logprobs of the same
    logits (cpu_ref.logprobs_from_logits), 1e-4."""
    n, R, V, mb = 6, 24, 4096, 2
    live, logits, labels, old, adv, ref, mask = _batch(dev, n, R, V, 11 + red)
    params = _params(red, R, ent=False)
    step = ops.PolicyTrainStep(old, adv, mask, params, mb, ref_log_probs=ref)
    for k in range(step.n_micro):
        i, j = step.rows(k)
        step.micro(k, logits[i:j].clone().requires_grad_(True), labels[i:j]).backward()
    losses, mets = step.fold()
    for k in range(step.n_micro):
        i, j = step.rows(k)
        lp = cpu_ref.logprobs_from_logits(logits[i:j].cpu(), labels[i:j].cpu())
        torch.testing.assert_close(step.logp[i:j].cpu(), lp, atol=1e-4, rtol=1e-4)
        loss, m = cpu_ref.policy_loss_assembly(lp, old[i:j].cpu(), adv[i:j].cpu(), mask[i:j].cpu(), ref[i:j].cpu(),
                                               None, dual_clip=True, reduction=RED[red], max_seq_len=R)
        assert abs(float(losses[k]) - float(loss)) < 1e-4, (k, float(losses[k]), float(loss))
        assert abs(float(mets[k][1]) - m["policy_loss"]) < 1e-4
        assert abs(float(mets[k][3]) - m["policy_kl"]) < 1e-4


def test_step_micro_without_tokens_and_errors(dev):
    """A micro-batch whose rows carry no loss mask folds to zero loss; index and shape errors raise."""
    n, R, V, mb = 4, 16, 1024, 2
    live, logits, labels, old, adv, ref, mask = _batch(dev, n, R, V, 5)
    mask[2:] = 0
    params = _params(0, R)
    step = ops.PolicyTrainStep(old, adv, mask, params, mb, ref_log_probs=ref)
    step.micro(0, logits[0:2].clone().requires_grad_(True), labels[0:2]).backward()
    losses, mets = step.fold()  # micro-batch 1 never launched: its positions have mask 0
    assert float(losses[1]) == 0.0 and float(mets[1][5]) == 0.0
    with pytest.raises(IndexError):
        step.micro(2, logits[0:2], labels[0:2])
    with pytest.raises(ValueError):
        step.micro(0, logits[0:1], labels[0:1])
