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


@pytest.mark.parametrize("G,norm,mdt", [(8, True, torch.int64), (4, False, torch.int64), (1, True, torch.float32),
                                        (16, True, torch.int32), (5, True, torch.bool)])
def test_plan_grpo_advantages_equal_grpo_kernel(dev, G, norm, mdt):
    """skyrl_policy_train_plan_grpo: the plan launch also writes the mini-batch's GRPO advantages
    (pack's reward row sums as scores, contiguous groups of G). They must be skyrl_grpo_advantage's
    bits (ops.grpo_advantage on the same scores), and the plan's loss scales those of the plain
    plan (the micro-batches' losses unchanged), for every mask dtype, singleton groups and
    zero-variance groups."""
    n, R, mb = 8 * G if G > 1 else 24, 1024 if G != 5 else 130, 4
    g = torch.Generator().manual_seed(G * 10 + int(norm))
    lens = torch.randint(1, R + 1, (n,), generator=g)
    live = torch.arange(R)[None] < lens[:, None]
    rew = torch.zeros(n, R)
    rew[torch.arange(n), lens - 1] = (torch.rand(n, generator=g) < 0.4).float()
    rew[:G, :] = 0.0  # a zero-variance group (all scores 0)
    rmask = live.to(mdt).to(dev)
    lmask = (live & (torch.rand(n, R, generator=g) < 0.9)).float().to(dev)
    scores = rew.sum(-1).to(dev)
    params = _params(0, R)
    ref_adv = ops.grpo_advantage(rew.to(dev), rmask, None, None, n // G, epsilon=1e-6, norm_by_std=norm, scores=scores)
    old = torch.zeros(n, R, device=dev)
    adv = torch.full((n, R), float("nan"), device=dev)
    step = ops.PolicyTrainStep(old, adv, lmask, params, mb,
                               grpo=dict(scores=scores, response_mask=rmask, group_size=G, norm_by_std=norm))
    torch.cuda.synchronize()
    assert torch.equal(adv, ref_adv)
    ws_g = step.ws[:4096].clone()  # header + micro slots: scales and tags
    step2 = ops.PolicyTrainStep(old, adv, lmask, params, mb)  # the plain plan
    torch.cuda.synchronize()
    ws_p = step2.ws[:4096].clone()
    for k in range(step.n_micro):  # scal[0..2] of every micro slot are the same bits
        o = 256 + 256 * k
        assert torch.equal(ws_g[o:o + 12], ws_p[o:o + 12]), k


def test_plan_and_fold_wide_grids_at_bench_shape(dev):
    """The wide plan / fold (one wave per row, last arriver per micro-batch) at the bench's
    512 x 1024 with 32 micro-batches of 16: the step's per-micro-batch loss and metrics equal
    the per-call epilogue's (ops.policy_train on each micro-batch's logits) bit for bit, and the
    plan's GRPO advantages feed the passes."""
    n, R, mb, V = 64, 256, 16, 4096
    live, logits, labels, old, adv, ref, mask = _batch(dev, n, R, V, 3)
    params = _params(0, R)
    step = ops.PolicyTrainStep(old, adv, mask, params, mb, ref_log_probs=ref)
    for k in range(step.n_micro):
        i, j = step.rows(k)
        z = logits[i:j].contiguous().requires_grad_(True)
        step.micro(k, z, labels[i:j]).backward()
    losses, mets = step.fold()
    for k in range(step.n_micro):
        i, j = step.rows(k)
        zc = logits[i:j].contiguous().requires_grad_(True)
        l_c, m_c, _, _ = ops.policy_train(zc, labels[i:j], old[i:j], adv[i:j], mask[i:j], params, ref_log_probs=ref[i:j])
        assert torch.equal(losses[k], l_c.detach()), k
        assert torch.equal(mets[k], m_c), k


@pytest.mark.parametrize("red", [0, 1, 2])
def test_plan_with_pack_row_sums_equals_mask_plan(dev, red):
    """The plan given pack's loss-mask row sums (no loss-mask read, no hand-over between rows) writes
    the same slot scalars, epoch tags and row scales as the plan that sums the loss mask itself,
    for every loss reduction, with GRPO advantages and a ragged last micro-batch."""
    n, R, mb, G = 40, 300, 16, 4
    g = torch.Generator().manual_seed(red + 77)
    lens = torch.randint(1, R + 1, (n,), generator=g)
    live = torch.arange(R)[None] < lens[:, None]
    lmask = (live & (torch.rand(n, R, generator=g) < 0.8)).float().to(dev)
    scores = (torch.rand(n, generator=g) < 0.5).float().to(dev)
    rmask = live.to(torch.int64).to(dev)
    params = _params(red, R)
    old = torch.zeros(n, R, device=dev)
    outs = []
    for rows in (None, lmask.sum(-1)):
        adv = torch.full((n, R), float("nan"), device=dev)
        step = ops.PolicyTrainStep(old, adv, lmask, params, mb,
                                   grpo=dict(scores=scores, response_mask=rmask, group_size=G, loss_mask_row_sum=rows))
        torch.cuda.synchronize()
        nm = step.n_micro
        pad = lambda x: (x + 255) // 256 * 256  # noqa: E731
        rows_end = 256 + pad(nm * 256) + pad(n * 4)  # header, micro slots, row scales
        outs.append((adv.clone(), step.ws[:rows_end].clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    w0, w1 = (o[1].view(torch.int32) for o in outs)  # one cached workspace: the tags advance by one plan
    for k in range(nm):
        e = (256 + 256 * k) // 4 + 16
        assert int(w1[e]) == int(w0[e]) + (1 << 12), k
        w1[e] = w0[e]
    assert torch.equal(w0, w1)
