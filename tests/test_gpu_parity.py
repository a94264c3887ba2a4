"""HIP hot path vs the reference: golden vectors (made by the real reference) and the CPU
oracle on the same seeded inputs, through the C ABI (skyrl_amd.ops -> libskyrl_hip.so).

Tolerances (north_star): token indices / integer / byte outputs bit-exact; logprobs,
advantages and losses within 1e-4 (fp32); gradients 1e-6 absolute on O(1e-3) values.
"""

import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import ops, ppo_utils, torch_utils
from skyrl_amd.config import AlgorithmConfig

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def close(a, b, atol=1e-5, rtol=1e-5):
    torch.testing.assert_close(torch.as_tensor(a).detach().float().cpu(), torch.as_tensor(b).detach().float().cpu(),
                               atol=atol, rtol=rtol)


def test_native_library_is_loaded():
    lib = ops._ffi.load()
    assert lib._name.endswith("skyrl_amd/lib/libskyrl_hip.so")
    maps = open("/proc/self/maps").read()
    assert "libskyrl_hip.so" in maps


# ------------------------------------------------------------------------------------------ a4 GRPO
@pytest.mark.parametrize("name", ["grpo_mixed", "grpo_synth"])
@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.float32, torch.bool])
def test_grpo_golden(golden, dev, name, mask_dtype):
    d = golden(name)
    for nbs in (1, 0):
        adv, ret = ppo_utils.compute_grpo_outcome_advantage(
            d["rewards"].to(dev), d["response_mask"].to(mask_dtype).to(dev), list(d["uids"]),
            grpo_norm_by_std=bool(nbs))
        assert adv.data_ptr() == ret.data_ptr()
        close(adv, d[f"adv_norm{nbs}"], atol=1e-6, rtol=1e-6)


def test_grpo_north_star_size_vs_oracle(dev):
    g = torch.Generator().manual_seed(1234)
    N, R, G = 512, 1024, 8
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None] < lens[:, None]).to(torch.int64)
    rew = torch.zeros(N, R)
    rew[torch.arange(N), lens - 1] = (torch.rand(N, generator=g) < 0.3).float()
    uids = [str(i // G) for i in range(N)]
    adv, _ = ppo_utils.compute_grpo_outcome_advantage(rew.to(dev), mask.to(dev), uids)
    close(adv, cpu_ref.grpo_advantage(rew, mask, uids), atol=1e-6, rtol=1e-6)
    # size-independent properties: per group the masked advantages sum to ~0 per row-score; padded = 0
    assert torch.all(adv.cpu()[mask == 0] == 0)
    again, _ = ppo_utils.compute_grpo_outcome_advantage(rew.to(dev), mask.to(dev), uids)
    assert torch.equal(adv, again)  # deterministic, bit for bit


def test_grpo_large_group_and_odd_width(dev):
    g = torch.Generator().manual_seed(5)
    N, R = 1500, 37  # one group of 1100 rows (> LDS cache of 1024 scores), odd R (scalar path)
    rew = torch.randn(N, R, generator=g)
    mask = (torch.rand(N, R, generator=g) < 0.9).to(torch.int64)
    uids = ["big"] * 1100 + [str(i) for i in range(400)]
    adv, _ = ppo_utils.compute_grpo_outcome_advantage(rew.to(dev), mask.to(dev), uids)
    close(adv, cpu_ref.grpo_advantage(rew, mask, uids), atol=2e-5, rtol=1e-4)


# ------------------------------------------------------------------------------------------ a5 GAE
def test_gae_golden(golden, dev):
    d = golden("gae")
    for tag, g, l in (("g1_l1", 1.0, 1.0), ("g099_l095", 0.99, 0.95), ("g05_l1", 0.5, 1.0)):
        adv, ret = ppo_utils.compute_gae_advantage_return(d["rewards"].to(dev), d["values"].to(dev),
                                                          d["response_mask"].to(dev), g, l)
        close(adv, d[f"adv_{tag}"], atol=1e-4)
        close(ret, d[f"ret_{tag}"], atol=1e-5)
    d = golden("gae_long")
    adv, ret = ppo_utils.compute_gae_advantage_return(d["rewards"].to(dev), d["values"].to(dev),
                                                      d["response_mask"].to(dev), 0.99, 0.95)
    close(adv, d["adv"], atol=1e-4)
    close(ret, d["ret"], atol=1e-5)


def test_gae_kat_and_errors(dev):
    r = torch.tensor([[1.0, 2.0, 3.0]], device=dev)
    v = torch.tensor([[0.5, 1.0, 1.5]], device=dev)
    adv, ret = ppo_utils.compute_gae_advantage_return(r, v, torch.tensor([[1.0, 0.0, 1.0]], device=dev), 1.0, 1.0)
    close(ret, [[6.0, 5.0, 3.0]])
    close(adv, [[0.7071, 0.1768, -0.7071]], atol=1e-4)
    with pytest.raises(ValueError, match="At least one element"):
        ppo_utils.compute_gae_advantage_return(r, v, torch.zeros(1, 3, device=dev), 1.0, 1.0)
    with pytest.raises(ValueError, match="sum of the mask is one"):
        ppo_utils.compute_gae_advantage_return(r, v, torch.tensor([[0.0, 1.0, 0.0]], device=dev), 1.0, 1.0)


def test_gae_north_star_size(dev):
    g = torch.Generator().manual_seed(3)
    N, R = 512, 1024
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None] < lens[:, None]).float()
    rew = torch.zeros(N, R)
    rew[torch.arange(N), lens - 1] = (torch.rand(N, generator=g) < 0.3).float()
    val = torch.randn(N, R, generator=g) * 0.1
    adv, ret = ppo_utils.compute_gae_advantage_return(rew.to(dev), val.to(dev), mask.to(dev), 1.0, 0.95)
    eadv, eret = cpu_ref.gae(rew, val, mask, 1.0, 0.95)
    close(ret, eret, atol=1e-4, rtol=1e-4)
    close(adv, eadv, atol=1e-4, rtol=1e-4)


# ------------------------------------------------------------------------------------------ a6 KL
def test_kl_golden(golden, dev):
    d = golden("kl")
    for k in ("k1", "abs", "k2", "k3"):
        close(ppo_utils.compute_approx_kl(d["log_probs"].to(dev), d["log_probs_base"].to(dev),
                                          d["loss_mask"].to(dev), k), d[f"kl_{k}_masked"], atol=1e-6)
        close(ppo_utils.compute_approx_kl(d["log_probs"].to(dev), d["log_probs_base"].to(dev), None, k),
              d[f"kl_{k}"], atol=1e-6)


def test_reward_kl_golden(golden, dev):
    d = golden("reward_kl")
    for kind in ("k1", "k3"):
        rew, m = ops.reward_kl_penalty(d["rewards"].to(dev), d["action_log_probs"].to(dev),
                                       d["base_action_log_probs"].to(dev), d["loss_mask"].to(dev), kind,
                                       float(d["kl_coef"]))
        close(rew, d[f"rewards_{kind}"], atol=1e-6)
        close(m[0], d[f"avg_kl_{kind}"], atol=1e-6)
        close(m[1], d[f"avg_kl_max_{kind}"], atol=1e-6)


# ------------------------------------------------------------------------------------------ a7 loss
@pytest.mark.parametrize("lt", ["regular", "dual_clip"])
@pytest.mark.parametrize("red", ["token_mean", "sequence_mean", "seq_mean_token_sum_norm"])
def test_ppo_golden(golden, dev, lt, red):
    d = golden("ppo")
    cfg = AlgorithmConfig(policy_loss_type=lt, loss_reduction=red, max_seq_len=50, eps_clip_low=0.2,
                          eps_clip_high=0.28)
    x = d["log_probs"].to(dev).requires_grad_(True)
    loss, m = ppo_utils.PolicyLossRegistry.get(lt)(x, d["old_log_probs"].to(dev), d["advantages"].to(dev), cfg,
                                                   loss_mask=d["loss_mask"].to(dev))
    loss.backward()
    tag = f"{lt}_{red}"
    close(loss, d[f"loss_{tag}"], atol=1e-6)
    assert m["clip_ratio"] == pytest.approx(float(d[f"clip_{tag}"]), abs=1e-6)
    close(x.grad, d[f"grad_{tag}"], atol=1e-7, rtol=1e-5)


@pytest.mark.parametrize("use_ent", [False, True])
def test_loss_assembly_golden(golden, dev, use_ent):
    d = golden("ppo")
    cfg = AlgorithmConfig(use_entropy_loss=use_ent)
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=use_ent, has_entropy=True)
    x = d["log_probs"].to(dev).requires_grad_(True)
    e = d["entropy"].to(dev).requires_grad_(use_ent)
    loss, m = ops.ppo_loss(x, d["old_log_probs"].to(dev), d["advantages"].to(dev), d["loss_mask"].to(dev), params,
                           ref_log_probs=d["ref_log_probs"].to(dev), entropy=e)
    loss.backward()
    tag = f"asm_ent{int(use_ent)}"
    close(loss, d[f"final_{tag}"], atol=1e-6)
    close(m[1], d[f"pg_{tag}"], atol=1e-6)
    close(m[3], d[f"kl_{tag}"], atol=1e-6)
    close(m[2], d[f"entropy_{tag}"], atol=1e-6)
    close(m[4], d[f"clip_{tag}"], atol=1e-6)
    close(x.grad, d[f"grad_lp_{tag}"], atol=1e-7, rtol=1e-5)
    if use_ent:
        close(e.grad, d[f"grad_ent_{tag}"], atol=1e-7, rtol=1e-5)


def test_ppo_upstream_grad_scaling_and_kat(dev):
    adv = torch.tensor([[1.0, -1.0, -4.0]], device=dev)
    old = torch.tensor([[-1.0, -1.0, -3.0]], device=dev)
    lp = torch.tensor([[-1.69315, -1.0, -0.69741]], device=dev, requires_grad=True)
    cfg = AlgorithmConfig(policy_loss_type="dual_clip", loss_reduction="token_mean", max_seq_len=4)
    loss, _ = ppo_utils.ppo_policy_loss(lp, old, adv, cfg)
    assert loss.item() == pytest.approx(4.1667, abs=1e-4)  # tests/cpu/algorithms/test_losses.py:32-82
    (loss * 3.0).backward()
    x = lp.detach().cpu().requires_grad_(True)
    e, _ = cpu_ref.ppo_policy_loss(x, old.cpu(), adv.cpu(), dual_clip=True)
    (e * 3.0).backward()
    close(lp.grad, x.grad, atol=1e-6)


def test_ppo_north_star_size_vs_oracle(dev):
    g = torch.Generator().manual_seed(1234)
    N, R = 512, 1024
    lens = torch.randint(1, R + 1, (N,), generator=g)
    mask = (torch.arange(R)[None] < lens[:, None]).float()
    lp = -2 + 0.1 * torch.randn(N, R, generator=g)
    old = lp + 0.05 * torch.randn(N, R, generator=g)
    ref = lp + 0.05 * torch.randn(N, R, generator=g)
    adv = torch.randn(N, R, generator=g) * mask
    ent = torch.rand(N, R, generator=g)
    cfg = AlgorithmConfig()
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, has_entropy=True)
    x = lp.to(dev).requires_grad_(True)
    loss, m = ops.ppo_loss(x, old.to(dev), adv.to(dev), mask.to(dev), params, ref.to(dev), ent.to(dev))
    loss.backward()
    xc = lp.clone().requires_grad_(True)
    e, em = cpu_ref.policy_loss_assembly(xc, old, adv, mask, ref, ent)
    e.backward()
    close(loss, e, atol=1e-6, rtol=1e-5)
    close(m[4], em["clip_ratio"], atol=1e-6)
    close(x.grad, xc.grad, atol=1e-9, rtol=1e-4)


@pytest.mark.parametrize("red", ["token_mean", "sequence_mean", "seq_mean_token_sum_norm"])
@pytest.mark.parametrize("n", [37, 1500])
def test_ppo_one_launch_paths_agree(dev, red, n):
    """The one-launch loss with the pack's row sums, with in-kernel row sums, and (n > 1024)
    with the separate token_mean total all give the oracle's loss/metrics/gradients; the
    backward rescales by a non-unit upstream gradient (and leaves unit ones untouched)."""
    g = torch.Generator().manual_seed(n)
    for R in (300, 1024, 2500):
        lens = torch.randint(0, R + 1, (n,), generator=g)
        mask = (torch.arange(R)[None] < lens[:, None]).float()
        lp = -2 + 0.1 * torch.randn(n, R, generator=g)
        old = lp + 0.05 * torch.randn(n, R, generator=g)
        ref = lp + 0.05 * torch.randn(n, R, generator=g)
        adv = torch.randn(n, R, generator=g) * mask
        ent = torch.rand(n, R, generator=g)
        cfg = AlgorithmConfig(loss_reduction=red, max_seq_len=R, use_entropy_loss=True, entropy_loss_coef=0.01,
                              policy_loss_type="dual_clip")
        params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=True, has_entropy=True)
        xc = lp.clone().requires_grad_(True)
        ec = ent.clone().requires_grad_(True)
        e, em = cpu_ref.policy_loss_assembly(xc, old, adv, mask, ref, ec, use_entropy_loss=True, ent_coef=0.01,
                                             reduction=red, max_seq_len=R, dual_clip=True)
        (e * 2.5).backward()
        outs = []
        for rows in (mask.sum(-1).to(dev), None):
            x = lp.to(dev).requires_grad_(True)
            en = ent.to(dev).requires_grad_(True)
            loss, m = ops.ppo_loss(x, old.to(dev), adv.to(dev), mask.to(dev), params, ref.to(dev), en,
                                   loss_mask_row_sum=rows)
            (loss * 2.5).backward()
            close(loss, e, atol=1e-6, rtol=1e-5)
            close(m[4], em["clip_ratio"], atol=1e-6)
            close(m[3], em["policy_kl"], atol=1e-6, rtol=1e-5)
            close(m[5], mask.sum(), atol=0)
            close(x.grad, xc.grad, atol=1e-9, rtol=1e-4)
            close(en.grad, ec.grad, atol=1e-12, rtol=1e-5)
            outs.append((loss.detach().cpu(), x.grad.cpu(), m.cpu()))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        assert torch.equal(outs[0][2], outs[1][2])


def test_pack_emits_loss_mask_row_sums(golden, dev):
    d = golden("pack")
    N = len(d["prompt_off"]) - 1
    P = int((d["prompt_off"][1:] - d["prompt_off"][:-1]).max())
    R = int((d["response_off"][1:] - d["response_off"][:-1]).max())
    pad = int(d["pad_size"])
    out = ops.pack_experience(d["prompt_vals"].to(dev), d["prompt_off"], d["response_vals"].to(dev),
                              d["response_off"], d["reward_vals"].to(dev), d["reward_off"],
                              d["loss_mask_vals"].to(dev), d["loss_mask_off"], d["logprob_vals"].to(dev),
                              d["logprob_off"], N=N, P=P, R=R, pad=pad, pad_token_id=0, return_row_sums=True)
    assert len(out) == 8
    assert torch.equal(out[4].cpu(), d["p_loss_mask"])
    assert torch.equal(out[6].cpu(), d["p_loss_mask"].sum(-1))
    # reward row sums = the GRPO scores of the padded rewards (ppo_utils.py:1156)
    torch.testing.assert_close(out[7].cpu(), d["p_rewards"].sum(-1), atol=1e-6, rtol=1e-6)


def test_pack_reward_row_sums_are_the_grpo_scores_bit_exact(dev):
    """pack's reward_row_sum is summed in the GRPO kernel's order: scores given to
    skyrl_grpo_advantage reproduce what it computes from the rewards, bit for bit (R % 4 == 0;
    dense per-token rewards so the summation order matters)."""
    g = torch.Generator().manual_seed(17)
    N, R, G = 96, 1024, 8
    rl = torch.randint(1, R + 1, (N,), generator=g)
    pl = torch.randint(1, 40, (N,), generator=g)
    roff = torch.zeros(N + 1, dtype=torch.int64)
    roff[1:] = torch.cumsum(rl, 0)
    poff = torch.zeros(N + 1, dtype=torch.int64)
    poff[1:] = torch.cumsum(pl, 0)
    tot = int(roff[-1])
    vals = torch.randn(tot, generator=g) * 0.1
    out = ops.pack_experience(torch.randint(0, 100, (int(poff[-1]),), generator=g).to(dev), poff.to(dev),
                              torch.randint(0, 100, (tot,), generator=g).to(dev), roff.to(dev), vals.to(dev),
                              roff.to(dev), torch.ones(tot, device=dev), roff.to(dev), None, None, N=N, P=40, R=R,
                              return_row_sums=True)
    rew, rmask, scores = out[3], out[2], out[7]
    own = torch.empty(N, device=dev)
    a0 = ops.grpo_advantage(rew, rmask, None, None, N // G, scores_out=own)
    a1 = ops.grpo_advantage(rew, rmask, None, None, N // G, scores=scores)
    assert torch.equal(own, scores)
    assert torch.equal(a0, a1)
    goff, grows, ng = ops.groups_from_index([str(i % 12) for i in range(N)])  # CSR groups
    a2 = ops.grpo_advantage(rew, rmask, goff, grows, ng)
    a3 = ops.grpo_advantage(rew, rmask, goff, grows, ng, scores=scores)
    assert torch.equal(a2, a3)


@pytest.mark.parametrize("case", ["tis_token", "tis_seq", "mask_geo", "mask_prod", "tis_outlier"])
@pytest.mark.parametrize("lt", ["regular", "dual_clip"])
def test_ppo_off_policy_correction_golden(golden, dev, case, lt):
    """ppo_policy_loss + apply_off_policy_correction (off_policy_correction_utils.py:7-296) on
    the HIP loss, against the reference's own outputs (tests/golden/ppo_offpolicy.npz)."""
    from skyrl_amd import ppo_utils
    from skyrl_amd.config import AlgorithmConfig, OffPolicyCorrectionConfig

    d = golden("ppo_offpolicy")
    kw = {"tis_token": dict(tis_ratio_type="token", token_tis_ratio_clip_high=2.0),
          "tis_seq": dict(tis_ratio_type="sequence", sequence_tis_ratio_clip_high=5.0),
          "mask_geo": dict(sequence_mask_metric="geometric", geo_mask_high=1.01, geo_mask_low=0.99),
          "mask_prod": dict(sequence_mask_metric="product", product_mask_high=2.0, product_mask_low=0.5),
          "tis_outlier": dict(tis_ratio_type="token", token_tis_ratio_clip_high=3.0,
                              outlier_token_is_threshold_low=0.2, outlier_token_is_threshold_high=4.0)}[case]
    cfg = AlgorithmConfig(policy_loss_type=lt, loss_reduction="token_mean", eps_clip_low=0.2, eps_clip_high=0.28,
                          off_policy_correction=OffPolicyCorrectionConfig(**kw))
    x = d["log_probs"].to(dev).requires_grad_(True)
    loss, m = ppo_utils.PolicyLossRegistry.get(lt)(x, d["old_log_probs"].to(dev), d["advantages"].to(dev), cfg,
                                                    loss_mask=d["loss_mask"].to(dev),
                                                    rollout_logprobs=d["rollout_logprobs"].to(dev))
    loss.backward()
    t = f"{case}_{lt}"
    ref_loss = float(d[f"loss_{t}"])
    assert float(loss.detach()) == pytest.approx(ref_loss, rel=1e-5, abs=1e-5)
    g = d[f"grad_{t}"]
    torch.testing.assert_close(x.grad.cpu(), g, atol=1e-5 * max(1.0, float(g.abs().max())), rtol=1e-4)
    keys = [str(k) for k in d[f"mkeys_{t}"]]
    assert sorted(m) == keys
    for k, v in zip(keys, d[f"mvals_{t}"].tolist()):
        assert m[k] == pytest.approx(v, rel=1e-5, abs=1e-6), k


# ------------------------------------------------------------------------------------------ a8 critic
def test_critic_golden(golden, dev):
    d = golden("critic")
    for tag, vc in (("clip", 0.2), ("noclip", None)):
        x = d["values"].to(dev).requires_grad_(True)
        loss, cf = ppo_utils.ppo_critic_loss(x, d["old_values"].to(dev), d["returns"].to(dev),
                                             AlgorithmConfig(value_clip=vc), loss_mask=d["loss_mask"].to(dev))
        loss.backward()
        close(loss, d[f"loss_{tag}"], atol=1e-6)
        close(x.grad, d[f"grad_{tag}"], atol=1e-7, rtol=1e-5)
        if vc is not None:
            assert cf == pytest.approx(float(d[f"clipfrac_{tag}"]), abs=1e-6)


# ------------------------------------------------------------------------------------------ a2/a3 logprob
@pytest.mark.parametrize("temp", [1.0, 0.7])
def test_logprob_f32_golden(golden, dev, temp):
    d = golden("logprob_f32")
    tag = f"f32_t{str(temp).replace('.', '')}"
    x = d["logits"].to(dev).requires_grad_(True)
    lp, ent = torch_utils.logprobs_and_entropy(x, d["labels"].to(dev), temperature=temp, entropy_requires_grad=True)
    (lp * d[f"glp_{tag}"].to(dev) + ent * d[f"gent_{tag}"].to(dev)).sum().backward()
    close(lp, d[f"logp_{tag}"], atol=1e-4)
    close(ent, d[f"ent_{tag}"], atol=1e-4)
    close(x.grad, d[f"dlogits_{tag}"], atol=1e-6)


def test_logprob_bf16_golden(golden, dev):
    d = golden("logprob_bf16")
    lg = d["logits"].to(dev)
    lab = d["labels"].to(dev)
    lp, ent = torch_utils.logprobs_and_entropy(lg, lab)
    close(lp, d["logp_fp32math"], atol=1e-4)
    close(ent, d["ent_fp32math"], atol=1e-4)
    close(ent, d["ent_bf16math"], atol=5e-2)  # the reference computes entropy in bf16
    lp6 = torch_utils.logprobs_from_logits(lg, lab, temperature=0.6)
    close(lp6, d["logp_t06"], atol=1e-4)
    close(torch_utils.chunked_entropy_from_logits(lg), d["ent_fp32math"], atol=1e-4)


def test_logprob_strided_response_slice_qwen_vocab(dev):
    """The model-wrapper call: logits[:, -R-1:-1] of a [n,S,V] tensor, V = 151,936 (Qwen2.5)."""
    g = torch.Generator().manual_seed(9)
    n, S, R, V = 2, 40, 24, 151936
    logits = (torch.randn(n, S, V, generator=g) * 3).to(torch.bfloat16)
    seq = torch.randint(0, V, (n, S), generator=g)
    view = logits.to(dev)[:, -R - 1:-1]
    labels = seq.to(dev)[:, -R:]
    x = view.detach().requires_grad_(True)
    lp, ent = torch_utils.logprobs_and_entropy(x, labels, entropy_requires_grad=True)
    close(lp, cpu_ref.logprobs_from_logits(logits[:, -R - 1:-1], seq[:, -R:]), atol=1e-4)
    close(ent, cpu_ref.entropy_from_logits(logits[:, -R - 1:-1]), atol=1e-4)
    g_lp = torch.randn(n, R, generator=g)
    (lp * g_lp.to(dev)).sum().backward()
    xc = logits[:, -R - 1:-1].float().requires_grad_(True)
    (cpu_ref.logprobs_from_logits(xc, seq[:, -R:]) * g_lp).sum().backward()
    close(x.grad, xc.grad, atol=4e-3, rtol=1e-2)  # dlogits are stored in bf16


def test_logprob_gpt2_odd_vocab(dev):
    g = torch.Generator().manual_seed(4)
    n, T, V = 3, 5, 50257  # GPT-2 (config 1): odd V -> misaligned rows take the scalar path
    logits = (torch.randn(n, T, V, generator=g) * 2).to(torch.bfloat16)
    labels = torch.randint(0, V, (n, T), generator=g)
    lp, ent = torch_utils.logprobs_and_entropy(logits.to(dev), labels.to(dev))
    close(lp, cpu_ref.logprobs_from_logits(logits, labels), atol=1e-4)
    close(ent, cpu_ref.entropy_from_logits(logits), atol=1e-4)


# ------------------------------------------------------------------------------------------ a9 pack
def test_pack_golden(golden, dev):
    d = golden("pack")
    N = len(d["prompt_off"]) - 1
    P = int((d["prompt_off"][1:] - d["prompt_off"][:-1]).max())
    R = int((d["response_off"][1:] - d["response_off"][:-1]).max())
    for pad, pre in ((0, ""), (int(d["pad_size"]), "p_")):
        out = ops.pack_experience(d["prompt_vals"].to(dev), d["prompt_off"], d["response_vals"].to(dev),
                                  d["response_off"], d["reward_vals"].to(dev), d["reward_off"],
                                  d["loss_mask_vals"].to(dev), d["loss_mask_off"], d["logprob_vals"].to(dev),
                                  d["logprob_off"], N=N, P=P, R=R, pad=pad, pad_token_id=0)
        for k, v in zip(("sequences", "attention_mask", "response_mask", "rewards", "loss_mask", "rollout_logprobs"),
                        out):
            assert torch.equal(v.cpu(), d[pre + k]), pre + k


# ------------------------------------------------------------------------------------------ a1 sampler
def _oracle_sample(logits_cpu, temperature, top_k, min_p, seed, seq_ids, step, top_p=1.0):
    from oracle import sampler as osamp

    return osamp.sample(logits_cpu, temperature, top_k, top_p, min_p, seed, seq_ids, step)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [(1.0, -1, 0.0), (0.7, -1, 0.0), (0.0, -1, 0.0), (1.0, 50, 0.0), (1.0, -1, 0.05),
                                 (0.8, 20, 0.1)])
def test_sampler_bit_exact_vs_oracle(dev, dtype, cfg):
    temp, top_k, min_p = cfg
    g = torch.Generator().manual_seed(17)
    n, V = 8, 151936
    logits = (torch.randn(n, V, generator=g) * 3).to(dtype)
    ids = torch.arange(100, 100 + n, dtype=torch.int64)
    for step in (0, 5):
        tok, lp = ops.sample(logits.to(dev), temperature=temp, top_k=top_k, min_p=min_p, seed=1234,
                             seq_ids=ids.to(dev), step=step)
        etok, elp = _oracle_sample(logits, temp, top_k, min_p, 1234, ids, step)
        assert torch.equal(tok.cpu(), etok), (tok.cpu(), etok)
        close(lp, elp, atol=1e-4)
        close(lp, torch.log_softmax(logits.float(), -1)[torch.arange(n), etok.long()], atol=1e-4)


@pytest.mark.parametrize("cfg", [(1.0, -1, 0.0), (0.0, -1, 0.0), (0.6, 40, 0.02)])
def test_sampler_row_mode_bit_exact(dev, cfg):
    """nseq >= 256: one workgroup per row (no split hand-off), rows strided as in the decode loop."""
    temp, top_k, min_p = cfg
    g = torch.Generator().manual_seed(23)
    n, V = 300, 32003
    full = (torch.randn(n, 2, V, generator=g) * 2.5).to(torch.bfloat16)
    ids = torch.arange(n, dtype=torch.int64) * 7
    x = full.to(dev)[:, 1]  # row stride 2V, odd V: unaligned rows take the ragged path
    tok, lp = ops.sample(x, temperature=temp, top_k=top_k, min_p=min_p, seed=5, seq_ids=ids.to(dev), step=3)
    etok, elp = _oracle_sample(full[:, 1].contiguous(), temp, top_k, min_p, 5, ids, 3)
    assert torch.equal(tok.cpu(), etok)
    close(lp, elp, atol=1e-4)


def test_sampler_extreme_logit_range(dev):
    """Logits spanning +-3e4 (bf16) with a spike: the online sum-exp must not overflow."""
    g = torch.Generator().manual_seed(4)
    n, V = 260, 4096
    logits = torch.randn(n, V, generator=g) * 50
    logits[:, 3] = 3.0e4
    logits[:, 100] = -3.0e4
    logits[::2, 4000] = 3.1e4
    logits = logits.to(torch.bfloat16)
    for temp in (1.0, 0.0):
        tok, lp = ops.sample(logits.to(dev), temperature=temp, seed=1, step=0)
        etok, elp = _oracle_sample(logits, temp, -1, 0.0, 1, torch.arange(n), 0)
        assert torch.equal(tok.cpu(), etok)
        close(lp, torch.log_softmax(logits.float(), -1)[torch.arange(n), etok.long()], atol=1e-4)
        assert torch.isfinite(lp).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [(1.0, -1, 0.9, 0.0), (0.8, 50, 0.9, 0.0), (1.0, -1, 0.5, 0.02), (1.3, 200, 0.97, 0.0),
                                 (1.0, -1, 0.001, 0.0)])
def test_sampler_top_p_bit_exact_vs_oracle(dev, dtype, cfg):
    """top_p (skyrl-tx generator.py:424-449) after top_k/min_p; 300 rows exercise the row mode."""
    temp, top_k, top_p, min_p = cfg
    g = torch.Generator().manual_seed(29)
    n, V = 300, 5003
    logits = (torch.randn(n, V, generator=g) * 2.0).to(dtype)
    ids = torch.arange(n, dtype=torch.int64) + 11
    tok, lp = ops.sample(logits.to(dev), temperature=temp, top_k=top_k, top_p=top_p, min_p=min_p, seed=9,
                         seq_ids=ids.to(dev), step=4)
    etok, elp = _oracle_sample(logits, temp, top_k, min_p, 9, ids, 4, top_p=top_p)
    assert torch.equal(tok.cpu(), etok)
    close(lp, elp, atol=1e-4)


def test_sampler_top_p_ties_and_support(dev):
    """bf16 logits on a coarse grid: the top_p cut lands inside tie groups (index-order rule)."""
    g = torch.Generator().manual_seed(31)
    n, V = 64, 2048
    logits = torch.round(torch.randn(n, V, generator=g) * 2) / 2  # ~12 distinct values, large tie groups
    logits = logits.to(torch.bfloat16)
    for top_p in (0.3, 0.75, 0.95):
        for step in range(3):
            tok, _ = ops.sample(logits.to(dev), top_p=top_p, seed=3, step=step)
            etok, _ = _oracle_sample(logits, 1.0, -1, 0.0, 3, torch.arange(n), step, top_p=top_p)
            assert torch.equal(tok.cpu(), etok)
        # every sampled token is inside the nucleus computed in float64 (cut ties in index order)
        x = logits.double()
        p = torch.softmax(x, -1)
        order = torch.sort(-x, dim=-1, stable=True).indices
        ps = torch.gather(p, 1, order)
        keep_sorted = (torch.cumsum(ps, -1) - ps) < top_p
        keep_sorted[:, 0] = True
        keep = torch.zeros_like(keep_sorted)
        keep.scatter_(1, order, keep_sorted)
        assert keep[torch.arange(n), tok.cpu().long()].all()


def test_sampler_top_p_distribution(dev):
    small = torch.tensor([[0.0, 1.0, 2.0, -1.0]]).repeat(20000, 1)
    tok, _ = ops.sample(small.to(dev), top_p=0.7, seed=5, seq_ids=torch.arange(20000, device=dev), step=0)
    freq = torch.bincount(tok.cpu().long(), minlength=4).float() / 20000
    p = torch.softmax(small[0], -1)
    expect = torch.tensor([0.0, p[1], p[2], 0.0]) / (p[1] + p[2])  # nucleus {2, 1}
    close(freq, expect, atol=0.015)


def test_sampler_odd_vocab_and_distribution(dev):
    g = torch.Generator().manual_seed(2)
    V = 1027
    logits = torch.randn(1, V, generator=g).to(torch.bfloat16)
    tok, _ = ops.sample(logits.to(dev), seed=7, seq_ids=torch.tensor([3], device=dev), step=11)
    etok, _ = _oracle_sample(logits, 1.0, -1, 0.0, 7, torch.tensor([3]), 11)
    assert torch.equal(tok.cpu(), etok)
    # Gumbel-max samples softmax(logits): frequencies over many independent streams
    small = torch.tensor([[0.0, 1.0, 2.0, -1.0]]).repeat(20000, 1)
    tok, _ = ops.sample(small.to(dev), seed=99, seq_ids=torch.arange(20000, device=dev), step=0)
    freq = torch.bincount(tok.cpu().long(), minlength=4).float() / 20000
    close(freq, torch.softmax(small[0], -1), atol=0.015)


# ------------------------------------------------------------------------------------------ fused training pass
@pytest.mark.parametrize("red", ["token_mean", "sequence_mean", "seq_mean_token_sum_norm"])
@pytest.mark.parametrize("use_ent", [False, True])
def test_policy_train_fused_matches_unfused_and_oracle(dev, red, use_ent):
    g = torch.Generator().manual_seed(31)
    n, R, V = 3, 40, 4096
    logits = (torch.randn(n, R, V, generator=g) * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (n, R), generator=g)
    lens = torch.tensor([40, 17, 1])
    mask = (torch.arange(R)[None] < lens[:, None]).float()
    lp0 = cpu_ref.logprobs_from_logits(logits, labels)
    old = lp0 + 0.1 * torch.randn(n, R, generator=g)
    ref = lp0 + 0.1 * torch.randn(n, R, generator=g)
    adv = torch.randn(n, R, generator=g)
    cfg = AlgorithmConfig(loss_reduction=red, max_seq_len=64, use_entropy_loss=use_ent, policy_loss_type="dual_clip")
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=use_ent, has_entropy=True)
    x = logits.to(dev).requires_grad_(True)
    loss, m, lp, ent = ops.policy_train(x, labels.to(dev), old.to(dev), adv.to(dev), mask.to(dev), params,
                                        ref_log_probs=ref.to(dev))
    (loss * 2.0).backward()
    # unfused HIP path
    x2 = logits.to(dev).requires_grad_(True)
    lp2, ent2 = ops.logprobs_and_entropy(x2, labels.to(dev), 1.0, compute_entropy=use_ent)
    loss2, m2 = ops.ppo_loss(lp2, old.to(dev), adv.to(dev), mask.to(dev), params, ref_log_probs=ref.to(dev),
                             entropy=ent2)
    (loss2 * 2.0).backward()
    close(lp, lp2, atol=1e-6)
    close(ent, ent2, atol=1e-6)
    close(loss, loss2, atol=1e-6)
    close(m[:6], m2[:6], atol=1e-6)
    close(x.grad, x2.grad, atol=1e-6, rtol=1e-2)
    # CPU oracle: torch autograd through the restated reference path (fp32 math on the bf16 logits)
    xc = logits.float().requires_grad_(True)
    lpc = cpu_ref.logprobs_from_logits(xc, labels)
    entc = cpu_ref.entropy_from_logits(xc)
    final, mc = cpu_ref.policy_loss_assembly(lpc, old, adv, mask, ref, entc, use_entropy_loss=use_ent,
                                             dual_clip=True, reduction=red, max_seq_len=64)
    (final * 2.0).backward()
    close(loss, final, atol=2e-5, rtol=1e-4)
    close(lp, lpc, atol=1e-4)
    close(x.grad, xc.grad, atol=2e-6, rtol=1e-2)  # dlogits stored in bf16


@pytest.mark.parametrize("temp", [1.0, 0.8])
def test_policy_train_resident_qwen_vocab(dev, temp):
    """V = 151,936 takes the register-resident fused kernel; compare with the two-sweep kernel."""
    g = torch.Generator().manual_seed(5)
    n, R, V = 2, 6, 151936
    logits = (torch.randn(n, R, V, generator=g) * 3).to(torch.bfloat16).to(dev)
    labels = torch.randint(0, V, (n, R), generator=g).to(dev)
    mask = torch.tensor([[1.0] * 6, [1.0] * 3 + [0.0] * 3], device=dev)
    old = torch.randn(n, R, generator=g).to(dev) - 12
    ref = old + 0.05
    adv = torch.randn(n, R, generator=g).to(dev)
    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(use_entropy_loss=True), use_kl_loss=True,
                                              use_entropy_loss=True, has_entropy=True)
    outs = []
    for resident in (1, 0):
        with ops.variant(train_resident=resident):
            x = logits.clone().requires_grad_(True)
            loss, m, lp, ent = ops.policy_train(x, labels, old, adv, mask, params, ref_log_probs=ref, temperature=temp)
            loss.backward()
        outs.append((loss.detach(), m.clone(), lp, ent, x.grad))
    for a, b in zip(outs[0], outs[1]):
        close(a, b, atol=1e-6, rtol=1e-5)
    lpc = cpu_ref.logprobs_from_logits(logits.cpu(), labels.cpu(), temperature=temp)
    close(outs[0][2], lpc, atol=1e-4)
