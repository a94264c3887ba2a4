"""Pin the CPU oracle (oracle/cpu_ref.py) to the reference: golden vectors produced by the real
reference (tools/gen_golden.py) and the reference's own known-answer tests (cited)."""

import numpy as np
import pytest
import torch

from oracle import cpu_ref


def close(a, b, atol=1e-5, rtol=1e-5):
    torch.testing.assert_close(torch.as_tensor(a).float(), torch.as_tensor(b).float(), atol=atol, rtol=rtol)


# ---------------------------------------------------------------- known answers from the reference tests
def test_kat_grpo_norm_std_false():
    # tests/cpu/utils/test_ppo_utils.py:146-172
    r = torch.tensor([[1.0, 2.0, 3.0], [1.0, 1.0, 1.0], [3.0, 3.0, 3.0], [4.0, 4.0, 4.0]])
    adv = cpu_ref.grpo_advantage(r, torch.ones_like(r), [0, 0, 1, 1], norm_by_std=False)
    close(adv, torch.tensor([1.5, -1.5, -1.5, 1.5]).unsqueeze(-1) * torch.ones_like(r))


def test_kat_grpo_singleton_and_bernoulli():
    # group [1,0,0,0] -> [1.49999702, -0.49999899 x3]
    r = torch.tensor([[1.0], [0.0], [0.0], [0.0]])
    adv = cpu_ref.grpo_advantage(r, torch.ones_like(r), ["a"] * 4)
    close(adv.squeeze(-1), torch.tensor([1.49999702, -0.49999899, -0.49999899, -0.49999899]), atol=1e-6)


def test_kat_gae():
    # tests/cpu/utils/test_ppo_utils.py:175-242
    rewards = torch.tensor([[1.0, 2.0, 3.0]])
    values = torch.tensor([[0.5, 1.0, 1.5]])
    adv, ret = cpu_ref.gae(rewards, values, torch.tensor([[1.0, 0.0, 1.0]]), 1.0, 1.0)
    close(ret, torch.tensor([[6.0, 5.0, 3.0]]))
    close(adv, torch.tensor([[0.7071, 0.1768, -0.7071]]), atol=1e-4)
    _, ret = cpu_ref.gae(rewards, values, torch.ones(1, 3), 0.5, 1.0)
    close(ret, torch.tensor([[2.75, 3.5, 3.0]]))
    _, ret = cpu_ref.gae(rewards, values, torch.ones(1, 3), 1.0, 0.5)
    close(ret, torch.tensor([[3.625, 4.25, 3.0]]))


def test_kat_dual_clip():
    # tests/cpu/algorithms/test_losses.py:32-82 -> 4.1667
    adv = torch.tensor([[1.0, -1.0, -4.0]])
    old = torch.tensor([[-1.0, -1.0, -3.0]])
    lp = torch.tensor([[-1.69315, -1.0, -0.69741]])
    loss, _ = cpu_ref.ppo_policy_loss(lp, old, adv, dual_clip=True, reduction="token_mean")
    assert loss.item() == pytest.approx(4.1667, abs=1e-4)


def test_kat_kl():
    # tests/cpu/utils/test_ppo_utils.py:44-62
    lp = torch.tensor([0.2, 0.3, 0.5])
    base = torch.tensor([0.1, 0.2, 0.4])
    close(cpu_ref.approx_kl(lp, base, kind="k1"), torch.tensor([0.1, 0.1, 0.1]))
    close(cpu_ref.approx_kl(lp, base, kind="abs"), torch.tensor([0.1, 0.1, 0.1]))
    close(cpu_ref.approx_kl(lp, base, kind="k2"), torch.tensor([0.005, 0.005, 0.005]))
    close(cpu_ref.approx_kl(lp, base, kind="k3"), torch.tensor([0.0048374, 0.0048374, 0.0048374]), atol=1e-6)


# ---------------------------------------------------------------- golden vectors from the real reference
@pytest.mark.parametrize("name", ["grpo_mixed", "grpo_synth"])
def test_grpo_golden(golden, name):
    d = golden(name)
    uids = list(d["uids"])
    for nbs in (1, 0):
        out = cpu_ref.grpo_advantage(d["rewards"], d["response_mask"], uids, norm_by_std=bool(nbs))
        close(out, d[f"adv_norm{nbs}"], atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("case", ["grpo", "dense", "const"])
def test_advnorm_golden(golden, case):
    """advantage_batch_normalize: normalize_advantages_dict (ppo_utils.py:127-145)."""
    d = golden("advnorm")
    out = cpu_ref.normalize_advantages(d[f"{case}_in"], d[f"{case}_mask"])
    close(out, d[f"{case}_out"], atol=1e-6, rtol=1e-6)


def test_gae_golden(golden):
    d = golden("gae")
    for tag, g, l in (("g1_l1", 1.0, 1.0), ("g099_l095", 0.99, 0.95), ("g05_l1", 0.5, 1.0)):
        adv, ret = cpu_ref.gae(d["rewards"], d["values"], d["response_mask"], g, l)
        close(adv, d[f"adv_{tag}"], atol=1e-5)
        close(ret, d[f"ret_{tag}"], atol=1e-5)
    d = golden("gae_long")
    adv, ret = cpu_ref.gae(d["rewards"], d["values"], d["response_mask"], 0.99, 0.95)
    close(adv, d["adv"], atol=1e-5)
    close(ret, d["ret"], atol=1e-5)


def test_kl_golden(golden):
    d = golden("kl")
    for k in ("k1", "abs", "k2", "k3"):
        close(cpu_ref.approx_kl(d["log_probs"], d["log_probs_base"], d["loss_mask"], k), d[f"kl_{k}_masked"])
        close(cpu_ref.approx_kl(d["log_probs"], d["log_probs_base"], None, k), d[f"kl_{k}"])


@pytest.mark.parametrize("lt", ["regular", "dual_clip"])
@pytest.mark.parametrize("red", ["token_mean", "sequence_mean", "seq_mean_token_sum_norm"])
def test_ppo_golden(golden, lt, red):
    d = golden("ppo")
    x = d["log_probs"].clone().requires_grad_(True)
    loss, m = cpu_ref.ppo_policy_loss(x, d["old_log_probs"], d["advantages"], eps_low=0.2, eps_high=0.28,
                                      dual_clip=lt == "dual_clip", reduction=red, mask=d["loss_mask"],
                                      max_seq_len=50)
    loss.backward()
    tag = f"{lt}_{red}"
    close(loss, d[f"loss_{tag}"], atol=1e-6)
    assert m["clip_ratio"] == pytest.approx(float(d[f"clip_{tag}"]), abs=1e-7)
    close(x.grad, d[f"grad_{tag}"], atol=1e-7)


@pytest.mark.parametrize("use_ent", [False, True])
def test_loss_assembly_golden(golden, use_ent):
    d = golden("ppo")
    x = d["log_probs"].clone().requires_grad_(True)
    e = d["entropy"].clone().requires_grad_(use_ent)
    final, m = cpu_ref.policy_loss_assembly(x, d["old_log_probs"], d["advantages"], d["loss_mask"],
                                            d["ref_log_probs"], e, use_entropy_loss=use_ent)
    final.backward()
    tag = f"asm_ent{int(use_ent)}"
    close(final, d[f"final_{tag}"], atol=1e-6)
    assert m["policy_kl"] == pytest.approx(float(d[f"kl_{tag}"]), abs=1e-7)
    close(x.grad, d[f"grad_lp_{tag}"], atol=1e-7)
    if use_ent:
        close(e.grad, d[f"grad_ent_{tag}"], atol=1e-7)


def test_critic_golden(golden):
    d = golden("critic")
    for tag, vc in (("clip", 0.2), ("noclip", None)):
        x = d["values"].clone().requires_grad_(True)
        loss, cf = cpu_ref.critic_loss(x, d["old_values"], d["returns"], d["loss_mask"], vc)
        loss.backward()
        close(loss, d[f"loss_{tag}"], atol=1e-6)
        close(x.grad, d[f"grad_{tag}"], atol=1e-7)
        if vc is not None:
            assert cf == pytest.approx(float(d[f"clipfrac_{tag}"]), abs=1e-7)


def test_logprob_golden(golden):
    d = golden("logprob_f32")
    for temp in (1.0, 0.7):
        tag = f"f32_t{str(temp).replace('.', '')}"
        x = d["logits"].clone().requires_grad_(True)
        lp = cpu_ref.logprobs_from_logits(x, d["labels"], temperature=temp)
        ent = cpu_ref.entropy_from_logits(x, temperature=temp)
        (lp * d[f"glp_{tag}"] + ent * d[f"gent_{tag}"]).sum().backward()
        close(lp, d[f"logp_{tag}"], atol=2e-5)
        close(ent, d[f"ent_{tag}"], atol=2e-5)
        close(x.grad, d[f"dlogits_{tag}"], atol=1e-6)
    d = golden("logprob_bf16")
    close(cpu_ref.logprobs_from_logits(d["logits"], d["labels"]), d["logp_fp32math"], atol=2e-5)
    close(cpu_ref.entropy_from_logits(d["logits"]), d["ent_fp32math"], atol=2e-5)
    close(cpu_ref.entropy_from_logits(d["logits"], in_dtype=True), d["ent_bf16math"], atol=1e-6)
    close(cpu_ref.logprobs_from_logits(d["logits"], d["labels"], temperature=0.6), d["logp_t06"], atol=2e-5)


def _ragged(vals, off):
    return [vals[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]


def test_pack_golden(golden):
    d = golden("pack")
    po, ro = d["prompt_off"].numpy(), d["response_off"].numpy()
    args = (_ragged(d["prompt_vals"].numpy(), po), _ragged(d["response_vals"].numpy(), ro),
            _ragged(d["reward_vals"].numpy(), d["reward_off"].numpy()),
            _ragged(d["loss_mask_vals"].numpy(), d["loss_mask_off"].numpy()),
            _ragged(d["logprob_vals"].numpy(), d["logprob_off"].numpy()))
    seq, att, rm, rw, lm, lp = cpu_ref.pack(*args, pad_id=0)
    for k, v in (("sequences", seq), ("attention_mask", att), ("response_mask", rm)):
        assert np.array_equal(v, d[k].numpy()), k
    for k, v in (("rewards", rw), ("loss_mask", lm), ("rollout_logprobs", lp)):
        assert np.array_equal(v, d[k].numpy()), k
    pad = int(d["pad_size"])
    seq, att, rm, rw, lm, lp = cpu_ref.pack(*args, pad_id=0, pad=pad)
    for k, v in (("p_sequences", seq), ("p_attention_mask", att), ("p_response_mask", rm), ("p_rewards", rw),
                 ("p_loss_mask", lm), ("p_rollout_logprobs", lp)):
        assert np.array_equal(v, d[k].numpy()), k


def test_reward_kl_golden(golden):
    d = golden("reward_kl")
    for kind in ("k1", "k3"):
        rew, avg, mx = cpu_ref.reward_kl_penalty(d["rewards"], d["action_log_probs"], d["base_action_log_probs"],
                                                 d["loss_mask"], kind, float(d["kl_coef"]))
        close(rew, d[f"rewards_{kind}"], atol=1e-7)
        assert avg == pytest.approx(float(d[f"avg_kl_{kind}"]), abs=1e-7)
        assert mx == pytest.approx(float(d[f"avg_kl_max_{kind}"]), abs=1e-7)
