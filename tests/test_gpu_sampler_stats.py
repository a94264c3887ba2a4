"""Statistical tests of the sampler's noise (a1), which bit-exactness vs oracle/sampler_ref.c
cannot pin (the oracle restates the same noise model: one hash per 8-token group, the group's
exponential race built from order statistics).

Over 200k independent sequence ids (one draw each) on V = 2048 logits spread over +-6:
  * the token frequencies match softmax(x / T) at T = 1 and T = 0.7 (chi-square p > 1e-3,
    low-probability tokens pooled to expected counts >= 5);
  * with top_p = 0.9 they match the renormalised nucleus (tx generator.py:424-449 semantics)
    and no token outside it is ever drawn;
  * groups are independent: equal-logit competitions between tokens in the same group
    (v, v+1), in adjacent groups (v, v+8) and two groups apart (v, v+16), at every slot offset,
    split 50/50, and a 3-way race over slots of three consecutive groups follows its softmax.
Reference semantics: vLLM samples from softmax(logits / T) after top-k/top-p/min-p
(inference_engines/utils.py:15-42; filter order skyrl-tx/tx/utils/generator.py:213-227,398-449).
"""

import numpy as np
import pytest
import torch
from scipy import stats

from skyrl_amd import ops

pytestmark = pytest.mark.gpu
N = 200_000
V = 2048


def _draw(dev, row, temp=1.0, top_p=1.0, seed=11, step=0):
    logits = row.to(torch.bfloat16).to(dev).unsqueeze(0).expand(N, V).contiguous()
    ids = torch.arange(N, dtype=torch.int64, device=dev) * 2654435761 % (1 << 40)
    tok, _ = ops.sample(logits, temperature=temp, top_p=top_p, seed=seed, seq_ids=ids, step=step, want_logprobs=False)
    return torch.bincount(tok.long().cpu(), minlength=V).numpy().astype(np.float64)


def _chi2_p(counts, probs):
    exp = probs * counts.sum()
    order = np.argsort(exp)
    # pool the smallest expectations into bins of >= 5 expected draws
    obs_b, exp_b, acc_o, acc_e = [], [], 0.0, 0.0
    for i in order:
        acc_o += counts[i]
        acc_e += exp[i]
        if acc_e >= 5.0:
            obs_b.append(acc_o)
            exp_b.append(acc_e)
            acc_o = acc_e = 0.0
    if acc_e > 0:
        obs_b[-1] += acc_o
        exp_b[-1] += acc_e
    return stats.chisquare(np.array(obs_b), np.array(exp_b)).pvalue


def _row(seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(V, generator=g) * 12 - 6).to(torch.bfloat16).float()


@pytest.mark.parametrize("temp", [1.0, 0.7])
def test_frequencies_match_softmax(dev, temp):
    x = _row(1).double()
    p = torch.softmax(x / temp, -1).numpy()
    counts = _draw(dev, x.float(), temp=temp)
    assert _chi2_p(counts, p) > 1e-3
    # and every slot of the group (p % 8) carries its own probability mass
    slot_obs = np.array([counts[s::8].sum() for s in range(8)])
    slot_exp = np.array([p[s::8].sum() for s in range(8)]) * N
    assert stats.chisquare(slot_obs, slot_exp).pvalue > 1e-3


def test_top_p_nucleus(dev):
    for seed in range(2, 64):  # a row whose cut is not within 1e-4 of p (the kernel's masses are fixed point)
        x = _row(seed).double()
        p = torch.softmax(x, -1).numpy()
        order = np.argsort(-p, kind="stable")
        before = np.concatenate([[0.0], np.cumsum(p[order])[:-1]])
        keep = order[before < 0.9]
        cut = before[len(keep)] if len(keep) < V else 1.0
        if abs(cut - 0.9) > 1e-4 and abs(before[len(keep) - 1] - 0.9) > 1e-4:
            break
    nucleus = np.zeros(V)
    nucleus[keep] = p[keep] / p[keep].sum()
    counts = _draw(dev, x.float(), top_p=0.9, seed=12)
    assert counts[nucleus == 0].sum() == 0
    assert _chi2_p(counts[keep], nucleus[keep]) > 1e-3


@pytest.mark.parametrize("gap", [1, 8, 16])
def test_group_noise_independence(dev, gap):
    """Equal logits at v and v + gap, everything else far below: P = 1/2 each, for every slot v % 8."""
    results = []
    for slot in range(8):
        v = 64 + slot
        x = torch.full((V,), -30.0)
        x[v] = 2.0
        x[v + gap] = 2.0
        c = _draw(dev, x, seed=100 + slot * 7 + gap)
        assert c[v] + c[v + gap] == N
        results.append(stats.binomtest(int(c[v]), N, 0.5).pvalue)
    assert min(results) > 1e-4, results


def test_three_group_race(dev):
    """Three tokens in consecutive groups at different slots with probabilities 0.2 / 0.3 / 0.5."""
    x = torch.full((V,), -30.0)
    idx = [200 + 3, 208 + 6, 216 + 0]
    pr = np.array([0.2, 0.3, 0.5])
    x[idx] = torch.log(torch.tensor(pr)).float()
    c = _draw(dev, x, seed=31)
    obs = c[idx]
    assert obs.sum() == N
    xb = x.to(torch.bfloat16).double()[idx]  # the kernel sees bf16 logits
    exp = torch.softmax(xb, -1).numpy() * N
    assert stats.chisquare(obs, exp).pvalue > 1e-3
