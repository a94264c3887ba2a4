"""a1 filter semantics pinned to the reference's own sampler fixtures.

The reference's only sampler fixtures are skyrl-tx's (tests/utils/test_generator.py:182-238,
testing tx/utils/generator.py:398-449):

* apply_top_k_batch keeps EXACTLY k tokens: lax.top_k, then the first-k mask; equal logits
  are taken in index order (the row [5, 4, 3, 3, 1] with k = 3 keeps indices 0, 1, 2).
* apply_top_p_batch keeps tokens in descending order (stable argsort) while the probability
  mass strictly before them is < p; the top token always (p = 0 keeps one token).

The fixture rows below are the literal inputs and kept supports (finite entries of the
expected arrays) of those tests. CPU tests pin the oracle (oracle/sampler_ref.c) to them and
to a numpy stable top-k on tie-heavy bf16 rows at V = 151,936; the GPU tests check that
skyrl_sample draws exactly that support and stays bit-exact against the oracle.
"""

import numpy as np
import pytest
import torch

# (logits row, top_k, top_p, kept indices) from skyrl-tx/tests/utils/test_generator.py
TOPK_ROWS = [
    ([1.0, 2.0, 3.0, 4.0, 5.0], 2, 1.0, [3, 4]),             # :185-191
    ([1.0, 2.0, 3.0, 4.0, 5.0], -1, 1.0, [0, 1, 2, 3, 4]),   # :193-195 (k <= 0: no filtering)
    ([5.0, 4.0, 3.0, 3.0, 1.0], 3, 1.0, [0, 1, 2]),          # :197-207 (ties: first 3.0 only)
]
TOPP_ROWS = [
    ([0.0, 1.0, 2.0, 3.0, 4.0, 6.0], -1, 1.0, [0, 1, 2, 3, 4, 5]),  # :215-217
    ([0.0, 1.0, 2.0, 3.0, 4.0, 6.0], -1, 0.0, [5]),                 # :219-222
    ([0.0, 1.0, 2.0, 3.0, 4.0, 6.0], -1, 0.9, [4, 5]),              # :224-227
]
FIXTURE_ROWS = TOPK_ROWS + TOPP_ROWS


def _expected_mask(V, kept):
    m = torch.zeros(V, dtype=torch.bool)
    m[kept] = True
    return m


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("row", FIXTURE_ROWS, ids=lambda r: f"k{r[1]}_p{r[2]}_{len(r[0])}")
def test_oracle_support_matches_tx_fixture(row, dtype):
    from oracle import sampler as osamp

    x, k, p, kept = row
    logits = torch.tensor([x], dtype=dtype)
    got = osamp.support(logits, temperature=1.0, top_k=k, top_p=p)[0]
    assert torch.equal(got, _expected_mask(len(x), kept)), (row, got)


def test_oracle_support_batched_tx_rows():
    """tx's batched cases (:197-207, :229-238): per-row parameters are the same as one row at a
    time, and the tie row keeps exactly k."""
    from oracle import sampler as osamp

    rows = torch.tensor([[1.0, 2.0, 3.0, 4.0, 5.0], [5.0, 4.0, 3.0, 3.0, 1.0]])
    assert torch.equal(osamp.support(rows[:1], top_k=2)[0], _expected_mask(5, [3, 4]))
    assert torch.equal(osamp.support(rows[1:], top_k=3)[0], _expected_mask(5, [0, 1, 2]))
    rp = torch.tensor([[0.0, 1.0, 2.0, 3.0, 4.0, 6.0]] * 2)
    assert osamp.support(rp, top_p=1.0).all()
    assert torch.equal(osamp.support(rp, top_p=0.0), torch.stack([_expected_mask(6, [5])] * 2))


def _tie_heavy_rows(n, V, seed):
    """bf16 logits N(0, 3^2) rounded to quarters: values repeat, so the k-th largest sits inside
    a tie group with larger values above it."""
    g = torch.Generator().manual_seed(seed)
    lv = torch.round(torch.randn(n, V, generator=g) * 12.0) * 0.25
    return lv.to(torch.bfloat16)


def _stable_topk_mask(row_bf16, k):
    """numpy restatement of lax.top_k + the first-k mask (apply_top_k_batch :410-418)."""
    x = row_bf16.float().numpy()
    idx = np.argsort(-x, kind="stable")[:k]
    m = np.zeros(x.shape[0], dtype=bool)
    m[idx] = True
    return torch.from_numpy(m)


@pytest.mark.parametrize("k", [1, 50, 777])
def test_oracle_topk_exact_k_on_tie_heavy_vocab(k):
    from oracle import sampler as osamp

    V = 151936
    rows = _tie_heavy_rows(3, V, 11 + k)
    sup = osamp.support(rows, temperature=0.8, top_k=k)
    for i in range(rows.shape[0]):
        assert int(sup[i].sum()) == k
        assert torch.equal(sup[i], _stable_topk_mask(rows[i], k))


def test_oracle_topk_then_topp_composes_like_tx():
    """tx applies top_p to the top_k-filtered logits (generator.py:217-220): the top_p mass is
    renormalised over the k kept tokens. Row [5,4,3,3,1], k = 3, T = 1: masses e^5, e^4, e^3
    over the three kept tokens are 0.665, 0.245, 0.090; p = 0.8 keeps two tokens (mass before
    the third is 0.910 >= 0.8), p = 0.95 keeps all three."""
    from oracle import sampler as osamp

    row = torch.tensor([[5.0, 4.0, 3.0, 3.0, 1.0]])
    assert torch.equal(osamp.support(row, top_k=3, top_p=0.8)[0], _expected_mask(5, [0, 1]))
    assert torch.equal(osamp.support(row, top_k=3, top_p=0.95)[0], _expected_mask(5, [0, 1, 2]))


# ------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("row", FIXTURE_ROWS, ids=lambda r: f"k{r[1]}_p{r[2]}_{len(r[0])}")
def test_gpu_sampler_draws_tx_fixture_support(dev, row, dtype):
    """20,000 independent draws (distinct sequence keys) of each fixture row through
    skyrl_sample: the set of drawn tokens equals tx's kept support, and every token equals the
    oracle's."""
    from oracle import sampler as osamp
    from skyrl_amd import ops

    x, k, p, kept = row
    n = 20000
    logits = torch.tensor([x], dtype=dtype).expand(n, -1).contiguous()
    ids = torch.arange(n, dtype=torch.int64) * 7 + 3
    tok, lp = ops.sample(logits.to(dev), temperature=1.0, top_k=k, top_p=p, seed=5, seq_ids=ids.to(dev), step=2)
    tok = tok.cpu()
    assert set(tok.tolist()) == set(kept), (row, sorted(set(tok.tolist())))
    etok, elp = osamp.sample(logits, 1.0, k, p, 0.0, 5, ids, 2)
    assert torch.equal(tok, etok)
    torch.testing.assert_close(lp.cpu(), elp, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("top_p", [1.0, 0.9])
def test_gpu_sampler_topk50_exactly_50_on_ties(dev, top_p):
    """bf16 tie-heavy rows at V = 151,936 with top_k = 50 (the §8(d) filter variant): the draws of
    a row never leave the stable top-50 set, at a high temperature every one of the 50 is drawn
    (so exactly 50 survive, not the whole tie group at the 50th value), and the tokens are
    bit-exact against the oracle."""
    from oracle import sampler as osamp
    from skyrl_amd import ops

    V, base, reps = 151936, 4, 2048
    rows = _tie_heavy_rows(base, V, 99)
    for i in range(base):  # the 50th value must be inside a tie group for the test to bite
        srt = torch.sort(rows[i].float(), descending=True).values
        assert srt[49] == srt[50]
    big = rows.repeat_interleave(reps, dim=0)
    ids = torch.arange(base * reps, dtype=torch.int64)
    temp = 1.0 if top_p < 1.0 else 50.0
    tok, _ = ops.sample(big.to(dev), temperature=temp, top_k=50, top_p=top_p, seed=13, seq_ids=ids.to(dev), step=0)
    tok = tok.cpu().view(base, reps)
    for i in range(base):
        allowed = set(torch.nonzero(_stable_topk_mask(rows[i], 50)).flatten().tolist())
        drawn = set(tok[i].tolist())
        assert drawn <= allowed, (i, sorted(drawn - allowed))
        if top_p == 1.0:
            assert drawn == allowed, (i, len(drawn))
    sub = torch.arange(0, base * reps, reps // 8)  # 32 rows through the oracle
    etok, _ = osamp.sample(big[sub], temp, 50, top_p, 0.0, 13, ids[sub], 0)
    assert torch.equal(tok.flatten()[sub], etok)
