"""§8(f)1 decode side: the MFMA lm_head GEMM (csrc/lmhead_gemm.hip) and the sampler fused into
its epilogue, against

  * torch (exact small-integer operands: every product and sum is exact, so the bf16 logits must
    match bit for bit, which pins the MFMA operand/accumulator maps and the tile edges);
  * torch fp32 on random operands (bf16 output resolution);
  * the unfused path: skyrl_sample over the logits skyrl_lmhead_gemm writes -- tokens bit-exact,
    logprobs 1e-4 -- and oracle/sampler_ref.c on those same logits (tokens bit-exact);

at every BASELINE.json vocabulary (GPT-2 50,257: odd V, misaligned output rows), hidden sizes
768 / 1536 / 3584 / 4096, ragged M and V tile edges, T = 1, 0.7 and greedy.
"""

import pytest
import torch

from skyrl_amd import ops

pytestmark = pytest.mark.gpu


def _ints(shape, g, lo=-3, hi=4):
    return torch.randint(lo, hi, shape, generator=g).to(torch.bfloat16)


@pytest.mark.parametrize("M,V,K", [(300, 1037, 192), (256, 256, 64), (1, 300, 128), (513, 2100, 256)])
def test_gemm_exact_small_integers(dev, M, V, K):
    g = torch.Generator().manual_seed(M + V + K)
    h, w = _ints((M, K), g), _ints((V, K), g)
    w[:, 0] += torch.arange(V).remainder(5).to(torch.bfloat16)  # asymmetric: a row/col swap cannot pass
    z = ops.lmhead_gemm(h.to(dev), w.to(dev))
    ref = (h.float() @ w.float().T).to(torch.bfloat16)
    assert torch.equal(z.cpu(), ref)


@pytest.mark.parametrize("pipe", list(range(15)))
@pytest.mark.parametrize("K", [64, 128, 192, 1536])
def test_gemm_pipeline_variants_exact(dev, pipe, K):
    """Every tile/pipeline variant (256x256 BK 64 x 2 stages, 256x128 BK 32 x 3, 256x256 BK 32 x 4),
    incl. fewer K tiles than stages."""
    from skyrl_amd import _ffi

    g = torch.Generator().manual_seed(K + pipe)
    M, V = 300, 700
    h, w = _ints((M, K), g, -2, 3), _ints((V, K), g, -2, 3)
    with _ffi.variant(lmhead_pipe=pipe):
        z = ops.lmhead_gemm(h.to(dev), w.to(dev))
        tf, _ = ops.lmhead_sample(h.to(dev), w.to(dev), seed=3, step=1)
    assert torch.equal(z.cpu(), (h.float() @ w.float().T).to(torch.bfloat16))
    tu, _ = ops.sample(z, seed=3, step=1)
    assert torch.equal(tf, tu)


def test_gemm_strided_operands(dev):
    """Row strides larger than K (a [n, S, H] hidden slice) and an output with ld > V."""
    g = torch.Generator().manual_seed(5)
    M, V, K = 70, 777, 128
    hb = _ints((M, K + 64), g)
    w = _ints((V, K), g)
    out = torch.full((M, V + 9), 7.0, dtype=torch.bfloat16, device=dev)
    ops.lmhead_gemm(hb.to(dev)[:, :K], w.to(dev), out=out[:, :V])
    assert torch.equal(out[:, :V].cpu(), (hb[:, :K].float() @ w.float().T).to(torch.bfloat16))
    assert bool((out[:, V:] == 7.0).all())  # nothing written past N


def test_gemm_random_vs_fp32(dev):
    g = torch.Generator().manual_seed(11)
    M, V, K = 512, 4136, 1536
    h = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(V, K, generator=g) * 0.05).to(torch.bfloat16)
    z = ops.lmhead_gemm(h.to(dev), w.to(dev)).float().cpu()
    ref = h.float() @ w.float().T
    torch.testing.assert_close(z, ref, rtol=8e-3, atol=2e-3)  # bf16 output rounding


def _case(M, V, K, seed):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(V, K, generator=g) * (3.0 / K ** 0.5)).to(torch.bfloat16)  # logits ~ N(0, 9)
    ids = torch.randint(0, 1 << 40, (M,), generator=g)
    return h, w, ids


@pytest.mark.parametrize("V,K", [(50257, 768), (128256, 4096), (151936, 1536), (152064, 3584)])
@pytest.mark.parametrize("temp", [1.0, 0.7, 0.0])
def test_fused_sample_equals_unfused_per_vocab(dev, V, K, temp):
    for M, seed in ((37, 1), (300, 2)):
        h, w, ids = _case(M, V, K, seed + V)
        hd, wd, idd = h.to(dev), w.to(dev), ids.to(dev)
        z = ops.lmhead_gemm(hd, wd)
        tu, lu = ops.sample(z, temperature=temp, seed=77, seq_ids=idd, step=5)
        tf, lf = ops.lmhead_sample(hd, wd, temperature=temp, seed=77, seq_ids=idd, step=5)
        assert torch.equal(tf.cpu(), tu.cpu()), f"M={M}: {(tf != tu).sum().item()} tokens differ"
        torch.testing.assert_close(lf.cpu(), lu.cpu(), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("temp", [1.0, 0.7, 0.0])
def test_fused_sample_vs_oracle(dev, temp):
    from oracle import sampler as osamp

    M, V, K = 24, 151936, 1536
    h, w, ids = _case(M, V, K, 99)
    hd, wd = h.to(dev), w.to(dev)
    z = ops.lmhead_gemm(hd, wd).cpu()
    for step in (0, 13):
        tf, lf = ops.lmhead_sample(hd, wd, temperature=temp, seed=2024, seq_ids=ids.to(dev), step=step)
        et, el = osamp.sample(z, temp, -1, 1.0, 0.0, 2024, ids, step)
        assert torch.equal(tf.cpu(), et)
        torch.testing.assert_close(lf.cpu(), el, atol=1e-4, rtol=1e-5)


def test_fused_sample_row_independence_and_edges(dev):
    """A row's token depends only on its own hidden state, key and step (not on M or on which
    tile row it lands in), and M = 1 / M = 257 / a ragged last vocab tile work."""
    V, K = 1000, 256
    h, w, ids = _case(257, V, K, 3)
    hd, wd, idd = h.to(dev), w.to(dev), ids.to(dev)
    t_all, l_all = ops.lmhead_sample(hd, wd, seed=1, seq_ids=idd, step=2)
    for lo, hi in ((0, 1), (256, 257), (100, 220)):
        t, lp = ops.lmhead_sample(hd[lo:hi].contiguous(), wd, seed=1, seq_ids=idd[lo:hi], step=2)
        assert torch.equal(t.cpu(), t_all[lo:hi].cpu())
        torch.testing.assert_close(lp.cpu(), l_all[lo:hi].cpu(), atol=1e-5, rtol=1e-6)


def test_fused_sample_distribution_small_vocab(dev):
    """Empirical frequencies over 40k independent rows follow softmax(logits / T) (chi-square)."""
    import numpy as np
    from scipy import stats

    V, K, M = 24, 64, 40000
    g = torch.Generator().manual_seed(8)
    w = (torch.randn(V, K, generator=g) * 0.3).to(torch.bfloat16)
    h1 = torch.randn(1, K, generator=g).to(torch.bfloat16)
    hd = h1.to(dev).expand(M, K).contiguous()
    wd = w.to(dev)
    logits = ops.lmhead_gemm(hd[:1], wd).float().cpu()[0]
    for temp in (1.0, 0.7):
        tok, _ = ops.lmhead_sample(hd, wd, temperature=temp, seed=5, seq_ids=torch.arange(M, device=dev), step=0)
        counts = np.bincount(tok.cpu().numpy(), minlength=V)
        p = torch.softmax(logits / temp, 0).double().numpy()
        keep = p * M >= 5
        obs = np.append(counts[keep], counts[~keep].sum()).astype(np.float64)
        exp = np.append(p[keep], p[~keep].sum())
        exp = exp / exp.sum() * obs.sum()
        pval = stats.chisquare(obs, exp).pvalue
        assert pval > 1e-3, (temp, pval)


def test_lmhead_rejects_bad_operands(dev):
    h = torch.zeros(4, 100, dtype=torch.bfloat16, device=dev)  # K not a multiple of 64
    w = torch.zeros(10, 100, dtype=torch.bfloat16, device=dev)
    from skyrl_amd._ffi import SkyrlHipError

    with pytest.raises(SkyrlHipError):
        ops.lmhead_gemm(h, w)
    with pytest.raises(TypeError):
        ops.lmhead_gemm(h.float(), w)


@pytest.mark.parametrize("temp", [1.0, 0.7, 0.0])
def test_fused_sample_many_rows_steps_and_ties(dev, temp):
    """512 rows x 3 steps at the config-2 shape (every noise-bound branch, incl. groups whose
    E_g is tiny, occurs), and logits with few distinct values (exact ties in x and in score order
    are broken by the lowest index, as the unfused sampler does)."""
    V, K = 151936, 1536
    h, w, ids = _case(512, V, K, 1234)
    hd, wd, idd = h.to(dev), w.to(dev), ids.to(dev)
    z = ops.lmhead_gemm(hd, wd)
    for step in (0, 1, 999):
        tu, lu = ops.sample(z, temperature=temp, seed=9, seq_ids=idd, step=step)
        tf, lf = ops.lmhead_sample(hd, wd, temperature=temp, seed=9, seq_ids=idd, step=step)
        assert torch.equal(tf.cpu(), tu.cpu())
        torch.testing.assert_close(lf.cpu(), lu.cpu(), atol=1e-4, rtol=1e-5)
    g = torch.Generator().manual_seed(3)
    hq = torch.ones(64, 64, dtype=torch.bfloat16)
    hq[:, 1:] = 0
    wq = torch.zeros(4099, 64, dtype=torch.bfloat16)
    wq[:, 0] = torch.randint(-2, 3, (4099,), generator=g).to(torch.bfloat16)  # logits in {-2..2}
    hd, wd = hq.to(dev), wq.to(dev)
    z = ops.lmhead_gemm(hd, wd)
    ids = torch.arange(64, device=dev)
    tu, _ = ops.sample(z, temperature=temp, seed=4, seq_ids=ids, step=0)
    tf, _ = ops.lmhead_sample(hd, wd, temperature=temp, seed=4, seq_ids=ids, step=0)
    assert torch.equal(tf.cpu(), tu.cpu())


def test_fused_greedy_persistent_ties_and_variants(dev):
    """Greedy decode batches of 512+ rows take the persistent tile kernel: on tie-heavy logits
    (values in {-2..2} over V = 151,936, ragged last vocab tile) the first maximum wins as in the
    unfused sampler, and the one-tile-per-workgroup kernel (lmhead_persist 0) gives the same
    tokens and logprobs."""
    from skyrl_amd import _ffi

    g = torch.Generator().manual_seed(11)
    M, V, K = 520, 151936, 128
    hq = torch.zeros(M, K, dtype=torch.bfloat16)
    hq[:, 0] = 1
    hq[:, 1] = torch.randint(0, 2, (M,), generator=g).to(torch.bfloat16)
    wq = torch.zeros(V, K, dtype=torch.bfloat16)
    wq[:, 0] = torch.randint(-2, 2, (V,), generator=g).to(torch.bfloat16)
    wq[:, 1] = torch.randint(0, 2, (V,), generator=g).to(torch.bfloat16)  # row-dependent maxima
    hd, wd = hq.to(dev), wq.to(dev)
    z = ops.lmhead_gemm(hd, wd)
    tu, lu = ops.sample(z, temperature=0.0)
    tf, lf = ops.lmhead_sample(hd, wd, temperature=0.0)
    assert torch.equal(tf.cpu(), tu.cpu())
    torch.testing.assert_close(lf.cpu(), lu.cpu(), atol=1e-4, rtol=1e-5)
    with _ffi.variant(lmhead_persist=0):
        t0, l0 = ops.lmhead_sample(hd, wd, temperature=0.0)
    assert torch.equal(t0.cpu(), tf.cpu())
    torch.testing.assert_close(l0.cpu(), lf.cpu(), atol=1e-5, rtol=1e-6)


@pytest.mark.parametrize("V,K,temp", [(151936, 1536, 1.0), (50257, 768, 0.6), (4099, 128, 1.0)])
def test_lmhead_logprob_fwd_matches_oracle_and_chunked(dev, V, K, temp):
    """Learner-side forward (old / ref log-probs): the GEMM's online-softmax epilogue equals the
    fp32 oracle on the same bf16 logits (the kernel's own plain-GEMM output) and the chunked
    hipBLASLt path (skyrl_amd.lmhead) -- ragged last tile, odd V, temperature (bf16 division
    as the reference), labels at tile edges."""
    from oracle import cpu_ref
    from skyrl_amd import lmhead

    g = torch.Generator().manual_seed(V + K)
    T = 300
    h = torch.randn(T, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(V, K, generator=g) * (3.0 / K ** 0.5)).to(torch.bfloat16)
    lab = torch.randint(0, V, (T,), generator=g)
    lab[:4] = torch.tensor([0, 255, 256, V - 1])
    hd, wd = h.to(dev), w.to(dev)
    lp, ent = ops.lmhead_logprob_fwd(hd, wd, lab.to(dev), temperature=temp)
    z = ops.lmhead_gemm(hd, wd).cpu()
    zt = (z.float() / temp).to(torch.bfloat16) if temp != 1.0 else z
    torch.testing.assert_close(lp.cpu(), cpu_ref.logprobs_from_logits(zt, lab), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ent.cpu(), cpu_ref.entropy_from_logits(zt), atol=1e-4, rtol=1e-5)
    with torch.no_grad():  # an explicit chunk keeps the chunked hipBLASLt path
        lc, ec = lmhead.lmhead_logprobs_and_entropy(hd, wd, lab.to(dev), temperature=temp, chunk=lmhead.default_chunk(T, V))
        # without grad and without a chunk the call is the GEMM-epilogue kernel itself
        lr, er = lmhead.lmhead_logprobs_and_entropy(hd, wd, lab.to(dev), temperature=temp)
    torch.testing.assert_close(lp, lc, atol=2e-2, rtol=0)  # different GEMMs: bf16 logits may differ by an ulp
    torch.testing.assert_close(ent, ec, atol=2e-2, rtol=0)
    assert torch.equal(lr, lp) and torch.equal(er, ent)


@pytest.mark.parametrize("T,temp,K", [(1, 1.0, 256), (255, 1.0, 256), (257, 0.6, 256), (2600, 1.0, 256), (700, 1.0, 128)])
def test_lmhead_logprob_fwd_variants_and_edges(dev, T, temp, K):
    """Every lmhead_persist variant (0: one tile per workgroup, LDS-image epilogue; 1-4: the
    persistent kernel's copy placements) against the fp32 oracle on the kernel's own bf16 logits,
    at token counts around the 256-row tile (ragged M), V not a multiple of 256 (ragged last N tile)
    and labels at the vocabulary's ends; the persistent variants agree bit for bit."""
    from oracle import cpu_ref
    from skyrl_amd import _ffi

    g = torch.Generator().manual_seed(T)
    V = 3000 + 37  # K = 128: two K steps per tile, so W(g + 2) is always the next tile's
    h = torch.randn(T, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(V, K, generator=g) * (3.0 / K ** 0.5)).to(torch.bfloat16)
    lab = torch.randint(0, V, (T,), generator=g)
    lab[0] = V - 1
    if T > 1:
        lab[1] = 0
    hd, wd = h.to(dev), w.to(dev)
    z = ops.lmhead_gemm(hd, wd).cpu()
    zt = (z.float() / temp).to(torch.bfloat16) if temp != 1.0 else z
    e_lp, e_ent = cpu_ref.logprobs_from_logits(zt, lab), cpu_ref.entropy_from_logits(zt)
    got = {}
    for pv in range(5):
        with _ffi.variant(lmhead_persist=pv):
            lp, ent = ops.lmhead_logprob_fwd(hd, wd, lab.to(dev), temperature=temp)
        torch.testing.assert_close(lp.cpu(), e_lp, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(ent.cpu(), e_ent, atol=1e-4, rtol=1e-5)
        got[pv] = (lp, ent)
    for pv in (2, 3, 4):
        assert torch.equal(got[pv][0], got[1][0]) and torch.equal(got[pv][1], got[1][1])
    lp_ne, ent_ne = ops.lmhead_logprob_fwd(hd, wd, lab.to(dev), temperature=temp, compute_entropy=False)
    assert ent_ne is None and torch.equal(lp_ne, got[4][0])  # the entropy-free epilogue: same log-probs


@pytest.mark.parametrize("group", [8, 4, 3, 0])
def test_gemm_grouped_tile_order_exact(dev, group):
    """The grouped tile order (skyrl_variant lmhead_group: M tiles per group, M fastest inside a group)
    with a partial last group (M = 2600 -> 11 M tiles), exact on small-integer operands; the fused
    sampler and the learner logprob epilogue give the same results under every order."""
    from skyrl_amd import _ffi

    g = torch.Generator().manual_seed(2600 + group)
    M, V, K = 2600, 3000, 128
    h, w = _ints((M, K), g, -2, 3), _ints((V, K), g, -2, 3)
    w[:, 0] += torch.arange(V).remainder(5).to(torch.bfloat16)
    hd, wd = h.to(dev), w.to(dev)
    lab = torch.randint(0, V, (M,), generator=g).to(dev)
    with _ffi.variant(lmhead_group=group):
        z = ops.lmhead_gemm(hd, wd)
        tok, lp = ops.lmhead_sample(hd, wd, temperature=1.0, seed=9, step=2)
        lpf, entf = ops.lmhead_logprob_fwd(hd, wd, lab)
    assert torch.equal(z.cpu(), (h.float() @ w.float().T).to(torch.bfloat16))
    tok_u, lp_u = ops.sample(z, temperature=1.0, seed=9, step=2)
    assert torch.equal(tok, tok_u)
    torch.testing.assert_close(lp, lp_u, atol=1e-4, rtol=0)
    lpf_d, entf_d = ops.lmhead_logprob_fwd(hd, wd, lab)  # default order
    assert torch.equal(lpf, lpf_d) and torch.equal(entf, entf_d)
