"""a1 filtered sampling without top_k: the top_p / min_p kernel (sample_topp_kernel) against the
two-kernel path it replaces (the filter pre-pass + the MODE 2 sampler,
skyrl_variant sampler_topp_fast = 0) and against oracle/sampler_ref.c. The tests force the kernel
with sampler_topp_fast = 2 (ops.variant, per call); the default (1) sends min_p without top_p below 256 rows
to the two-kernel path, which is faster there.

Pass 1 takes the row max, a count histogram per exact bf16 key and MODE 2's race over the whole
row (every scored element recorded); the top_p cut is found on chip and the race's best record
decides the row when it is admissible (RowFilter.tk = 1). The other rows run pass 2 (MODE 2 over
the keys above the cut, the cut key's elements ranked by index): for top_p in a second launch,
sample_topp_pass2_kernel, each left row cut into 8 pieces with the last piece merging; for min_p
alone in the same workgroup. Tokens, logprobs and the recorded cut (key, last kept index) must be
the two-kernel path's bit for bit. Rows outside its bounds (the cut among the values below 2^-16
or the zeros, a tie group over 1024 at the cut, NaN / +inf, values >= 2^16, over 512 nonzero
values below 2^-16) run the two-kernel path's code in the workgroup (RowFilter.ik =
kRowFallback); the rest are kRowDone. The variant topp_probe = 5 sends every row through pass 2.
The recipe this serves: top_p = 0.95 alone (examples/text_to_sql/run_skyrl_sql.sh:60 and eight
more example scripts), semantics skyrl-tx/tx/utils/generator.py:423-449.
"""

import pytest
import torch

from skyrl_amd import ops

pytestmark = pytest.mark.gpu

_COUNTER_BYTES = 1024 * 4  # sampler workspace: 1024 per-row split counters first, then one 20-B RowFilter per row
_ROW_DONE = -2
_ROW_FALLBACK = -3


def _filters(x):
    ws = ops.WORKSPACES.get(x.device, "sample", ops._ffi.query("skyrl_sample_workspace_bytes", x.shape[0], x.shape[1]))
    n = x.shape[0]
    return ws[_COUNTER_BYTES:_COUNTER_BYTES + 20 * n].view(torch.int32).view(n, 5).cpu().clone()


def _run(x, fast, **kw):
    with ops.variant(sampler_topp_fast=2 if fast else 0):  # 2: the one-pass kernel at any row count
        tok, lp = ops.sample(x, **kw)
        torch.cuda.synchronize()
        return tok.cpu(), lp.cpu(), _filters(x)


def _ab(x, min_done, **kw):
    tf, lf, ff = _run(x, True, **kw)
    ts, ls, fs = _run(x, False, **kw)
    assert torch.equal(tf, ts), (kw, int((tf != ts).sum()))
    assert torch.allclose(lf, ls, atol=2e-5, rtol=1e-5, equal_nan=True), (kw, (lf - ls).abs().max())
    done = ff[:, 2] == _ROW_DONE
    assert bool(((ff[:, 2] == _ROW_DONE) | (ff[:, 2] == _ROW_FALLBACK)).all())
    if kw.get("top_p", 1.0) < 1.0:  # the cut (key, and the last kept index where the kernel resolved it:
        # -1 = a split tie group that pass 1's certified decision did not need to rank) of every row
        assert torch.equal(ff[done][:, 3], fs[done][:, 3])
        rk = done & (ff[:, 4] != -1)
        assert torch.equal(ff[rk][:, 4], fs[rk][:, 4])
    assert int(done.sum()) >= min_done, (kw, int(done.sum()), x.shape[0])
    return tf, lf, int(done.sum())


@pytest.mark.parametrize("cfg", [(1.0, 0.95, 0.0), (1.0, 0.9, 0.0), (0.7, 0.9, 0.05), (1.3, 0.5, 0.0),
                                 (1.0, 1.0, 0.1), (0.8, 1.0, 0.02), (1.0, 0.0, 0.0), (1.0, 0.999, 0.0)])
def test_topp_fast_equals_two_kernel_path_bench_shape(dev, cfg):
    """[512, 151,936] bf16 N(0, 3^2) rows (the bench's decode step): every row is decided by the
    two-pass kernel and tokens, logprobs and cuts equal the two-kernel path's."""
    temp, p, mp = cfg
    g = torch.Generator().manual_seed(int(p * 1000) + int(mp * 100) + 3)
    x = (torch.randn(512, 151936, generator=g) * 3).to(torch.bfloat16).to(dev)
    ids = torch.arange(512, dtype=torch.int64, device=dev) * 5 + 2
    _ab(x, 512, temperature=temp, top_p=p, min_p=mp, seed=11, seq_ids=ids, step=4)


def test_topp_fast_bench_shape_matches_oracle(dev):
    """top_p = 0.95 alone (the SkyRL-SQL recipe), T = 1, at the bench's V = 151,936 against
    oracle/sampler_ref.c directly, 512 rows: tokens bit-exact, logprobs 1e-4."""
    from oracle import sampler as osamp

    g = torch.Generator().manual_seed(95)
    x = (torch.randn(512, 151936, generator=g) * 3).to(torch.bfloat16)
    ids = torch.arange(512, dtype=torch.int64) * 3 + 1
    tok, lp, ff = _run(x.to(dev), True, temperature=1.0, top_p=0.95, seed=21, seq_ids=ids.to(dev), step=5)
    assert int((ff[:, 2] == _ROW_DONE).sum()) == 512
    etok, elp = osamp.sample(x, 1.0, -1, 0.95, 0.0, 21, ids, 5)
    assert torch.equal(tok, etok), int((tok != etok).sum())
    torch.testing.assert_close(lp, elp, atol=1e-4, rtol=1e-4)


def test_topp_fast_matches_oracle_small_batches(dev):
    """Both row-mode sizes (fewer rows than 256 use the split sampler on the two-kernel path;
    this kernel is one workgroup per row at any count) against oracle/sampler_ref.c."""
    from oracle import sampler as osamp

    V = 32000
    g = torch.Generator().manual_seed(4)
    for n, (temp, p, mp) in ((5, (1.0, 0.9, 0.0)), (300, (0.7, 0.8, 0.02)), (64, (1.0, 1.0, 0.2)), (7, (2.0, 0.3, 0.0))):
        x = (torch.randn(n, V, generator=g) * 2).to(torch.bfloat16)
        ids = torch.arange(n, dtype=torch.int64) + 100
        tok, lp, ff = _run(x.to(dev), True, temperature=temp, top_p=p, min_p=mp, seed=5, seq_ids=ids.to(dev), step=7)
        etok, elp = osamp.sample(x, temp, -1, p, mp, 5, ids, 7)
        assert int((ff[:, 2] == _ROW_DONE).sum()) == n
        assert torch.equal(tok, etok), (n, int((tok != etok).sum()))
        torch.testing.assert_close(lp, elp, atol=1e-4, rtol=1e-4)


def test_topp_fast_ranks_cut_key_ties_in_pass1(dev):
    """Rows on a coarse grid (values k/4): the top_p cut splits a tie group of tens to hundreds in
    most rows, and with the R-th-best race bar (sampler.hip SKYRL_TP_RBAR) pass 1 often records
    cut-key elements above e*, which it ranks by a scan of the row prefix (SKYRL_TP_TIERES) instead
    of leaving the row to pass 2: tokens bit-exact and logprobs against oracle/sampler_ref.c over
    three decode steps, and equal to the two-kernel path's."""
    from oracle import sampler as osamp

    V, n = 32000, 96
    g = torch.Generator().manual_seed(17)
    x = (torch.round(torch.randn(n, V, generator=g) * 12) / 4).to(torch.bfloat16)
    ids = torch.arange(n, dtype=torch.int64) * 7 + 3
    for step, (temp, p) in ((1, (1.0, 0.9)), (2, (1.0, 0.95)), (3, (0.6, 0.7))):
        tok, lp, ff = _run(x.to(dev), True, temperature=temp, top_p=p, seed=9, seq_ids=ids.to(dev), step=step)
        etok, elp = osamp.sample(x, temp, -1, p, 0.0, 9, ids, step)
        assert torch.equal(tok, etok), (step, int((tok != etok).sum()))
        torch.testing.assert_close(lp, elp, atol=1e-4, rtol=1e-4)
        assert bool(((ff[:, 2] == _ROW_DONE) | (ff[:, 2] == _ROW_FALLBACK)).all())
        _ab(x.to(dev), 0, temperature=temp, top_p=p, seed=9, seq_ids=ids.to(dev), step=step)


def test_minp_list_mode_overflow_and_ordinary_rows(dev):
    """min_p alone: pass 1 lists the elements within T |ln min_p| of the running max and decides
    from the list (sampler.hip SKYRL_MP_LIST). Rows with thousands of elements at the max overflow
    the list (2048) and take the in-row pass 2; rows whose max comes late in the row list many
    elements early; ordinary rows: tokens bit-exact and logprobs against oracle/sampler_ref.c."""
    from oracle import sampler as osamp

    V, n = 32000, 48
    g = torch.Generator().manual_seed(23)
    flat = torch.randint(0, 3, (8, V), generator=g).float()                 # a third of the row at the max
    late = torch.randn(8, V, generator=g) * 2
    late[:, -64:] += 9.0                                                      # the max in the last vectors
    ordinary = torch.randn(n - 16, V, generator=g) * 3
    x = torch.cat([flat, late, ordinary]).to(torch.bfloat16)
    ids = torch.arange(n, dtype=torch.int64) * 11 + 5
    for step, (temp, mp) in ((1, (1.0, 0.05)), (2, (0.6, 0.1)), (3, (1.5, 0.3))):
        tok, lp, ff = _run(x.to(dev), True, temperature=temp, min_p=mp, seed=13, seq_ids=ids.to(dev), step=step)
        etok, elp = osamp.sample(x, temp, -1, 1.0, mp, 13, ids, step)
        assert torch.equal(tok, etok), (step, int((tok != etok).sum()))
        torch.testing.assert_close(lp, elp, atol=1e-4, rtol=1e-4)
        assert bool((ff[:, 2] == _ROW_DONE).all())


def test_topp_fast_split_ties_and_fallback_rows(dev):
    """Rows built to take every branch: few distinct values (a tie group of ~25k at the cut: the
    fallback), rows -inf but for a handful of logits (taken: -inf weighs nothing), all-negative
    rows (taken: the cut in the negative window), rows with NaN / +inf / 2^16 (fallback),
    -2^16 (taken: weighs nothing), exact +-0 (their own counters) and values below 2^-16 (the
    short list; over 512 of them: fallback), and ordinary rows whose cut splits a tie group
    (taken: the cut key's elements ranked by index)."""
    from oracle import sampler as osamp

    V, k = 151936, 16
    g = torch.Generator().manual_seed(12)
    ties = torch.randint(0, 6, (k, V), generator=g).float()
    masked = torch.full((k, V), float("-inf"))
    masked.scatter_(1, torch.randint(0, V, (k, 20), generator=g), torch.randn(k, 20, generator=g) + 4)
    negative = -torch.rand(k, V, generator=g) * 5 - 0.5
    special = torch.randn(k, V, generator=g) * 3
    special[0, 5], special[1, 7], special[2, 9], special[3, 11] = float("nan"), float("inf"), 70000.0, -70000.0
    special[4, :30000] = 0.0  # +0 and -0 have their own counters
    special[4, 30000:31000] = -0.0
    special[5, :200] = 1e-7  # below the window: the short list
    special[6, :1000] = 1e-7  # too many for it: fallback
    ordinary = torch.randn(k, V, generator=g) * 3
    x = torch.cat([ties, masked, negative, special, ordinary]).to(torch.bfloat16)
    n = x.shape[0]
    ids = torch.arange(n, dtype=torch.int64)
    for p in (0.9, 0.95):
        tf, lf, done = _ab(x.to(dev), k * 3, temperature=1.0, top_p=p, seed=3, seq_ids=ids.to(dev), step=1)
        ok = ~torch.isnan(x.float()).any(-1)  # the oracle's NaN rows are garbage either way
        etok, _ = osamp.sample(x, 1.0, -1, p, 0.0, 3, ids, 1)
        assert torch.equal(tf[ok], etok[ok])
    _, _, ff = _run(x.to(dev), True, temperature=1.0, top_p=0.95, seed=3, seq_ids=ids.to(dev), step=1)
    assert bool((ff[:k, 2] == _ROW_FALLBACK).all())
    assert bool((ff[k:3 * k, 2] == _ROW_DONE).all()) and bool((ff[4 * k:, 2] == _ROW_DONE).all())
    assert bool((ff[3 * k:3 * k + 3, 2] == _ROW_FALLBACK).all()) and bool((ff[3 * k + 3:3 * k + 6, 2] == _ROW_DONE).all())
    assert int(ff[3 * k + 6, 2]) == _ROW_FALLBACK and bool((ff[3 * k + 7:4 * k, 2] == _ROW_DONE).all())


def test_minp_default_route_by_row_count(dev):
    """Default routing (sampler_topp_fast 1): min_p alone at 64 rows takes the two-kernel path
    (the RowFilter's state is the pre-pass's, not the one-pass kernel's done mark), at 256 rows the
    one-pass kernel; both give oracle/sampler_ref.c's tokens."""
    from oracle import sampler as osamp

    V = 32000
    g = torch.Generator().manual_seed(12)
    for n, one_pass in ((64, False), (256, True)):
        x = (torch.randn(n, V, generator=g) * 2).to(torch.bfloat16)
        ids = torch.arange(n, dtype=torch.int64) + 7
        tok, lp = ops.sample(x.to(dev), temperature=1.0, min_p=0.05, seed=3, seq_ids=ids.to(dev), step=5)
        torch.cuda.synchronize()
        ff = _filters(x.to(dev))
        assert bool((ff[:, 2] == _ROW_DONE).all()) == one_pass, n
        etok, elp = osamp.sample(x, 1.0, -1, 1.0, 0.05, 3, ids, 5)
        assert torch.equal(tok.cpu(), etok), (n, int((tok.cpu() != etok).sum()))
        torch.testing.assert_close(lp.cpu(), elp, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("V", [100, 517, 1000, 4097, 50257])
def test_topp_fast_small_and_ragged_vocab(dev, V):
    """Vocabularies with fewer elements than the workgroup has threads and ragged tails (16-B
    aligned rows: stride a multiple of 8)."""
    from oracle import sampler as osamp

    g = torch.Generator().manual_seed(V)
    n = 40
    width = (V + 7) // 8 * 8 + 8
    base = (torch.randn(n, width, generator=g) * 2).to(torch.bfloat16)
    x = base.to(dev)[:, :V]
    ids = torch.arange(n, dtype=torch.int64)
    for p, mp in ((0.9, 0.0), (1.0, 0.05), (0.7, 0.01)):
        tf, lf, _ = _ab(x, n, temperature=1.0, top_p=p, min_p=mp, seed=9, seq_ids=ids.to(dev), step=2)
        etok, elp = osamp.sample(base[:, :V].contiguous(), 1.0, -1, p, mp, 9, ids, 2)
        assert torch.equal(tf, etok)
        torch.testing.assert_close(lf, elp, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("V", [517, 4097, 50257, 151936])
def test_every_row_through_pass2(dev, V):
    """variant topp_probe = 5: no row decided in pass 1, so every row runs pass 2 (top_p: the
    second launch's 8 pieces, the ragged tail in the last piece; min_p: in the workgroup), against
    the two-kernel path and the oracle."""
    from oracle import sampler as osamp

    g = torch.Generator().manual_seed(V + 1)
    n = 24
    width = (V + 7) // 8 * 8 + 8
    base = (torch.randn(n, width, generator=g) * 3).to(torch.bfloat16)
    x = base.to(dev)[:, :V]
    ids = torch.arange(n, dtype=torch.int64)
    for p, mp in ((0.95, 0.0), (0.5, 0.0), (1.0, 0.05)):
        with ops.variant(topp_probe=5):
            tf, lf, ff = _run(x, True, temperature=1.0, top_p=p, min_p=mp, seed=4, seq_ids=ids.to(dev), step=9)
        ts, ls, fs = _run(x, False, temperature=1.0, top_p=p, min_p=mp, seed=4, seq_ids=ids.to(dev), step=9)
        assert torch.equal(tf, ts), (V, p, mp, int((tf != ts).sum()))
        assert torch.allclose(lf, ls, atol=2e-5, rtol=1e-5)
        assert bool((ff[:, 2] == _ROW_DONE).all()) and bool((ff[:, 1] == 0).all())
        if p < 1.0:
            assert torch.equal(ff[:, 3], fs[:, 3]) and torch.equal(ff[:, 4], fs[:, 4])
        etok, elp = osamp.sample(base[:, :V].contiguous(), 1.0, -1, p, mp, 4, ids, 9)
        assert torch.equal(tf, etok)
        torch.testing.assert_close(lf, elp, atol=1e-4, rtol=1e-4)



def test_pass2_state_across_batch_sizes(dev):
    """One cached workspace through top_p calls whose batch sizes change (the pass-2 state regions
    move with the batch size, and hold the previous calls' ties and states), with every row left
    to pass 2 (topp_probe 5) or the usual few: tokens equal the two-kernel path's each time."""
    V = 151936
    g = torch.Generator(device=dev).manual_seed(17)
    x = torch.empty((512, V), dtype=torch.bfloat16, device=dev).normal_(0, 3, generator=g)
    ids = torch.arange(512, dtype=torch.int64, device=dev)
    for k, (n, probe) in enumerate(((512, 5), (300, 0), (5, 5), (512, 0), (64, 5), (300, 5), (7, 0))):
        with ops.variant(topp_probe=probe):
            tf, lf, ff = _run(x[:n], True, temperature=1.0, top_p=0.9, seed=8, seq_ids=ids[:n], step=k)
        ts, ls, _ = _run(x[:n], False, temperature=1.0, top_p=0.9, seed=8, seq_ids=ids[:n], step=k)
        assert torch.equal(tf, ts), (n, probe, int((tf != ts).sum()))
        assert bool((ff[:, 2] == _ROW_DONE).all()), (n, probe)
