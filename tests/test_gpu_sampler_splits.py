"""a1 sampling at the per-rank batch sizes of a strong-scaling job (512 / N rows: 256, 128, 64 at
N = 2, 4, 8; the engine's shrinking decode batches too): rows split over workgroups whose last
arriver folds the partials (sc1 records, drained before the ticket; arrive.h),
against oracle/sampler_ref.c (tokens bit-exact, logprobs 1e-4) and against the same rows decided
by one workgroup per row (tokens identical: every split decides with exact scores, the lowest
index on ties). The split count follows the variant field sampler_split_wgs and the row threshold
sampler_split_rows, the split workgroup size sampler_split_nt; every setting must give the same
tokens (T = 1 runs the multiplicative bound in row mode and the additive one in split mode).
The merging workgroup takes one agent acquire before it loads the records (arrive.h)."""

import pytest
import torch

from skyrl_amd import ops

pytestmark = pytest.mark.gpu

V = 151936


def _knobs(rows=256, wgs=1024, gran=8192, nt=256):
    """The calls' kernel variant (skyrl_variant through ops.variant, per call)."""
    return ops.variant(sampler_split_nt=nt, sampler_split_rows=rows, sampler_split_wgs=wgs, sampler_split_gran=gran)


@pytest.mark.parametrize("n", [1, 13, 64, 128, 255])
@pytest.mark.parametrize("temp", [1.0, 0.7, 0.0])
@pytest.mark.parametrize("kernel", ["split256", "split512"])
def test_split_rows_match_oracle(dev, n, temp, kernel):
    from oracle import sampler as osamp

    g = torch.Generator().manual_seed(n * 10 + int(temp * 10))
    x = (torch.randn(n, V, generator=g) * 3).to(torch.bfloat16)
    ids = torch.arange(n, dtype=torch.int64) * 7 + 3
    with _knobs(nt=int(kernel[5:])):
        tok, lp = ops.sample(x.to(dev), temperature=temp, seed=9, seq_ids=ids.to(dev), step=11)
    etok, elp = osamp.sample(x, temp, -1, 1.0, 0.0, 9, ids, 11)
    assert torch.equal(tok.cpu(), etok), int((tok.cpu() != etok).sum())
    torch.testing.assert_close(lp.cpu(), elp, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("n", [1, 7, 64, 100, 192, 256, 300])
def test_split_settings_give_identical_tokens(dev, n):
    """Row-per-workgroup (threshold 1), the default split policy, and other split counts on the
    same rows, in a strided view of a larger resident tensor (the bench's layout)."""
    g = torch.Generator(device=dev).manual_seed(n)
    big = torch.empty((n, 3, V), dtype=torch.bfloat16, device=dev).normal_(0, 3, generator=g)
    x = big[:, 1]  # row stride 3 V
    ids = torch.arange(n, dtype=torch.int64, device=dev) + 1000
    outs = {}
    for rows, wgs, gran, nt in (
            (1, 2048, 8192, 256), (256, 2048, 8192, 256), (1024, 2048, 8192, 256), (1024, 512, 8192, 256),
            (1024, 8192, 8192, 256), (1024, 1024, 2048, 256), (1024, 8192, 2048, 256), (1024, 960, 4096, 256),
            (1024, 256, 16384, 512), (1024, 2048, 2048, 512), (256, 1024, 8192, 256), (256, 64, 8192, 256)):
        with _knobs(rows, wgs, gran, nt):
            for temp in (1.0, 0.0, 1.3):
                tok, lp = ops.sample(x, temperature=temp, seed=2, seq_ids=ids, step=5)
                outs.setdefault(temp, []).append((tok.clone(), lp.clone()))
    for temp, res in outs.items():
        for tok, lp in res[1:]:
            assert torch.equal(tok, res[0][0]), (n, temp)
            torch.testing.assert_close(lp, res[0][1], atol=1e-5, rtol=1e-5)


def test_split_workspace_reused_across_sizes_and_settings(dev):
    """One cached workspace through calls whose split counts change with the batch size and the
    knobs (the counters re-armed by every last arriver): tokens equal fresh single calls."""
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.empty((300, V), dtype=torch.bfloat16, device=dev).normal_(0, 3, generator=g)
    ids = torch.arange(300, dtype=torch.int64, device=dev)
    seq = [(64, 2048), (200, 2048), (7, 512), (300, 2048), (128, 8192), (64, 1024), (255, 2048), (33, 2048),
           (300, 512)]
    for k, (n, wgs) in enumerate(seq):
        with _knobs(1024, wgs):
            tok, _ = ops.sample(x[:n], temperature=1.0, seed=3, seq_ids=ids[:n], step=k)
        with _knobs(1, 2048):  # one workgroup per row: no counters
            ref, _ = ops.sample(x[:n], temperature=1.0, seed=3, seq_ids=ids[:n], step=k)
        assert torch.equal(tok, ref), (n, wgs)
