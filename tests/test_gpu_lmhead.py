"""§8(f)1 lm_head-fused logprob + entropy vs the oracle.

The exact case builds hidden states and weights whose logits every GEMM computes exactly:
sparse hidden rows, with dyadic values of a few bits. The chunked-GEMM path can then be held
to the fp32 oracle (cpu_ref) at 1e-5 on logp/entropy, for any GEMM kernel and accumulation
order. Gradients are checked against torch-CPU autograd of the reference's bf16 graph:
logits bf16 -> div_(T) -> fp32 logprob/entropy. That graph rounds dlogits to bf16, and the
two lm_head backward GEMMs are then applied to it.
"""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import ops
from skyrl_amd.lmhead import default_chunk, lmhead_logprobs_and_entropy

pytestmark = pytest.mark.gpu


def exact_inputs(T, H, V, seed, nnz=4):
    g = torch.Generator().manual_seed(seed)
    h = torch.zeros(T, H)
    cols = torch.stack([torch.randperm(H, generator=g)[:nnz] for _ in range(T)])
    vals = torch.tensor([-2.0, -1.0, -0.5, 0.5, 1.0, 2.0])[torch.randint(0, 6, (T, nnz), generator=g)]
    h.scatter_(1, cols, vals)
    W = torch.randint(-4, 5, (V, H), generator=g).float() * 0.25
    return h.to(torch.bfloat16), W.to(torch.bfloat16), g


def reference(h, W, labels, temperature, g_lp, g_ent):
    """Reference graph on CPU: bf16 logits (exact here), in-dtype /T, fp32 logprob/entropy,
    bf16 dlogits, then the lm_head backward GEMMs in fp32."""
    z = (h.float() @ W.float().t()).to(torch.bfloat16).requires_grad_(True)
    x = z / temperature if temperature != 1.0 else z
    lp = cpu_ref.logprobs_from_logits(x, labels)
    ent = cpu_ref.entropy_from_logits(x)
    (lp * g_lp).sum().add((ent * g_ent).sum()).backward()
    dz = z.grad.float()
    return lp.detach(), ent.detach(), dz @ W.float(), dz.t() @ h.float()


@pytest.mark.parametrize("T,H,V,chunk,temperature", [
    (64, 64, 5003, 1024, 1.0),     # 5 chunks, ragged last chunk (5003 % 8 != 0)
    (37, 96, 4096, 4096, 0.7),     # one chunk (no state), temperature in bf16
    (128, 64, 3000, 512, 1.3),     # many chunks
])
def test_lmhead_exact_vs_oracle(dev, T, H, V, chunk, temperature):
    h, W, g = exact_inputs(T, H, V, seed=T + V)
    labels = torch.randint(0, V, (T,), generator=g)
    labels[0], labels[1], labels[2] = 0, V - 1, min(chunk, V - 1)  # first / last column, chunk edge
    g_lp = torch.randn(T, generator=g)
    g_ent = torch.randn(T, generator=g)
    e_lp, e_ent, e_dh, e_dw = reference(h, W, labels, temperature, g_lp, g_ent)

    hd = h.to(dev).requires_grad_(True)
    Wd = W.to(dev).requires_grad_(True)
    lp, ent = lmhead_logprobs_and_entropy(hd, Wd, labels.to(dev), temperature, True, chunk)
    torch.testing.assert_close(lp.cpu(), e_lp, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ent.cpu(), e_ent, atol=1e-4, rtol=1e-5)
    (lp * g_lp.to(dev)).sum().add((ent * g_ent.to(dev)).sum()).backward()
    # dlogits are bf16 on both sides (an ulp apart at rounding ties); the GEMMs accumulate fp32
    for got, exp in ((hd.grad.float().cpu(), e_dh), (Wd.grad.float().cpu(), e_dw)):
        scale = exp.abs().max().item()
        torch.testing.assert_close(got, exp, atol=2e-2 * scale, rtol=2e-2)
        assert (got - exp).norm() <= 1e-2 * exp.norm()


def test_lmhead_matches_unfused_kernels_dense(dev):
    """Dense random inputs through hipBLASLt: fused vs the unfused logprob kernel on the full
    logits from one GEMM. Chunked and whole-V GEMMs may round a logit differently by one bf16
    ulp, so the bound is the ulp of the largest logit, and the mean error is ~1e-6."""
    g = torch.Generator().manual_seed(7)
    T, H, V = 512, 256, 20011
    h = (torch.randn(T, H, generator=g)).to(torch.bfloat16).to(dev)
    W = (torch.randn(V, H, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    lab2d = torch.randint(0, V, (4, 2 * T // 4), generator=g).to(dev)
    labels = lab2d[:, ::2]  # non-unit stride, shape [4, T/4]
    hh = h.view(4, T // 4, H)
    lp, ent = lmhead_logprobs_and_entropy(hh, W, labels, 1.0, True, 4096)
    z = torch.mm(h, W.t()).view(4, T // 4, V)
    elp, eent = ops.logprobs_and_entropy(z, labels, 1.0)
    ulp = 2.0 ** (torch.floor(torch.log2(z.float().abs().max())) - 7)
    assert lp.shape == labels.shape and ent.shape == labels.shape
    assert (lp - elp).abs().max() <= 2 * ulp
    assert (lp - elp).abs().mean() < 1e-3
    assert (ent - eent).abs().max() < 1e-2


def test_lmhead_no_entropy_and_grad_only_hidden(dev):
    h, W, g = exact_inputs(50, 32, 2500, seed=3)
    labels = torch.randint(0, 2500, (50,), generator=g)
    e_lp, _, e_dh, _ = reference(h, W, labels, 1.0, torch.ones(50), torch.zeros(50))
    hd = h.to(dev).requires_grad_(True)
    lp, ent = lmhead_logprobs_and_entropy(hd, W.to(dev), labels.to(dev), 1.0, False, 1000)
    assert ent is None
    torch.testing.assert_close(lp.cpu(), e_lp, atol=1e-5, rtol=1e-5)
    lp.sum().backward()
    assert (hd.grad.float().cpu() - e_dh).norm() <= 1e-2 * e_dh.norm()


def test_lmhead_empty_and_errors(dev):
    W = torch.zeros(100, 16, dtype=torch.bfloat16, device=dev)
    lp, ent = lmhead_logprobs_and_entropy(torch.zeros(0, 16, dtype=torch.bfloat16, device=dev), W,
                                          torch.zeros(0, dtype=torch.int64, device=dev))
    assert lp.numel() == 0 and ent.numel() == 0
    with pytest.raises(TypeError):
        lmhead_logprobs_and_entropy(torch.zeros(4, 16, device=dev), W, torch.zeros(4, dtype=torch.int64, device=dev))
    with pytest.raises(ValueError):
        lmhead_logprobs_and_entropy(torch.zeros(4, 8, dtype=torch.bfloat16, device=dev), W,
                                    torch.zeros(4, dtype=torch.int64, device=dev))


def test_default_chunk_fits_mall():
    assert default_chunk(8192, 151936) * 8192 * 2 <= 256 << 20
    assert default_chunk(16, 1000) == 1000
