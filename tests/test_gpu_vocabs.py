"""Every BASELINE.json configuration's vocabulary through the sampler (a1), the logprob/entropy
kernels (a2/a3) and the fused training pass (a2+a3+a6+a7) against the oracle:

  GPT-2-small      V =  50,257  (config 1; odd V: misaligned rows, the split kernel's EDGE form)
  Llama-3-8B       V = 128,256  (config 4; resident kernel, 16 vectors per thread)
  Qwen2.5-1.5B     V = 151,936  (config 2; resident kernel, 19 vectors per thread)
  Qwen2.5-7B       V = 152,064  (configs 3 and 5)

Tokens bit-exact vs oracle/sampler_ref.c; logprobs/entropy 1e-4 vs the fp32 oracle; the
training pass's loss/metrics vs the oracle's loss assembly (1e-4) and its bf16 dlogits vs
torch-CPU autograd of the reference formulas (bf16 resolution); register-resident vs
two-sweep kernels identical.
"""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import ops, ppo_utils
from skyrl_amd.config import AlgorithmConfig

pytestmark = pytest.mark.gpu

VOCABS = [50257, 128256, 151936, 152064]


def close(a, b, atol=1e-5, rtol=1e-5):
    torch.testing.assert_close(torch.as_tensor(a).detach().float().cpu(), torch.as_tensor(b).detach().float().cpu(),
                               atol=atol, rtol=rtol)


@pytest.mark.parametrize("V", VOCABS)
@pytest.mark.parametrize("cfg", [(1.0, -1, 1.0, 0.0), (0.7, -1, 1.0, 0.0), (0.0, -1, 1.0, 0.0), (1.0, 50, 0.9, 0.0),
                                 (0.9, -1, 0.95, 0.02)])
def test_sampler_bit_exact_per_vocab(dev, V, cfg):
    from oracle import sampler as osamp

    temp, top_k, top_p, min_p = cfg
    g = torch.Generator().manual_seed(V % 1000)
    for n in (6, 300):  # split mode and one-workgroup-per-row mode
        full = (torch.randn(n, 2, V, generator=g) * 3).to(torch.bfloat16)
        x = full.to(dev)[:, 1]  # decode-loop layout: a strided row view
        ids = torch.arange(n, dtype=torch.int64) * 3 + 1
        tok, lp = ops.sample(x, temperature=temp, top_k=top_k, top_p=top_p, min_p=min_p, seed=77,
                             seq_ids=ids.to(dev), step=9)
        etok, elp = osamp.sample(full[:, 1].contiguous(), temp, top_k, top_p, min_p, 77, ids, 9)
        assert torch.equal(tok.cpu(), etok), (V, n, cfg)
        close(lp, elp, atol=1e-4)


def test_sampler_workspace_reused_across_batch_sizes(dev):
    """One cached sampler workspace serves calls of any batch size (the engine's decode batches
    grow and shrink): split-mode calls after calls with fewer or more rows, with and without the
    filter pre-pass, keep the oracle's tokens (the arrival counters sit in a fixed region that no
    other call's filters or partials overlap)."""
    from oracle import sampler as osamp

    V = 4100
    g = torch.Generator().manual_seed(4100)
    for step, (n, top_p) in enumerate([(6, 0.9), (200, 1.0), (3, 1.0), (130, 0.8), (300, 1.0), (64, 1.0)]):
        x = (torch.randn(n, V, generator=g) * 3).to(torch.bfloat16)
        ids = torch.arange(n, dtype=torch.int64) + 1
        tok, lp = ops.sample(x.to(dev), temperature=1.0, top_p=top_p, seed=21, seq_ids=ids.to(dev), step=step)
        etok, elp = osamp.sample(x, 1.0, -1, top_p, 0.0, 21, ids, step)
        assert torch.equal(tok.cpu(), etok), (n, top_p)
        close(lp, elp, atol=1e-4)


@pytest.mark.parametrize("V", VOCABS)
def test_logprob_entropy_per_vocab(dev, V):
    """The model-wrapper slice logits[:, -R-1:-1] of [n, S, V] (model_wrapper.py:370), fwd + bwd."""
    g = torch.Generator().manual_seed(V % 997)
    n, S, R = 2, 13, 8
    logits = (torch.randn(n, S, V, generator=g) * 3).to(torch.bfloat16)
    seq = torch.randint(0, V, (n, S), generator=g)
    x = logits.to(dev)[:, -R - 1:-1].detach().requires_grad_(True)
    lp, ent = ops.logprobs_and_entropy(x, seq.to(dev)[:, -R:], 1.0, compute_entropy=True)
    xc = logits[:, -R - 1:-1].float().requires_grad_(True)
    lpc = cpu_ref.logprobs_from_logits(xc, seq[:, -R:])
    entc = cpu_ref.entropy_from_logits(xc)
    close(lp, lpc, atol=1e-4)
    close(ent, entc, atol=1e-4)
    w1 = torch.randn(n, R, generator=g)
    w2 = torch.randn(n, R, generator=g) * 0.1
    ((lp * w1.to(dev)).sum() + (ent * w2.to(dev)).sum()).backward()
    ((lpc * w1).sum() + (entc * w2).sum()).backward()
    close(x.grad, xc.grad, atol=2e-4, rtol=1e-2)  # bf16 dlogits


@pytest.mark.parametrize("V", VOCABS)
@pytest.mark.parametrize("temp", [1.0, 0.7])
def test_policy_train_per_vocab(dev, V, temp):
    """Fused training pass on the [:, -R-1:-1] slice (GPT-2: misaligned rows): the default
    kernel (split rows where the layout allows, else resident) vs the resident and the
    two-sweep kernels, and vs torch-CPU autograd of the oracle's loss assembly."""
    g = torch.Generator().manual_seed(V % 991)
    n, S, R = 2, 11, 6
    logits = (torch.randn(n, S, V, generator=g) * 3).to(torch.bfloat16)
    seq = torch.randint(0, V, (n, S), generator=g)
    labels = seq[:, -R:]
    mask = torch.tensor([[1.0] * R, [1.0] * 4 + [0.0] * (R - 4)])
    lp0 = cpu_ref.logprobs_from_logits(logits[:, -R - 1:-1], labels, temperature=temp)
    old = lp0 + 0.2 * torch.randn(n, R, generator=g)
    ref = lp0 + 0.1 * torch.randn(n, R, generator=g)
    adv = torch.randn(n, R, generator=g)
    cfg = AlgorithmConfig(use_entropy_loss=True, policy_loss_type="dual_clip", clip_ratio_c=1.5)
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=True, has_entropy=True)
    outs = []
    for split, resident in ((1, 1), (0, 1), (0, 0)):
        with ops.variant(train_split=split, train_resident=resident):
            full = logits.to(dev).requires_grad_(True)
            x = full[:, -R - 1:-1]
            loss, m, lp, ent = ops.policy_train(x, labels.to(dev), old.to(dev), adv.to(dev), mask.to(dev), params,
                                                ref_log_probs=ref.to(dev), temperature=temp)
            (loss * 1.5).backward()
        outs.append((loss.detach(), m.clone(), lp, ent, full.grad))
    for a, b in zip(outs[1], outs[2]):  # resident vs two-sweep: the same per-thread order
        close(a, b, atol=1e-6, rtol=1e-5)
    # split vs resident: another softmax summation order (fp32), dlogits within a bf16 rounding
    for a, b in zip(outs[0][:4], outs[1][:4]):
        close(a, b, atol=1e-5, rtol=1e-5)
    close(outs[0][4], outs[1][4], atol=2e-6, rtol=1e-2)
    assert float(outs[0][1][6]) == 0.0  # no split-exchange timeout
    loss, m, lp, ent, grad = outs[0]
    assert torch.count_nonzero(grad[:, :S - R - 1]) == 0 and torch.count_nonzero(grad[:, -1]) == 0
    # the reference divides the bf16 logits by T in place (model_wrapper.py:314), then the fp32 path
    sl = logits[:, -R - 1:-1]
    xs = (sl / temp if temp != 1.0 else sl).float().requires_grad_(True)
    lpc = cpu_ref.logprobs_from_logits(xs, labels)
    entc = cpu_ref.entropy_from_logits(xs)
    final, mc = cpu_ref.policy_loss_assembly(lpc, old, adv, mask, ref, entc, use_entropy_loss=True, dual_clip=True,
                                             clip_c=1.5)
    (final * 1.5).backward()
    close(loss, final, atol=1e-5, rtol=1e-4)
    close(lp, lpc, atol=1e-4)
    close(ent, entc, atol=1e-4)
    close(m[4], mc["clip_ratio"], atol=1e-6)
    close(grad[:, -R - 1:-1], xs.grad / temp, atol=2e-6, rtol=1e-2)  # d(x/T)/dx = 1/T; dlogits in bf16

