"""§8(f)1, tensor-parallel vocabulary: the lm_head-fused logprob/entropy with the vocab sharded
over ranks (reference: DistributedLogprob + vocab_parallel_entropy,
distributed/megatron/model_utils.py:64-136, 250-321, 548-590), and the logits-input
DistributedLogprob mirror.

* shard simulation in one process: each shard's states from the chunk kernel, merged by
  skyrl_lmhead_state_merge, must equal the fp32 oracle on exactly-representable logits (as
  test_gpu_lmhead.py), and the per-shard backward (dh summed over shards, dW concatenated)
  must equal the reference graph's gradients;
* two real ranks (gloo over the one GPU) through vocab_parallel_lmhead_logprobs_and_entropy:
  identical full-vocab outputs on both ranks, gradients as in the simulation;
* DistributedLogprob over bf16 logits shards vs torch log_softmax on the full logits.
"""

import os

import pytest
import torch

from skyrl_amd import _ffi
from skyrl_amd.lmhead import (_labels_flat, _merge, _shard_bwd, _shard_states, from_parallel_logits_to_logprobs,
                              lmhead_logprobs_and_entropy, vocab_parallel_lmhead_logprobs_and_entropy)
from test_gpu_lmhead import exact_inputs, reference

pytestmark = pytest.mark.gpu
T, H, V, CHUNK, TEMP = 64, 64, 5003, 512, 0.7
SPLITS = (0, 1700, 3400, V)  # three uneven shards, shard edges inside chunks of the unsharded run


def case():
    h, W, g = exact_inputs(T, H, V, seed=11)
    labels = torch.randint(0, V, (T,), generator=g)
    labels[:6] = torch.tensor([0, 1699, 1700, 3399, 3400, V - 1])  # first/last column of each shard
    return h, W, labels, torch.randn(T, generator=g), torch.randn(T, generator=g)


def assert_grads(dh, dw, e_dh, e_dw):
    for got, exp in ((dh.float().cpu(), e_dh), (dw.float().cpu(), e_dw)):
        scale = exp.abs().max().item()
        torch.testing.assert_close(got, exp, atol=2e-2 * scale, rtol=2e-2)
        assert (got - exp).norm() <= 1e-2 * exp.norm()


def test_vocab_shards_merge_to_the_oracle(dev):
    h, W, labels, g_lp, g_ent = case()
    e_lp, e_ent, e_dh, e_dw = reference(h, W, labels, TEMP, g_lp, g_ent)
    hd, Wd = h.to(dev), W.to(dev)
    lab, lstride = _labels_flat(labels.to(dev), T, dev)
    states = [_shard_states(hd, Wd[a:b], lab, lstride, a, TEMP, CHUNK)[: T * 16].view(torch.float32).view(T, 4)
              for a, b in zip(SPLITS[:-1], SPLITS[1:])]
    lp, ent, lse = _merge(torch.cat(states), len(states), T, True, dev)
    torch.testing.assert_close(lp.cpu(), e_lp, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ent.cpu(), e_ent, atol=1e-4, rtol=1e-5)
    # the label logit comes from exactly one shard: same as the unsharded fused kernel
    ulp, uent = lmhead_logprobs_and_entropy(hd, Wd, lab, TEMP, True, CHUNK)
    torch.testing.assert_close(lp, ulp, atol=1e-5, rtol=1e-5)
    dh = torch.zeros(T, H, device=dev)
    dws = []
    for a, b in zip(SPLITS[:-1], SPLITS[1:]):
        d_h, d_w = _shard_bwd(hd, Wd[a:b], lab, lstride, a, TEMP, CHUNK, lse, ent, g_lp.to(dev), g_ent.to(dev),
                              True, True)
        dh += d_h
        dws.append(d_w)
    assert_grads(dh, torch.cat(dws), e_dh, e_dw)


def test_single_shard_state_merge_equals_finalize(dev):
    """nstates = 1 (one rank) is the unsharded last-chunk finalize."""
    h, W, labels, _, _ = case()
    hd, Wd = h.to(dev), W.to(dev)
    lp, ent = vocab_parallel_lmhead_logprobs_and_entropy(hd, Wd, labels.to(dev), 0, None, TEMP, True, CHUNK)
    ulp, uent = lmhead_logprobs_and_entropy(hd, Wd, labels.to(dev), TEMP, True, CHUNK)
    torch.testing.assert_close(lp, ulp, atol=0, rtol=0)
    torch.testing.assert_close(ent, uent, atol=0, rtol=0)
    with pytest.raises(_ffi.SkyrlHipError):
        _ffi.call("skyrl_lmhead_state_merge", None, 0, 4, None, None, None, None)


def _rank(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    h, W, labels, g_lp, g_ent = case()
    bounds = [0, 2600, V]  # two uneven shards
    a, b = bounds[rank], bounds[rank + 1]
    hd = h.to(dev).requires_grad_(True)
    Wd = W[a:b].to(dev).requires_grad_(True)
    lp, ent = vocab_parallel_lmhead_logprobs_and_entropy(hd, Wd, labels.to(dev), a, dist.group.WORLD, TEMP, True,
                                                         CHUNK)
    (lp * g_lp.to(dev)).sum().add((ent * g_ent.to(dev)).sum()).backward()
    torch.save({"lp": lp.detach().cpu(), "ent": ent.detach().cpu(), "dh": hd.grad.float().cpu(),
                "dw": Wd.grad.float().cpu()}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_vocab_parallel(tmp_path):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    h, W, labels, g_lp, g_ent = case()
    e_lp, e_ent, e_dh, e_dw = reference(h, W, labels, TEMP, g_lp, g_ent)
    r0, r1 = (torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in (0, 1))
    for r in (r0, r1):
        torch.testing.assert_close(r["lp"], e_lp, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(r["ent"], e_ent, atol=1e-4, rtol=1e-5)
        assert torch.equal(r["dh"], r0["dh"])  # dh all-reduced: the same on every rank
    assert_grads(r0["dh"], torch.cat([r0["dw"], r1["dw"]]), e_dh, e_dw)


def test_distributed_logprob_over_logits_shards(dev):
    """from_parallel_logits_to_logprobs (one rank holding the whole vocab, and the merge over
    two shards simulated by hand) vs torch log_softmax of the full bf16 logits."""
    g = torch.Generator().manual_seed(5)
    B, S, Vt = 3, 40, 3001
    logits = (torch.randn(B, S, Vt, generator=g) * 3).to(torch.bfloat16).to(dev).requires_grad_(True)
    seq = torch.randint(0, Vt, (B, S), generator=g).to(dev)
    lp = from_parallel_logits_to_logprobs(logits, seq, 0, Vt, None)
    tgt = seq.roll(-1, dims=-1)
    ref_full = torch.log_softmax(logits.detach().float(), -1).gather(-1, tgt[..., None])[..., 0]
    torch.testing.assert_close(lp, ref_full[:, :-1], atol=2e-5, rtol=1e-5)
    gout = torch.randn(B, S - 1, generator=g).to(dev)
    (lp * gout).sum().backward()
    x = logits.detach().float().requires_grad_(True)
    (torch.log_softmax(x, -1).gather(-1, tgt[..., None])[..., :-1, 0] * gout).sum().backward()
    torch.testing.assert_close(logits.grad.float(), x.grad, atol=1e-2, rtol=1e-2)
    # two shards merged by hand through the same state path
    lab, lstride = _labels_flat(tgt, B * S, dev)
    z = logits.detach().view(B * S, Vt)
    sts = []
    for a, b in ((0, 1234), (1234, Vt)):
        st = torch.empty(_ffi.query("skyrl_lmhead_state_bytes", B * S), dtype=torch.uint8, device=dev)
        zs = z[:, a:b]
        _ffi.call("skyrl_lmhead_chunk_fwd", zs.data_ptr(), zs.stride(0), B * S, b - a, a, lab.data_ptr(), lstride,
                  1.0, st.data_ptr(), 1, 0, None, None, None, torch.cuda.current_stream(dev).cuda_stream)
        sts.append(st.view(torch.float32).view(B * S, 4))
    lp2, _, _ = _merge(torch.cat(sts), 2, B * S, False, dev)
    torch.testing.assert_close(lp2.view(B, S), ref_full, atol=2e-5, rtol=1e-5)
