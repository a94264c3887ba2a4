"""a12–a14 collectives at world_size 2 over gloo on CPU (the RCCL path runs the same calls).

Checked against single-process restatements of the reference semantics:
  all_reduce_metrics        workers/worker_utils.py:25-35 + distributed/strategy.py:70-95
  sharded grad reduce +     FSDP2 reduce-scatter (mean) + clip_grad_norm_ + torch AdamW
  AdamW + bf16 all-gather   (fsdp_strategy.py:160-190,284-296, fsdp_utils.py:388-401)
  chunked weight broadcast  weight_sync/broadcast_strategy.py:98-191 (same names/shapes/bytes)
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from skyrl_amd import comm


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, world=2):
    port = _free_port()
    mp.spawn(_entry, args=(fn, world, port), nprocs=world, join=True)


def _entry(rank, fn, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world)
    finally:
        dist.destroy_process_group()


# --------------------------------------------------------------------------- a13
def _metrics_case(rank, world):
    m = {"policy_loss": 1.0 + rank, "clip_ratio": 0.25 * rank, "kl_max": 3.0 - rank, "ratio_min": 0.5 + rank,
         "ratio_max": -1.0 - rank}
    out = comm.all_reduce_metrics(m, device="cpu")
    assert list(out) == list(m)
    assert out["policy_loss"] == pytest.approx(1.5)
    assert out["clip_ratio"] == pytest.approx(0.125)
    assert out["kl_max"] == pytest.approx(3.0)
    assert out["ratio_min"] == pytest.approx(0.5)
    assert out["ratio_max"] == pytest.approx(-1.0)


def test_all_reduce_metrics_gloo():
    _run(_metrics_case)


def test_all_reduce_metrics_single_process_is_identity():
    assert comm.all_reduce_metrics({"a": 2, "b_max": 3}) == {"a": 2.0, "b_max": 3.0}


def _forced_solo_case(rank, world):
    """SKYRL_FORCE_COLLECTIVES=1 on a one-rank group: the exchanges run as collectives (the
    code path the N > 1 run takes) and give the world-1 result."""
    os.environ["SKYRL_FORCE_COLLECTIVES"] = "1"
    try:
        assert comm._collective(1)
        m = {"loss": 1.5, "r_min": -2.0, "r_max": 4.0}
        assert comm.all_reduce_metrics(m, device="cpu") == m
        red = comm.GradReducer(1000, "cpu", bucket_bytes=256 * 4)
        assert red.collective and red.grad_shard.data_ptr() != red.grad.data_ptr()
        red.grad.copy_(torch.arange(red.layout.padded, dtype=torch.float32))
        red.launch()
        red.wait()
        assert torch.equal(red.grad_shard, red.grad)  # one rank: the shard is the whole bucket
        net = _mlp(0)
        x = torch.randn(4, 12)
        net(x).sum().backward()
        before = [p.grad.clone() for p in net.parameters()]
        assert comm.allreduce_grads(net.parameters()) > 0
        assert all(torch.equal(a, p.grad) for a, p in zip(before, net.parameters()))
    finally:
        del os.environ["SKYRL_FORCE_COLLECTIVES"]
    assert not comm._collective(1)


def test_forced_collectives_one_rank_gloo():
    _run(_forced_solo_case, world=1)


# --------------------------------------------------------------------------- a12 layout
def test_flat_layout_pieces_cover_every_index_once():
    for numel, world, bucket in ((1000, 2, 256), (4097, 4, 1024), (64, 1, 1 << 20), (123457, 8, 5000)):
        lay = comm.FlatLayout(numel, world, bucket)
        assert lay.padded % (world * 64) == 0 and lay.padded >= numel
        allidx = torch.cat([lay.shard_index(r) for r in range(world)])
        assert allidx.numel() == lay.padded
        assert torch.equal(allidx.sort().values, torch.arange(lay.padded))
        for r in range(world):
            assert lay.shard_index(r).numel() == lay.shard_numel


def _adamw_ref(p, g, cfg, steps_grads):
    """Single-process reference: torch AdamW + clip_grad_norm_ on the DP-mean gradient."""
    w = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([w], lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                            foreach=False)
    norms = []
    for grad in steps_grads:
        w.grad = grad.clone()
        norms.append(float(torch.nn.utils.clip_grad_norm_([w], max_norm=cfg.max_grad_norm)))
        opt.step()
        opt.zero_grad()
    return w.detach(), norms


def _sharded_case(rank, world):
    torch.manual_seed(0)
    numel, n_micro = 5000, 2
    cfg = comm.AdamWConfig(lr=1e-2, max_grad_norm=0.5)
    p0 = torch.randn(numel)
    grads = [[torch.randn(numel) for _ in range(world)] for _ in range(3)]  # [step][rank], sums over micro-batches
    red = comm.GradReducer(numel, "cpu", bucket_bytes=1024 * 4)
    lay = red.layout
    assert len(lay.buckets) > 1
    idx = lay.shard_index(rank)
    flat = torch.zeros(lay.padded)
    flat[:numel] = p0
    p, m, v = flat[idx].clone(), torch.zeros(lay.shard_numel), torch.zeros(lay.shard_numel)
    norms = []
    for step, per_rank in enumerate(grads, start=1):
        red.grad[:numel] = per_rank[rank]
        red.launch()
        red.wait()
        # reduce-scatter result == SUM over ranks at this rank's indices
        full_sum = torch.zeros(lay.padded)
        full_sum[:numel] = sum(per_rank)
        assert torch.allclose(red.grad_shard, full_sum[idx], atol=1e-6)
        # sharded optimizer: norm via one scalar all-reduce, then the AdamW math on the shard
        scale = 1.0 / (n_micro * world)
        sumsq = (red.grad_shard.double() ** 2).sum().reshape(1)
        dist.all_reduce(sumsq)
        norm = float(sumsq.sqrt()) * scale
        norms.append(norm)
        coef = min(1.0, cfg.max_grad_norm / (norm + 1e-6))
        g = red.grad_shard * scale * coef
        b1, b2 = cfg.betas
        p.mul_(1 - cfg.lr * cfg.weight_decay)
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / (1 - b2 ** step) ** 0.5).add_(cfg.eps)
        p.addcdiv_(m, denom, value=-cfg.lr / (1 - b1 ** step))
        red.zero_grad()
    # all-gather the bf16 shard into the full rollout weights, as ShardedAdamW.sync_weights does
    full_bf16 = torch.empty(lay.padded, dtype=torch.bfloat16)
    shard_bf16 = p.to(torch.bfloat16)
    for b, (s, e) in enumerate(lay.buckets):
        po = lay.piece_off[b]
        n = (e - s) // world
        dist.all_gather_into_tensor(full_bf16[s:e], shard_bf16[po:po + n])
    ref, ref_norms = _adamw_ref(p0, None, cfg, [sum(pr) / (n_micro * world) for pr in grads])
    assert norms == pytest.approx(ref_norms, rel=1e-5)
    assert torch.allclose(full_bf16[:numel].float(), ref.to(torch.bfloat16).float(), atol=0, rtol=1e-2)
    assert torch.allclose(p, torch.cat([ref, torch.zeros(lay.padded - numel)])[idx], atol=1e-6, rtol=1e-5)


def test_sharded_grad_reduce_and_adamw_layout_gloo():
    _run(_sharded_case)


# --------------------------------------------------------------------------- a14
def _broadcast_case(rank, world):
    torch.manual_seed(1)
    named = [(f"layer{i}.weight", torch.randn(3 + i, 5).to(torch.bfloat16)) for i in range(6)]
    chunks = list(comm.pack_chunks(named, chunk_bytes=3 * 40 * 2))
    assert len(chunks) > 1 and sum(len(c) for c in chunks) == len(named)
    if rank == 0:
        sent = []
        n = comm.BroadcastWeightSender(src=0, on_request=sent.append).send_chunks(chunks)
        assert n == len(chunks) == len(sent)
    else:
        recv = comm.BroadcastWeightReceiver(torch.bfloat16, src=0, device="cpu")
        got = []
        for c in chunks:
            req = comm.WeightUpdateRequest(c.names, c.dtypes, c.shapes)
            got.extend(recv.receive_weights(req))
        assert [n for n, _ in got] == [n for n, _ in named]
        for (_, a), (_, b) in zip(got, named):
            assert torch.equal(a, b)  # bit-exact bf16


def test_chunked_weight_broadcast_gloo():
    _run(_broadcast_case)


def test_weight_update_request_validation():
    with pytest.raises(ValueError, match="same length"):
        comm.WeightUpdateRequest(["a"], [], [[1]])
    r = comm.WeightUpdateRequest(["a"], ["torch.bfloat16"], [[2, 3]])
    assert comm.WeightUpdateRequest.from_json_dict(r.to_json_dict()) == r


# --------------------------------------------------------------------------- a14 sharded sources
def _sharded_bcast_case(rank, world):
    learners = [0, 1]  # ranks 0, 1 learn; rank 2 is a rollout engine
    g = torch.Generator().manual_seed(0)
    named = [("model.embed_tokens.weight", torch.randn(37, 16, generator=g)),
             ("model.norm.weight", torch.randn(16, generator=g)),
             ("model.layers.0.mlp.up_proj.weight", torch.randn(48, 16, generator=g))]
    if rank in learners:
        req = comm.ShardedBroadcastWeightSender(learners).send(named)
        assert req.names == [n for n, _ in named]
    else:
        req = comm.WeightUpdateRequest([n for n, _ in named], ["torch.bfloat16"] * 3, [list(t.shape) for _, t in named])
        got = dict(comm.ShardedBroadcastWeightReceiver(learners, device="cpu").receive_weights(req))
        for n, t in named:
            assert torch.equal(got[n], t.to(torch.bfloat16)), n  # bit-exact bf16 copy


def test_sharded_source_weight_broadcast_gloo():
    _run(_sharded_bcast_case, world=3)


def _grad_allreduce_case(rank, world):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    x = torch.randn(6, 8, generator=torch.Generator().manual_seed(rank))
    m(x).pow(2).sum().backward()
    mine = [p.grad.clone() for p in m.parameters()]
    n = comm.allreduce_grads(m.parameters(), bucket_bytes=256)
    assert n >= 2  # several buckets
    # reference: the mean of every rank's gradient (recomputed locally for both ranks)
    ref = []
    for r in range(world):
        mm = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
        mm.load_state_dict(m.state_dict())
        mm(torch.randn(6, 8, generator=torch.Generator().manual_seed(r))).pow(2).sum().backward()
        ref.append([p.grad for p in mm.parameters()])
    for p, *gs in zip(m.parameters(), *ref):
        torch.testing.assert_close(p.grad, sum(gs) / world, rtol=1e-6, atol=1e-6)
    assert any(not torch.equal(a, p.grad) for a, p in zip(mine, m.parameters()))


def test_allreduce_grads_gloo():
    _run(_grad_allreduce_case)


# --------------------------------------------------------------------------- a12, overlapped
def _mlp(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32), torch.nn.Tanh(),
                               torch.nn.Linear(32, 5))


def _bucketed_case(rank, world):
    """BucketedGradAllReduce: buckets launched from the last micro-batch's backward hooks give
    the DP mean of the accumulated micro-batch gradients (FSDP2's reduce during backward)."""
    model = _mlp(0)
    ref = _mlp(0)
    sync = comm.BucketedGradAllReduce(model.parameters(), bucket_bytes=100 * 4)
    assert len(sync.buckets) >= 3
    g = torch.Generator().manual_seed(100 + rank)
    xs = [torch.randn(7, 12, generator=g) for _ in range(2)]
    for step in range(2):
        for k, x in enumerate(xs):
            if k == len(xs) - 1:
                sync.arm()
            (model(x * (step + 1)).square().mean() / len(xs)).backward()
            (ref(x * (step + 1)).square().mean() / len(xs)).backward()
        launched = sync.wait()
        assert launched == len(sync.buckets)  # every bucket went out from inside the backward
        for p, q in zip(model.parameters(), ref.parameters()):
            local = q.grad.clone()
            allg = [torch.empty_like(local) for _ in range(world)]
            dist.all_gather(allg, local)
            torch.testing.assert_close(p.grad, sum(allg) / world, atol=1e-6, rtol=1e-6)
        sync.zero_grad()
        for q in ref.parameters():
            q.grad = None


def test_bucketed_grad_allreduce_during_backward_gloo():
    _run(_bucketed_case)


def _bucketed_unused_case(rank, world):
    """A parameter no rank produced a gradient for ends with .grad None (AdamW skips it, as at
    world size 1); one that only rank 1 used is averaged on both; a .grad detached from its
    bucket raises instead of averaging stale buckets."""
    torch.manual_seed(0)
    used, only1, unused = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)
    params = list(used.parameters()) + list(only1.parameters()) + list(unused.parameters())
    sync = comm.BucketedGradAllReduce(params, bucket_bytes=16 * 4)
    x = torch.randn(3, 4, generator=torch.Generator().manual_seed(rank))
    sync.arm()
    y = used(x).sum() + (only1(x).sum() if rank == 1 else 0.0)
    y.backward()
    sync.wait()
    assert all(p.grad is not None for p in used.parameters())
    assert all(p.grad is not None for p in only1.parameters())  # rank 0 too: the mean is nonzero
    assert all(p.grad is None for p in unused.parameters())
    sync.zero_grad()  # views re-attached, zeroed
    assert all(p.grad is not None and not p.grad.any() for p in params)
    sync.arm()
    used(x).sum().backward()
    used.weight.grad = None  # detached (e.g. zero_grad(set_to_none=True))
    with pytest.raises(RuntimeError, match="bucket view"):
        sync.wait()


def test_bucketed_grad_allreduce_unused_and_detached_gloo():
    _run(_bucketed_unused_case)
