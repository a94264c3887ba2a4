"""The multi-rank product path of a12/a14 on the GPU: 2 ranks on one MI355X over gloo (RCCL
refuses two ranks on one device; the 8-GPU RCCL run is the driver's).

  * GradReducer (bucketed SUM reduce-scatter on the comm stream) + ShardedAdamW.step(n_micro)
    (sharded norm via one scalar all-reduce, clip, non-finite skip, HIP AdamW writing the bf16
    shard) + sync_weights / wait_weights (per-bucket bf16 all-gather = the learner -> rollout
    weight sync) for 3 steps, against single-process torch AdamW + clip_grad_norm_ on the
    rank-mean gradient (fsdp_strategy.py:160-190,284-296; worker.py:909-914): parameters within
    1e-6, grad_norm within 1e-5 relative, the gathered bf16 weights bit-exact to the ranks'
    fp32 shards cast to bf16.
  * BucketedGradAllReduce on CUDA modules: bucket all-reduces launched on the comm stream from
    the last micro-batch's backward hooks give the DP mean gradient.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, fn, world, port):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world)
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    mp.spawn(_entry, args=(fn, world, _free_port()), nprocs=world, join=True)


def _sharded_adamw_case(rank, world):
    from skyrl_amd import comm

    dev = torch.device("cuda", 0)
    numel, n_micro, steps = 100_003, 2, 3
    cfg = comm.AdamWConfig(lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=0.05)
    p0 = torch.randn(numel, generator=torch.Generator().manual_seed(0))
    red = comm.GradReducer(numel, dev, bucket_bytes=64 << 10)
    lay = red.layout
    assert len(lay.buckets) >= 4 and red.world == world
    opt = comm.ShardedAdamW(red, p0.to(dev), cfg)
    torch.cuda.synchronize()
    assert torch.equal(opt.weights_bf16[:numel].cpu(), p0.to(torch.bfloat16))  # initial all-gather
    w = torch.nn.Parameter(p0.clone())
    topt = torch.optim.AdamW([w], lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay)
    idx = lay.shard_index(rank)
    for step in range(steps):
        grads = [torch.randn(numel, generator=torch.Generator().manual_seed(1000 * step + r)) * (r + 1) * 0.01
                 for r in range(world)]  # each rank's sum over its micro-batches
        red.grad[:numel] = grads[rank].to(dev)
        red.launch()
        gn = float(opt.step(n_micro=n_micro).item())
        opt.sync_weights()
        opt.wait_weights()
        torch.cuda.synchronize()
        # reference: DP mean (FSDP reduce-scatter mean) x 1/n_micro, clip, AdamW
        w.grad = sum(grads) / (world * n_micro)
        gn_ref = float(torch.nn.utils.clip_grad_norm_([w], max_norm=cfg.max_grad_norm))
        topt.step()
        topt.zero_grad()
        assert gn == pytest.approx(gn_ref, rel=1e-5), (step, gn, gn_ref)
        assert gn_ref > cfg.max_grad_norm  # the clip path is exercised
        ref_pad = torch.zeros(lay.padded)
        ref_pad[:numel] = w.detach()
        torch.testing.assert_close(opt.param.cpu(), ref_pad[idx], atol=1e-6, rtol=1e-5)
        # the gathered rollout weights are exactly every rank's fp32 shard cast to bf16
        shards = [torch.empty_like(opt.param) for _ in range(world)]
        dist.all_gather(shards, opt.param)
        full = torch.zeros(lay.padded)
        for r in range(world):
            full[lay.shard_index(r)] = shards[r].cpu()
        assert torch.equal(opt.weights_bf16.cpu(), full.to(torch.bfloat16)), step
    assert int(opt.step_count.item()) == steps


def test_sharded_adamw_two_ranks_one_gpu():
    _run(_sharded_adamw_case)


def _bucketed_cuda_case(rank, world):
    from skyrl_amd import comm

    dev = torch.device("cuda", 0)

    def mlp():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 256),
                                   torch.nn.GELU(), torch.nn.Linear(256, 16)).to(dev)

    model, ref = mlp(), mlp()
    sync = comm.BucketedGradAllReduce(model.parameters(), bucket_bytes=8 << 10)
    assert len(sync.buckets) >= 3 and sync.stream is not None
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    xs = [torch.randn(33, 64, device=dev, generator=g) for _ in range(3)]
    for k, x in enumerate(xs):
        if k == len(xs) - 1:
            sync.arm()
        (model(x).square().mean() / len(xs)).backward()
        (ref(x).square().mean() / len(xs)).backward()
    assert sync.wait() == len(sync.buckets)
    for p, q in zip(model.parameters(), ref.parameters()):
        allg = [torch.empty_like(q.grad) for _ in range(world)]
        dist.all_gather(allg, q.grad)
        torch.testing.assert_close(p.grad, sum(allg) / world, atol=1e-6, rtol=1e-5)


def test_bucketed_grad_allreduce_two_ranks_one_gpu():
    _run(_bucketed_cuda_case)
