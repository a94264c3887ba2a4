"""Where the bench's AdamW time goes (8.78 ms in one run, 10.45 in another).
The bench's optimizer (ShardedAdamW over Qwen2.5-1.5B's 1,543,714,304 parameters, one rank) is
timed per step with HIP events, and its kernels one by one, in three settings: alone; after the
bench's resident-logits allocation (most of HBM taken, as in bench.py); and right after a burst of
streaming reads (the step's training passes before it). One JSON line; run it under rocprofv3
--kernel-trace --stats for the kernels' own durations."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import comm  # noqa: E402
from skyrl_amd.ops import _ffi, _ptr  # noqa: E402

P = 1543714304


def timed(fn, reps=5, before=None):
    out = []
    for _ in range(reps):
        if before is not None:
            before()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(round(a.elapsed_time(b), 3))
    return out


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    reducer = comm.GradReducer(P, dev, bucket_bytes=256 << 20)
    init = torch.empty(P, dtype=torch.float32, device=dev).normal_(0.0, 0.02)
    opt = comm.ShardedAdamW(reducer, init, comm.AdamWConfig())
    del init
    reducer.grad.normal_(0.0, 1e-3)
    torch.cuda.synchronize()
    g = reducer.grad_shard
    s = torch.cuda.current_stream().cuda_stream
    step = lambda: opt.step(n_micro=32, zero_grad=False)  # noqa: E731
    sumsq = lambda: _ffi.call("skyrl_sumsq", _ptr(g), g.numel(), _ptr(opt.sumsq), _ptr(opt._ws), s)  # noqa: E731
    res = {"params": P}
    step()
    torch.cuda.synchronize()
    res["alone_step_ms"] = timed(step)
    res["alone_sumsq_ms"] = timed(sumsq)
    # the bench's resident logits: most of the free HBM in 8-GiB pieces
    free, _ = torch.cuda.mem_get_info(dev)
    hold = []
    left = free - (12 << 30)
    while left > (8 << 30):
        hold.append(torch.empty(8 << 30, dtype=torch.uint8, device=dev))
        left -= 8 << 30
    res["held_GiB"] = len(hold) * 8
    res["after_alloc_step_ms"] = timed(step)
    # right after ~40 ms of streaming reads of the held memory (the training passes' pattern)
    src = hold[0].view(torch.float32) if hold else torch.empty(1 << 30, dtype=torch.float32, device=dev)
    acc = torch.empty(1, dtype=torch.float32, device=dev)

    def burst():
        for _ in range(8):
            torch.sum(src, 0, out=acc)
    res["after_burst_step_ms"] = timed(step, before=burst)
    del hold
    torch.cuda.synchronize()
    res["after_free_step_ms"] = timed(step)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
