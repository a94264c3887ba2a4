"""Sweep a fixed-chunk split for the paged decode kernel: part_min = C tokens, nparts =
ceil(max_ctx / C), so a sequence gets ceil(ctx / C)-ish waves (work-proportional) instead of
every sequence being cut into the same number of parts. Ragged U[17,1536] and uniform contexts
at the rollout head shape (12 q / 2 kv heads, D=128). Probe only: one JSON line per point."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from skyrl_amd.inference_engines import kernels  # noqa: E402

NH, NKV, D, BS = 12, 2, 128, 16


def setup(dev, nseq, ctx_lo, ctx_hi, seed=11):
    g = torch.Generator(device=dev).manual_seed(seed)
    ctx = torch.randint(ctx_lo, ctx_hi + 1, (nseq,), device=dev, generator=g, dtype=torch.int32)
    nb = (ctx + BS - 1) // BS
    max_ctx = int(ctx.max())
    width = (max_ctx + BS - 1) // BS
    nblk = int(nb.sum())
    kc = torch.randn(nblk, NKV, BS, D, device=dev, generator=g).to(torch.bfloat16)
    vc = torch.randn(nblk, NKV, D, BS, device=dev, generator=g).to(torch.bfloat16)
    perm = torch.randperm(nblk, device=dev, generator=g).int()
    bt = torch.zeros(nseq, width, dtype=torch.int32, device=dev)
    starts = torch.cumsum(nb, 0) - nb
    col = torch.arange(width, device=dev)
    live = col[None] < nb[:, None]
    bt[live] = perm[(starts[:, None] + col[None])[live]]
    q = torch.randn(nseq, NH, D, device=dev, generator=g).to(torch.bfloat16)
    return q, kc, vc, bt, ctx, max_ctx


def time_it(dev, args, nparts, part_min, reps=50):
    q, kc, vc, bt, ctx, max_ctx = args
    out = torch.empty_like(q)
    ws = kernels.DecodeWorkspace(dev)
    run = lambda: kernels.paged_decode(q, kc, vc, bt, ctx, max_ctx, 1 / math.sqrt(D), out=out,  # noqa: E731
                                       workspace=ws, nparts=nparts, part_min=part_min)
    run()
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        run()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    nbytes = int(ctx.sum()) * NKV * D * 4 + 2 * q.shape[0] * NH * D * 2
    return us, nbytes / (us * 1e-6) / 1e9, out.clone()


def main():
    dev = torch.device("cuda:0")
    cases = [(512, 17, 1536), (256, 17, 1536), (1024, 17, 1536), (512, 1280, 1280), (128, 17, 1536),
             (64, 17, 1536)]
    for nseq, lo, hi in cases:
        args = setup(dev, nseq, lo, hi)
        max_ctx = args[5]
        base = kernels.choose_nparts(nseq, NKV, max_ctx)
        us, gbs, ref = time_it(dev, args, base, kernels.MIN_PARTITION)
        print(json.dumps({"nseq": nseq, "ctx": f"U[{lo},{hi}]", "mode": "default", "nparts": base,
                          "us": round(us, 2), "GBps": round(gbs, 1)}), flush=True)
        for chunk in (128, 192, 256, 320, 384, 512, 768):
            np_ = math.ceil(max_ctx / chunk)
            us, gbs, o = time_it(dev, args, np_, chunk)
            err = float((o.float() - ref.float()).abs().max())
            print(json.dumps({"nseq": nseq, "ctx": f"U[{lo},{hi}]", "mode": "chunk", "chunk": chunk,
                              "nparts": np_, "us": round(us, 2), "GBps": round(gbs, 1),
                              "max_abs_diff_vs_default": err}), flush=True)


if __name__ == "__main__":
    main()
