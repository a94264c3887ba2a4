"""A/B of the paged decode kernel's K/V prefetch depth (skyrl_variant "attn_pf": blocks in flight per wave).

Times the decode kernel (Qwen2.5-1.5B heads: 12 q / 2 kv, D = 128) with the knob
interleaved over depths, on ragged U[17,1536] and uniform contexts, and checks every depth gives
bit-identical outputs (the depth only changes when loads are issued). Probe only; prints one JSON line per measurement."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from skyrl_amd import _ffi  # noqa: E402
from skyrl_amd.inference_engines import kernels  # noqa: E402


PFS = (4, 6, 8)  # 3 was measured too (126 us at 512 ragged: it spills); dropped from the knob


def same_outputs(dev):
    nh, nkv, D, BS, nseq = 12, 2, 128, 16, 256
    g = torch.Generator(device=dev).manual_seed(5)
    ctx = torch.randint(17, 1537, (nseq,), device=dev, generator=g, dtype=torch.int32)
    nb = (ctx + BS - 1) // BS
    width = int(nb.max())
    nblk = int(nb.sum())
    kc = torch.randn(nblk, nkv, BS, D, device=dev, generator=g).to(torch.bfloat16)
    vc = torch.randn(nblk, nkv, D, BS, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.zeros(nseq, width, dtype=torch.int32, device=dev)
    starts = torch.cumsum(nb, 0) - nb
    col = torch.arange(width, device=dev)
    live = col[None] < nb[:, None]
    bt[live] = (starts[:, None] + col[None])[live].int()
    q = torch.randn(nseq, nh, D, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for p in PFS:
        _ffi.set_default_variant(attn_pf=p)
        ws = kernels.DecodeWorkspace(dev)
        o = kernels.paged_decode(q, kc, vc, bt, ctx, int(ctx.max()), 1 / math.sqrt(D), workspace=ws,
                                 nparts=kernels.choose_nparts(nseq, nkv, int(ctx.max())))
        torch.cuda.synchronize(dev)
        outs.append(o.clone())
    return all(bool(torch.equal(outs[0], o)) for o in outs[1:])


def main():
    dev = torch.device("cuda:0")
    print(json.dumps({"bit_identical": same_outputs(dev)}), flush=True)
    sys.path.insert(0, "scripts/probe")
    from attn_chunk_sweep import setup, time_it
    for nseq, lo, hi in ((512, 17, 1536), (256, 17, 1536), (1024, 17, 1536), (512, 1280, 1280), (64, 4096, 4096)):
        args = setup(dev, nseq, lo, hi)
        nparts = kernels.choose_nparts(nseq, 2, args[5])
        for rep in range(2):
            for p in PFS:
                _ffi.set_default_variant(attn_pf=p)
                us, gbs, _ = time_it(dev, args, nparts, kernels.MIN_PARTITION, reps=50)
                print(json.dumps({"nseq": nseq, "ctx": f"U[{lo},{hi}]", "nparts": nparts, "attn_pf": p, "rep": rep,
                                  "us": round(us, 2), "GBps": round(gbs, 1)}), flush=True)
    _ffi.set_default_variant(attn_pf=0)


if __name__ == "__main__":
    main()
