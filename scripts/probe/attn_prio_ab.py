"""A/B of the paged decode kernel's remaining-work priority variant (skyrl_variant "attn_prio").

Times bench.rollout_attention_leg (ragged U[17,1536] contexts, Qwen2.5-1.5B heads) with the knob
off/on interleaved, and checks the two variants give bit-identical outputs (only wave issue
priority changes). Probe only; prints one JSON line per measurement."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from skyrl_amd import _ffi  # noqa: E402
from skyrl_amd.inference_engines import kernels  # noqa: E402


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
    for p in (0, 1):
        _ffi.set_default_variant(attn_prio=p)
        ws = kernels.DecodeWorkspace(dev)
        o = kernels.paged_decode(q, kc, vc, bt, ctx, int(ctx.max()), 1 / math.sqrt(D), workspace=ws,
                                 nparts=kernels.choose_nparts(nseq, nkv, int(ctx.max())))
        torch.cuda.synchronize(dev)
        outs.append(o.clone())
    return bool(torch.equal(outs[0], outs[1]))


def main():
    dev = torch.device("cuda:0")
    print(json.dumps({"bit_identical": same_outputs(dev)}), flush=True)
    for nseq in (512, 256, 1024):
        for rep in range(3):
            for p in (0, 1):
                _ffi.set_default_variant(attn_prio=p)
                r = bench.rollout_attention_leg(dev, nseq, reps=50)
                r.update({"nseq": nseq, "attn_prio": p, "rep": rep})
                print(json.dumps(r), flush=True)
    _ffi.set_default_variant(attn_prio=0)


if __name__ == "__main__":
    main()
