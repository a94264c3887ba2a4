"""Does longest-first dispatch shorten the ragged paged-decode launch? The bench's rollout
attention shape (512 sequences, contexts U[17, 1536], Qwen2.5-1.5B heads): the same batch in
random order vs sorted by context length, longest first (blockIdx.z = sequence, so the
dispatcher hands out the long sequences' waves first). Interleaved rounds, one process."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd.inference_engines import kernels  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    nseq, nh, nkv, D, BS = 512, 12, 2, 128, 16
    g = torch.Generator(device=dev).manual_seed(11)
    ctx = torch.randint(17, 1537, (nseq,), device=dev, generator=g, dtype=torch.int32)
    nb = (ctx + BS - 1) // BS
    max_ctx = int(ctx.max())
    width = (max_ctx + BS - 1) // BS
    nblk = int(nb.sum())
    kc = torch.randn(nblk, nkv, BS, D, device=dev, generator=g).to(torch.bfloat16)
    vc = torch.randn(nblk, nkv, D, BS, device=dev, generator=g).to(torch.bfloat16)
    perm = torch.randperm(nblk, device=dev, generator=g).int()
    bt = torch.zeros(nseq, width, dtype=torch.int32, device=dev)
    starts = torch.cumsum(nb, 0) - nb
    col = torch.arange(width, device=dev)
    live = col[None] < nb[:, None]
    bt[live] = perm[(starts[:, None] + col[None])[live]]
    q = torch.randn(nseq, nh, D, device=dev, generator=g).to(torch.bfloat16)
    order = torch.argsort(ctx, descending=True)
    variants = {"random": (q, bt, ctx), "longest_first": (q[order].contiguous(), bt[order].contiguous(),
                                                           ctx[order].contiguous()),
                "shortest_first": (q[order.flip(0)].contiguous(), bt[order.flip(0)].contiguous(),
                                   ctx[order.flip(0)].contiguous())}
    ws = kernels.DecodeWorkspace(dev)
    nparts = kernels.choose_nparts(nseq, nkv, max_ctx)
    outs = {k: torch.empty_like(q) for k in variants}

    def run(k):
        qq, bb, cc = variants[k]
        kernels.paged_decode(qq, kc, vc, bb, cc, max_ctx, 1 / math.sqrt(D), out=outs[k], workspace=ws, nparts=nparts)

    for k in variants:
        run(k)
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(5):
        for k in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                run(k)
            b.record()
            b.synchronize()
            res[k].append(round(a.elapsed_time(b) * 1e3 / 20, 2))
    same = torch.equal(outs["longest_first"], outs["random"][order])
    print(json.dumps({"nparts": nparts, "us_per_launch": res, "outputs_equal_permuted": bool(same)}))


if __name__ == "__main__":
    main()
