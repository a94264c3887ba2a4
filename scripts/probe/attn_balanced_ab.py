"""A/B of block-balanced decode attention (kernels.paged_decode_balanced: plan + attention +
merge) against the per-sequence split (kernels.paged_decode) on ragged and uniform contexts at
the rollout head shape (12 q / 2 kv heads, D = 128), over wave counts. Prints one JSON line per
point; `max_abs_diff` is against the per-sequence kernel's output. Probe only."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts/probe")
from attn_chunk_sweep import D, NH, NKV, setup, time_it  # noqa: E402

from skyrl_amd.inference_engines import kernels  # noqa: E402


def time_balanced(dev, args, waves, reps=50):
    q, kc, vc, bt, ctx, _ = args
    out = torch.empty_like(q)
    ws = kernels.DecodeWorkspace(dev)
    run = lambda: kernels.paged_decode_balanced(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out=out,  # noqa: E731
                                                workspace=ws, waves=waves)
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
    for nseq, lo, hi in ((512, 17, 1536), (256, 17, 1536), (1024, 17, 1536), (512, 1280, 1280), (64, 4096, 4096),
                         (128, 17, 1536)):
        args = setup(dev, nseq, lo, hi)
        nparts = kernels.choose_nparts(nseq, NKV, args[5])
        for rep in range(2):
            us, gbs, ref = time_it(dev, args, nparts, kernels.MIN_PARTITION)
            print(json.dumps({"nseq": nseq, "ctx": f"U[{lo},{hi}]", "mode": "per_sequence", "nparts": nparts,
                              "rep": rep, "us": round(us, 2), "GBps": round(gbs, 1)}), flush=True)
            for waves in (256, 384, 512, 768, 1024):
                us, gbs, o = time_balanced(dev, args, waves)
                print(json.dumps({"nseq": nseq, "ctx": f"U[{lo},{hi}]", "mode": "balanced", "waves_per_kv": waves,
                                  "rep": rep, "us": round(us, 2), "GBps": round(gbs, 1),
                                  "max_abs_diff": float((o.float() - ref.float()).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
