"""Paged decode attention at the bench's ragged rollout shape (512 seqs, ctx U[17,1536],
Qwen2.5-1.5B heads): sweep the wave count per (sequence, kv head) that choose_nparts picks."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from skyrl_amd.inference_engines import kernels  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda:0")
    res = {}
    orig = kernels.choose_nparts
    for nseq in (512, 64):
        for np_ in (1, 2, 3, 4, 6, 8, 12, 24):
            kernels.choose_nparts = lambda *a, _n=np_, **k: _n
            r = bench.rollout_attention_leg(dev, nseq)
            res[f"{nseq}/{np_}"] = (r["avg_launch_us"], r["achieved_GBps"])
            print(nseq, np_, res[f"{nseq}/{np_}"], flush=True)
        kernels.choose_nparts = orig
        res[f"{nseq}/auto"] = bench.rollout_attention_leg(dev, nseq)["achieved_GBps"]
    print(json.dumps(res), flush=True)
