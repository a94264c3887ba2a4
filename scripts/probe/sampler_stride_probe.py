"""Does the bench's strided sampler view cost time? One decode step's [512, V] rows taken from the
resident [N, R, V] logits (row stride R V: rows 311 MB apart) vs the same rows in one contiguous
[512, V] buffer (what the lm_head GEMM hands a real decode step). Interleaved rounds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, R, V = 512, 1024, 151936
    big = torch.empty((N, R, V), dtype=torch.bfloat16, device=dev)
    res = {}
    views = {}
    for t in (0, 511):
        big[:, t].normal_(0.0, 3.0)
        views[f"strided_t{t}"] = big[:, t]
    contig = big[:, 0].contiguous()
    views["contiguous"] = contig
    ids = torch.arange(N, dtype=torch.int64, device=dev)
    tok = torch.empty(N, dtype=torch.int32, device=dev)
    lp = torch.empty(N, dtype=torch.float32, device=dev)
    outs = {}
    for k, x in views.items():
        ops.sample(x, temperature=1.0, seed=1, seq_ids=ids, step=3, tokens_out=tok, logp_out=lp)
        outs[k] = tok.clone()
    torch.cuda.synchronize()
    res = {k: [] for k in views}
    for _ in range(5):
        for k, x in views.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(64):
                ops.sample(x, temperature=1.0, seed=1, seq_ids=ids, step=i, tokens_out=tok, logp_out=lp)
            b.record()
            b.synchronize()
            res[k].append(round(a.elapsed_time(b) * 1e3 / 64, 2))
    print(json.dumps({"us_per_launch": res, "tokens_equal": bool(torch.equal(outs["strided_t0"], outs["contiguous"]))}))


if __name__ == "__main__":
    main()
