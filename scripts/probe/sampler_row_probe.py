"""Row-mode sampler A/B (skyrl_variant "sampler_row" 0 / 1) at the bench shape (512 x 151,936 bf16):
interleaved passes of 64 launches, plus token/logprob equality against variant 0."""
import json
import sys

import torch

sys.path.insert(0, ".")
from skyrl_amd import _ffi, ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    N, V = 512, 151936
    logits = torch.empty((8, N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(N, device=dev)
    tok = torch.empty(N, dtype=torch.int32, device=dev)
    lp = torch.empty(N, dtype=torch.float32, device=dev)
    res = {}
    variants = (0, 1)
    for T in (1.0, 0.0):
        ref = None
        for var in variants:
            _ffi.set_default_variant(sampler_row=var)
            ops.sample(logits[0], temperature=T, seed=1, seq_ids=ids, step=3, tokens_out=tok, logp_out=lp)
            got = (tok.clone(), lp.clone())
            ref = got if ref is None else ref
            res[f"T{T}_v{var}_same"] = bool(torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1]))
        for rep in range(4):
            for var in variants:
                _ffi.set_default_variant(sampler_row=var)
                for i in range(3):
                    ops.sample(logits[i], temperature=T, seed=1, seq_ids=ids, step=i, tokens_out=tok, logp_out=lp)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(64):
                    ops.sample(logits[i % 8], temperature=T, seed=1, seq_ids=ids, step=i, tokens_out=tok, logp_out=lp)
                b.record()
                b.synchronize()
                res.setdefault(f"T{T}_v{var}_us", []).append(round(a.elapsed_time(b) / 64 * 1e3, 2))
    _ffi.set_default_variant(sampler_row=1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
