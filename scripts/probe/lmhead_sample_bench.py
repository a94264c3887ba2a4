"""Decode-step lm_head + sampler (§8(f)1 decode side) at the config-2 shape (H=1536, V=151,936):

  unfused : torch F.linear (hipBLASLt) -> bf16 logits [M,V] -> skyrl_sample
  gemm    : skyrl_lmhead_gemm alone (the fused kernel's GEMM with a bf16 store epilogue)
  linear  : torch F.linear alone
  fused   : skyrl_lmhead_sample (sampler in the GEMM epilogue + one merge launch)

One JSON line per (M, T). Random operands (bf16 GEMMs clock lower on random data than on zeros).
"""

import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from skyrl_amd import ops  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[512, 256, 64, 8])
    ap.add_argument("--H", type=int, default=1536)
    ap.add_argument("--V", type=int, default=151936)
    ap.add_argument("--T", type=float, nargs="+", default=[1.0])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--pipes", type=int, nargs="+", default=[-1], help="skyrl_variant lmhead_pipe variants (-1: default)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    H, V = args.H, args.V
    w = (torch.randn(V, H, device=dev) * (3.0 / H ** 0.5)).to(torch.bfloat16)
    from skyrl_amd import _ffi
    for M, pipe in [(m, p) for m in args.M for p in args.pipes]:
        _ffi.set_default_variant(lmhead_pipe=pipe)
        h = torch.randn(M, H, device=dev).to(torch.bfloat16)
        ids = torch.arange(M, device=dev)
        z = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        tok = torch.empty(M, dtype=torch.int32, device=dev)
        lp = torch.empty(M, dtype=torch.float32, device=dev)
        flops = 2.0 * M * H * V
        for T in args.T:
            def unfused():
                torch.matmul(h, w.T, out=z)
                ops.sample(z, temperature=T, seed=1, seq_ids=ids, step=3, tokens_out=tok, logp_out=lp)

            def fused():
                ops.lmhead_sample(h, w, temperature=T, seed=1, seq_ids=ids, step=3, tokens_out=tok, logp_out=lp)

            res = {"M": M, "H": H, "V": V, "T": T, "pipe": pipe,
                   "linear_us": timeit(lambda: torch.matmul(h, w.T, out=z), args.iters),
                   "gemm_us": timeit(lambda: ops.lmhead_gemm(h, w, out=z), args.iters),
                   "unfused_us": timeit(unfused, args.iters),
                   "fused_us": timeit(fused, args.iters)}
            res["sampler_us"] = res["unfused_us"] - res["linear_us"]
            for k in ("linear", "gemm", "fused"):
                res[f"{k}_TFs"] = round(flops / (res[f"{k}_us"] * 1e-6) / 1e12, 1)
            res["fused_speedup"] = round(res["unfused_us"] / res["fused_us"], 3)
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)




def learner_main():
    """Learner-side forward logprob at T tokens: chunked hipBLASLt path vs the fused epilogue."""
    import sys as _s
    from skyrl_amd import lmhead

    dev = torch.device("cuda")
    H, V = 1536, 151936
    w = (torch.randn(V, H, device=dev) * (3.0 / H ** 0.5)).to(torch.bfloat16)
    for T in (4096, 8192, 16384):
        h = torch.randn(T, H, device=dev).to(torch.bfloat16)
        lab = torch.randint(0, V, (T,), device=dev)
        with torch.no_grad():
            chunked = timeit(lambda: lmhead.lmhead_logprobs_and_entropy(h, w, lab), 5)
            fused = timeit(lambda: ops.lmhead_logprob_fwd(h, w, lab), 5)
        flops = 2.0 * T * H * V
        print(json.dumps({"T": T, "chunked_us": round(chunked, 1), "fused_us": round(fused, 1),
                          "fused_TFs": round(flops / (fused * 1e-6) / 1e12, 1),
                          "chunked_TFs": round(flops / (chunked * 1e-6) / 1e12, 1)}), flush=True)


PIPES = (12, 14)


def gemm_sweep(shapes=((512, 151936), (8192, 151936))):
    """Plain GEMM (STORE epilogue) per pipeline variant vs torch, interleaved passes."""
    from skyrl_amd import _ffi

    dev = torch.device("cuda")
    H = 1536
    for M, V in shapes:
        w = (torch.randn(V, H, device=dev) * (3.0 / H ** 0.5)).to(torch.bfloat16)
        h = torch.randn(M, H, device=dev).to(torch.bfloat16)
        z = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        flops = 2.0 * M * H * V
        it = 20 if M <= 512 else 4
        for rep in range(2):
            res = {"M": M, "V": V, "rep": rep, "torch_us": round(timeit(lambda: torch.matmul(h, w.T, out=z), it), 1)}
            for pipe in PIPES:
                _ffi.set_default_variant(lmhead_pipe=pipe)
                res[f"pipe{pipe}_us"] = round(timeit(lambda: ops.lmhead_gemm(h, w, out=z), it), 1)
            zs = []
            for pipe in PIPES:
                _ffi.set_default_variant(lmhead_pipe=pipe)
                zs.append(ops.lmhead_gemm(h, w).clone())
            res["all_equal"] = all(bool(torch.equal(zs[0], z)) for z in zs[1:])
            _ffi.set_default_variant(lmhead_pipe=-1)
            res["best_TFs"] = round(flops / (min(v for k, v in res.items() if k.startswith("pipe") and k.endswith("_us")) * 1e-6) / 1e12, 1)
            print(json.dumps(res), flush=True)


def gemm_group_sweep():
    """Tile order (skyrl_variant lmhead_group: M tiles per group, 0 = all) x pipeline, learner and
    decode shapes; every configuration's Z must equal the default's bit for bit."""
    from skyrl_amd import _ffi

    dev = torch.device("cuda")
    H, V = 1536, 151936
    w = (torch.randn(V, H, device=dev) * (3.0 / H ** 0.5)).to(torch.bfloat16)
    for M in (8192, 2048, 512):
        h = torch.randn(M, H, device=dev).to(torch.bfloat16)
        z = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        flops = 2.0 * M * H * V
        it = 20 if M <= 512 else 4
        ref = ops.lmhead_gemm(h, w).clone()
        res = {"M": M, "torch_us": round(timeit(lambda: torch.matmul(h, w.T, out=z), it), 1)}
        same = True
        for rep in range(2):
            for pipe in (4, 12):
                for grp in (0, 4, 8):
                    _ffi.set_default_variant(lmhead_pipe=pipe)
                    _ffi.set_default_variant(lmhead_group=grp)
                    t = round(timeit(lambda: ops.lmhead_gemm(h, w, out=z), it), 1)
                    res.setdefault(f"p{pipe}_g{grp}_us", []).append(t)
                    if rep == 0:
                        same = same and bool(torch.equal(ops.lmhead_gemm(h, w), ref))
        _ffi.set_default_variant(lmhead_pipe=-1)
        _ffi.set_default_variant(lmhead_group=0)
        best = min(min(v) for k, v in res.items() if k.endswith("_us") and k != "torch_us")
        res.update({"all_equal": same, "best_TFs": round(flops / (best * 1e-6) / 1e12, 1)})
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    import sys as _sys
    if "--gemm-sweep" in _sys.argv:
        gemm_sweep()
    elif "--gemm-groups" in _sys.argv:
        gemm_group_sweep()
    elif "--gemm-shapes" in _sys.argv:
        gemm_sweep(((8192, 8192), (4096, 32768), (2048, 151936), (512, 151936)))
    elif "--learner" in _sys.argv:
        learner_main()
    else:
        main()
