"""Learner lm_head forward (old / ref log-probs) at the config-2 shape (H = 1536, V = 151,936):
the persistent tile kernel (skyrl_variant lmhead_persist = 1, the default) vs the one-tile-per-
workgroup epilogue kernel (lmhead_persist = 0, pipe 12) vs the V-chunked hipBLASLt path, with a
correctness check of the persistent form against the fp32 oracle on the kernel's own bf16 logits.
Variants interleaved over rounds in one process; one JSON line."""

import argparse
import json
import statistics

import torch

from skyrl_amd import _ffi, lmhead, ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[4096, 8192, 16384])
    ap.add_argument("--H", type=int, default=1536)
    ap.add_argument("--V", type=int, default=151936)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1, 2, 3], help="skyrl_variant lmhead_persist values")
    ap.add_argument("--groups", type=int, nargs="*", default=[], help="skyrl_variant lmhead_group values for the persistent default")
    ap.add_argument("--no-chunked", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    H, V = args.H, args.V
    g = torch.Generator(device=dev).manual_seed(0)
    W = (torch.randn(V, H, device=dev, generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16)
    out = {"H": H, "V": V}
    if args.check:
        from oracle import cpu_ref
        for T, temp in ((300, 1.0), (1000, 0.7)):
            h = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
            lab = torch.randint(0, V, (T,), device=dev, generator=g)
            lab[:4] = torch.tensor([0, 255, 256, V - 1], device=dev)
            z = ops.lmhead_gemm(h, W).cpu()
            zt = (z.float() / temp).to(torch.bfloat16) if temp != 1.0 else z
            e_lp = cpu_ref.logprobs_from_logits(zt, lab.cpu())
            e_ent = cpu_ref.entropy_from_logits(zt)
            chk = {}
            for pv in args.variants:
                with _ffi.variant(lmhead_persist=pv):
                    lp, ent = ops.lmhead_logprob_fwd(h, W, lab, temperature=temp)
                chk[f"persist{pv}"] = [float((lp.cpu() - e_lp).abs().max()), float((ent.cpu() - e_ent).abs().max())]
            out[f"check_T{T}_lp_ent_maxerr"] = chk
    for T in args.T:
        h = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
        lab = torch.randint(0, V, (T,), device=dev, generator=g)
        fl = 2.0 * T * H * V

        def fused(pv):
            def f():
                with _ffi.variant(lmhead_persist=pv):
                    ops.lmhead_logprob_fwd(h, W, lab)
            return f

        def chunked():
            with torch.no_grad():
                lmhead.lmhead_logprobs_and_entropy(h, W, lab, 1.0, True)

        fns = {f"persist{pv}": fused(pv) for pv in args.variants}

        def grouped(gp):
            def f():
                with _ffi.variant(lmhead_group=gp):
                    ops.lmhead_logprob_fwd(h, W, lab)
            return f

        for gp in args.groups:
            fns[f"group{gp}"] = grouped(gp)
        fns["persist_default_noentropy"] = lambda: ops.lmhead_logprob_fwd(h, W, lab, compute_entropy=False)
        if not args.no_chunked:
            fns["chunked"] = chunked
        res = {k: [] for k in fns}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for k, f in fns.items():
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.iters):
                    f()
                b.record()
                torch.cuda.synchronize()
                res[k].append(a.elapsed_time(b) / args.iters)
        out[f"T{T}"] = {k: {"ms_median": statistics.median(v), "ms_min": min(v),
                            "PFLOPs_median": fl / statistics.median(v) / 1e12} for k, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
