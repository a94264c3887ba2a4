"""Per-kernel microbenchmarks at the north-star sizes (GPU box), variants A/B'd in one process.

Times each hot-path kernel with HIP events on its launch stream, interleaving variants over
rounds (guide §5.4 rule 24), and prints one JSON object: median ms and algorithmic GB/s.
"""

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from skyrl_amd import _ffi, ops, ppo_utils  # noqa: E402
from skyrl_amd.config import AlgorithmConfig  # noqa: E402


def timeit(fn, iters=5):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    R, V, mb, N = 1024, 151936, 16, 512
    rows = mb * R
    gen = torch.Generator(device=dev).manual_seed(0)
    logits = torch.empty((2 * rows, V), dtype=torch.bfloat16, device=dev).normal_(0, 3, generator=gen)
    dlog = torch.empty((mb, R, V), dtype=torch.bfloat16, device=dev)
    labels = torch.randint(0, V, (mb, R), device=dev, generator=gen)
    lp = torch.empty((mb, R), device=dev)
    ent = torch.empty_like(lp)
    lse = torch.empty_like(lp)
    glp = torch.randn((mb, R), device=dev, generator=gen) * 1e-3
    st = ops._stream(dev)
    res = {}
    want = set(args.only.split(",")) if args.only else None

    def on(k):
        return want is None or k in want

    # ---- measured copy peak (read+write) on a same-size buffer
    if on("copy"):
        src = logits[:rows]
        dst = dlog.view(rows, V)
        ms = statistics.median(timeit(lambda: dst.copy_(src)) for _ in range(args.rounds))
        res["copy_bf16_5GB"] = {"ms": ms, "GBps": 2 * src.numel() * 2 / ms / 1e6}

    x0 = logits[:rows].view(mb, R, V)
    x1 = logits[rows:].view(mb, R, V)
    fwd_bytes = rows * (V * 2 + 8 + 12)
    bwd_bytes = rows * (V * 4 + 8 + 16)
    variants = [(4, 1), (8, 1), (4, 0), (8, 0)]

    def fwd(x):
        _ffi.call("skyrl_logprob_fwd", ops._ptr(x), _ffi.BF16, x.stride(0), x.stride(1), mb, R, V, ops._ptr(labels),
                  labels.stride(0), labels.stride(1), 1.0, ops._ptr(lp), ops._ptr(ent), ops._ptr(lse), st)

    def bwd(x):
        _ffi.call("skyrl_logprob_bwd", ops._ptr(x), _ffi.BF16, x.stride(0), x.stride(1), mb, R, V, ops._ptr(labels),
                  labels.stride(0), labels.stride(1), 1.0, ops._ptr(lse), ops._ptr(ent), ops._ptr(glp), None,
                  ops._ptr(dlog), st)

    if on("logprob"):
        times = {v: {"fwd": [], "bwd": []} for v in variants}
        for r in range(args.rounds):
            for (u, nt) in variants:
                _ffi.set_default_variant(logprob_unroll=u)
                _ffi.set_default_variant(logprob_nt=nt)
                times[(u, nt)]["fwd"].append(timeit(lambda: (fwd(x0), fwd(x1))) / 2)
                times[(u, nt)]["bwd"].append(timeit(lambda: (bwd(x0), bwd(x1))) / 2)
        for (u, nt), t in times.items():
            f, b = statistics.median(t["fwd"]), statistics.median(t["bwd"])
            res[f"logprob_fwd_u{u}_nt{nt}"] = {"ms": f, "GBps": fwd_bytes / f / 1e6}
            res[f"logprob_bwd_u{u}_nt{nt}"] = {"ms": b, "GBps": bwd_bytes / b / 1e6}
        _ffi.set_default_variant(logprob_unroll=4)
        _ffi.set_default_variant(logprob_nt=1)

    if on("fused"):
        from skyrl_amd import ppo_utils as pu

        params = pu.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=True)
        old = torch.randn((mb, R), device=dev, generator=gen) - 12
        adv = torch.randn((mb, R), device=dev, generator=gen)
        msk = torch.ones((mb, R), device=dev)
        ref = old + 0.01
        loss = torch.empty((), device=dev)
        met = torch.empty(8, device=dev)
        ws = torch.zeros(_ffi.query("skyrl_policy_train_workspace_bytes", mb, R), dtype=torch.uint8, device=dev)
        import ctypes

        def fused(x):
            _ffi.call("skyrl_policy_train_fwd", ops._ptr(x), _ffi.BF16, x.stride(0), x.stride(1), mb, R, V,
                      ops._ptr(labels), labels.stride(0), labels.stride(1), 1.0, ops._ptr(old), ops._ptr(adv),
                      ops._ptr(msk), ops._ptr(ref), ctypes.byref(params), ops._ptr(loss), ops._ptr(met), ops._ptr(lp),
                      ops._ptr(ent), ops._ptr(dlog), R * V, V, ops._ptr(ws), st)
        # (split, resident, nt stores, resident threads)
        # (split, resident, nt stores, resident threads, 100 * split parts)
        # (split, resident, nt stores, resident threads, split shape: skyrl_variant "train_split_shape")
        variants = [(1, 1, 1, 1024, 0), (1, 1, 1, 1024, 1), (1, 1, 0, 1024, 0), (0, 1, 1, 1024, 0)]
        times = {v: [] for v in variants}
        for _ in range(args.rounds):  # interleaved rounds
            for v in variants:
                split, resident, nts, nt, sm = v
                _ffi.set_default_variant(train_split_shape=sm)
                _ffi.set_default_variant(train_split=split)
                _ffi.set_default_variant(train_resident=resident)
                _ffi.set_default_variant(train_ntstore=nts)
                _ffi.set_default_variant(train_resident_nt=nt)
                times[v].append(timeit(lambda: (fused(x0), fused(x1))) / 2)
        _ffi.set_default_variant(train_split=1)
        _ffi.set_default_variant(train_split_shape=0)
        for (split, resident, nts, nt, sm), t in times.items():
            ms = statistics.median(t)
            res[f"policy_train_fused_split{split}_shape{sm}_resident{resident}_nts{nts}_nt{nt}"] = {
                "ms": ms, "GBps_hbm_algorithmic": rows * (V * 4 + 40) / ms / 1e6,
                "vs_unfused_bytes": rows * (V * 6) / ms / 1e6}
        _ffi.set_default_variant(train_resident=1)
        _ffi.set_default_variant(train_ntstore=1)
        _ffi.set_default_variant(train_resident_nt=1024)

    if on("fused_mb"):  # the fused pass at smaller micro-batches (bytes per launch vs rate)
        from skyrl_amd import ppo_utils as pu
        import ctypes

        params = pu.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=True)
        old = torch.randn((mb, R), device=dev, generator=gen) - 12
        adv = torch.randn((mb, R), device=dev, generator=gen)
        msk = torch.ones((mb, R), device=dev)
        ref = old + 0.01
        loss = torch.empty((), device=dev)
        met = torch.empty(8, device=dev)
        ws = torch.zeros(_ffi.query("skyrl_policy_train_workspace_bytes", mb, R), dtype=torch.uint8, device=dev)

        def fused_m(x, m, off):
            _ffi.call("skyrl_policy_train_fwd", ops._ptr(x[off:off + m]), _ffi.BF16, x.stride(0), x.stride(1), m, R, V,
                      ops._ptr(labels), labels.stride(0), labels.stride(1), 1.0, ops._ptr(old), ops._ptr(adv),
                      ops._ptr(msk), ops._ptr(ref), ctypes.byref(params), ops._ptr(loss), ops._ptr(met), ops._ptr(lp),
                      ops._ptr(ent), ops._ptr(dlog[off:off + m]), R * V, V, ops._ptr(ws), st)
        times = {m: [] for m in (4, 8, 16)}
        for _ in range(args.rounds):
            for m in times:
                # the same 2 x 16 sequences in launches of m
                def run():
                    for x in (x0, x1):
                        for off in range(0, mb, m):
                            fused_m(x, m, off)
                times[m].append(timeit(run) / 2)
        for m, t in times.items():
            ms = statistics.median(t)
            res[f"policy_train_fused_mb{m}"] = {"ms_per_16_seqs": ms, "GBps_hbm_algorithmic": rows * (V * 4 + 40) / ms / 1e6}

    if on("fused_vocab"):  # split pieces per row vs vocabulary (odd V = 50,257: EDGE forms)
        from skyrl_amd import ppo_utils as pu
        import ctypes

        params = pu.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=True)
        old = torch.randn((mb, R), device=dev, generator=gen) - 10
        adv = torch.randn((mb, R), device=dev, generator=gen)
        msk = torch.ones((mb, R), device=dev)
        ref = old + 0.01
        loss = torch.empty((), device=dev)
        met = torch.empty(8, device=dev)
        ws = torch.zeros(_ffi.query("skyrl_policy_train_workspace_bytes", mb, R), dtype=torch.uint8, device=dev)
        del logits
        for V2 in (50257, 50264, 128256, 151936):
            lab2 = torch.randint(0, V2, (mb, R), device=dev, generator=gen)
            g2 = [torch.empty((mb, R, V2), dtype=torch.bfloat16, device=dev).normal_(0, 3, generator=gen)
                  for _ in range(2)]
            d2 = torch.empty((mb, R, V2), dtype=torch.bfloat16, device=dev)

            def fused2(x):
                _ffi.call("skyrl_policy_train_fwd", ops._ptr(x), _ffi.BF16, x.stride(0), x.stride(1), mb, R, V2,
                          ops._ptr(lab2), lab2.stride(0), lab2.stride(1), 1.0, ops._ptr(old), ops._ptr(adv),
                          ops._ptr(msk), ops._ptr(ref), ctypes.byref(params), ops._ptr(loss), ops._ptr(met),
                          ops._ptr(lp), ops._ptr(ent), ops._ptr(d2), R * V2, V2, ops._ptr(ws), st)
            # (split, shape: skyrl_variant "train_split_shape"); split 0 = the resident kernel
            variants = [(1, sh) for sh in range(0, 6)] + [(0, 0)]  # shape 0: the default by vocabulary
            times = {v: [] for v in variants}
            for _ in range(args.rounds):
                for v in variants:
                    _ffi.set_default_variant(train_split=v[0])
                    _ffi.set_default_variant(train_split_shape=v[1])
                    times[v].append(timeit(lambda: (fused2(g2[0]), fused2(g2[1]))) / 2)
            _ffi.set_default_variant(train_split=1)
            _ffi.set_default_variant(train_split_shape=0)
            for (split, shape), t in times.items():
                ms = statistics.median(t)
                res[f"policy_train_V{V2}_split{split}_shape{shape}"] = {
                    "ms": ms, "GBps_hbm_algorithmic": rows * (V2 * 4 + 40) / ms / 1e6}
            del g2, d2
            torch.cuda.empty_cache()
        print(json.dumps(res, indent=1))
        return

    if on("sample"):
        from skyrl_amd.config import SamplingParams
        from skyrl_amd.sampler import TokenSampler

        sh = torch.cuda.current_stream(dev).cuda_stream
        for name, sp in (("sample_t1", SamplingParams()), ("sample_greedy", SamplingParams(temperature=0.0)),
                         ("sample_topk50", SamplingParams(top_k=50)), ("sample_minp", SamplingParams(min_p=0.05)),
                         ("sample_topp09", SamplingParams(top_p=0.9)),
                         ("sample_topk50_topp09", SamplingParams(top_k=50, top_p=0.9))):
            smp = TokenSampler(N, V, R, dev, sp, seed=1)

            def go(t=[0]):
                t[0] += 1
                # 512 rows with row stride 64*V (like the bench's [N,R,V][:, t] view)
                smp.step_ptr(logits.data_ptr() + 2 * V * (t[0] % 64), 64 * V, t[0] % R, sh)
            ms = statistics.median(timeit(go, iters=50) for _ in range(args.rounds))
            res[name] = {"ms": ms, "GBps": N * V * 2 / ms / 1e6}

    if on("small"):
        g = torch.Generator().manual_seed(1234)
        lens = torch.randint(1, R + 1, (N,), generator=g)
        mask = (torch.arange(R)[None] < lens[:, None]).to(torch.int64).to(dev)
        rew = torch.zeros(N, R, device=dev)
        rew[torch.arange(N), (lens - 1).to(dev)] = 1.0
        uids = [str(i // 8) for i in range(N)]
        goff, grows, ng = ops.groups_from_index(uids)
        goff, grows = goff.to(dev), grows.to(dev)
        ms = statistics.median(timeit(lambda: ops.grpo_advantage(rew, mask, goff, grows, ng), 50)
                               for _ in range(args.rounds))
        res["grpo_adv"] = {"ms": ms, "GBps": N * R * (4 + 8 + 4) / ms / 1e6}
        lmask = mask.float()
        a = torch.randn(N, R, device=dev)
        l0 = -2 + 0.1 * torch.randn(N, R, device=dev)
        params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=True)

        def loss_fb():
            x = l0.requires_grad_(True)
            loss, m = ops.ppo_loss(x, l0.detach() + 0.01, a, lmask, params, ref_log_probs=l0.detach() - 0.01,
                                   entropy=a)
            torch.autograd.grad(loss, x)
        ms = statistics.median(timeit(loss_fb, 50) for _ in range(args.rounds))
        res["ppo_loss_fwd_bwd"] = {"ms": ms, "GBps": N * R * (20 + 4 + 4 + 12) / ms / 1e6}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
