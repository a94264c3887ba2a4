"""Where the two-pass top_p kernel's time goes at the bench shape [512, 151,936] bf16, T = 1:
skyrl_variant ("topp_probe") 1 = pass 1 alone, 2 = pass 1 + the cut, 3 / 4 = pass 1 + the cut + a bare
re-read of the row (nontemporal / cached loads) (tokens invalid in 1-4), 0 = the whole kernel; beside it the unfiltered T = 1 and greedy samplers (one read of the row) and
the two-kernel path. One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import ops  # noqa: E402

FILT = 1024 * 4  # the RowFilter array's offset (csrc/sampler.hip kCounterBytes)


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / reps, 2)


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    n, V = 512, 151936
    x = (torch.randn(n, V, device=dev, generator=g) * 3).to(torch.bfloat16)
    ids = torch.arange(n, dtype=torch.int64, device=dev)
    tok = torch.empty(n, dtype=torch.int32, device=dev)
    lp = torch.empty(n, dtype=torch.float32, device=dev)
    out = {}
    for name, kw in (("top_p0.95", dict(top_p=0.95)), ("top_p0.95_T0.6", dict(top_p=0.95, temperature=0.6)),
                     ("top_p0.9", dict(top_p=0.9)), ("min_p0.05", dict(min_p=0.05))):
        temp = kw.pop("temperature", 1.0)
        res = {}
        for probe in (1, 2, 3, 4, 0):
            ops._ffi.set_default_variant(topp_probe=probe)
            res[f"probe{probe}_us"] = timed(lambda: ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=1,
                                                               tokens_out=tok, logp_out=lp, **kw))
        ops._ffi.set_default_variant(topp_probe=0)
        ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=1, tokens_out=tok, logp_out=lp, **kw)
        ws = ops.WORKSPACES.get(dev, "sample", ops._ffi.query("skyrl_sample_workspace_bytes", n, V))
        ff = ws[FILT:FILT + 20 * n].view(torch.int32).view(n, 5).cpu()
        res["pass1_decided"] = int((ff[:, 1] == 1).sum())  # RowFilter.tk = 1: certified in pass 1
        # per-row in-row pass-2 time (min_p alone; top_p's left rows go to the pass-2 kernel): 5 every
        # row takes pass 2, 6 the rows that do, 7 as 6 with the stage loop's visits replaced by an xor
        for probe in ((6, 7) if name.startswith("min_p") else ()):
            ops._ffi.set_default_variant(topp_probe=probe)
            tok.fill_(-1)
            ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=1, tokens_out=tok, logp_out=lp, **kw)
            ff = ws[FILT:FILT + 20 * n].view(torch.int32).view(n, 5).cpu()
            p2 = tok.cpu()[ff[:, 1] != 1].float() / 100.0  # us
            pre = lp.cpu()[ff[:, 1] != 1].float() / 100.0
            if p2.numel():
                res[f"probe{probe}_rows"] = int(p2.numel())
                res[f"probe{probe}_pass2_us"] = [round(float(p2.min()), 2), round(float(p2.median()), 2), round(float(p2.max()), 2)]
                res[f"probe{probe}_before_us"] = [round(float(pre.min()), 2), round(float(pre.median()), 2), round(float(pre.max()), 2)]
        if name.startswith("top_p"):  # 11: per row, the cut's time (tokens) and pass 1's (logprobs)
            ops._ffi.set_default_variant(topp_probe=11)
            ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=1, tokens_out=tok, logp_out=lp, **kw)
            c = tok.cpu().float() / 100.0
            p1 = lp.cpu().float() / 100.0
            res["probe11_cut_us"] = [round(float(c.min()), 2), round(float(c.median()), 2), round(float(c.max()), 2)]
            res["probe11_pass1_us"] = [round(float(p1.min()), 2), round(float(p1.median()), 2), round(float(p1.max()), 2)]
        ops._ffi.set_default_variant(topp_probe=0)
        if name.startswith("top_p"):
            ops._ffi.set_default_variant(topp_probe=5)  # every row through the pass-2 kernel
            res["all_pass2_kernel_us"] = timed(lambda: ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=1,
                                                              tokens_out=tok, logp_out=lp, **kw))
            ops._ffi.set_default_variant(topp_probe=0)
        steps, dec = [], []
        for st in range(2, 22):  # fresh noise per decode step: how many rows pass 1 leaves varies
            steps.append(timed(lambda: ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=st, tokens_out=tok,
                                                  logp_out=lp, **kw), reps=5))
            ws = ops.WORKSPACES.get(dev, "sample", ops._ffi.query("skyrl_sample_workspace_bytes", n, V))
            dec.append(int((ws[FILT:FILT + 20 * n].view(torch.int32).view(n, 5)[:, 1] == 1).sum()))
        res["steps_2_21_us"] = [min(steps), round(sum(steps) / len(steps), 2), max(steps)]
        res["steps_2_21_rows_left"] = [n - d for d in dec]
        ops._ffi.set_default_variant(sampler_topp_fast=0)
        res["two_kernel_us"] = timed(lambda: ops.sample(x, temperature=temp, seed=3, seq_ids=ids, step=1,
                                                        tokens_out=tok, logp_out=lp, **kw), reps=10)
        ops._ffi.set_default_variant(sampler_topp_fast=1)
        out[name] = res
    out["t1_unfiltered_us"] = timed(lambda: ops.sample(x, temperature=1.0, seed=3, seq_ids=ids, step=1, tokens_out=tok,
                                                       logp_out=lp))
    out["greedy_us"] = timed(lambda: ops.sample(x, temperature=0.0, seed=3, seq_ids=ids, step=1, tokens_out=tok,
                                                logp_out=lp))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
