"""Wide split sampler (r06, sample_wide_kernel: every load of a workgroup in flight at once) vs the
streaming split kernel (sample_kernel in split mode) on the product library, selected with
skyrl_variant ("sampler_wide_rows", 0 | 256). Rows in ROWS (default 1,8,16,32,64,96,128,192) x V =
151,936 bf16 N(0, 3) logits, T = 1, 0.7 and greedy; interleaved rounds of 200 back-to-back
launches through TokenSampler.step_ptr, medians (us). The tokens of both kernels must be equal
(both take the exact-score argmax) and the logprobs within 1e-5. Prints one JSON line.
Run (GPU): python scripts/probe/sampler_wide_ab.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import _ffi  # noqa: E402
from skyrl_amd.config import SamplingParams  # noqa: E402
from skyrl_amd.sampler import TokenSampler  # noqa: E402

ROWS = [int(v) for v in os.environ.get("ROWS", "1,8,16,32,64,96,128,192").split(",")]
WGS = [int(v) for v in os.environ.get("WIDE_WGS", "512").split(",")]


def main():
    dev = torch.device("cuda:0")
    V = 151936
    big = torch.empty((max(ROWS), V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    sh = torch.cuda.current_stream(dev).cuda_stream
    samplers = {(n, temp): TokenSampler(n, V, 200, dev, SamplingParams(temperature=temp), seed=1)
                for n in ROWS for temp in (1.0, 0.7, 0.0)}
    variants = [("split", 0, 512)] + [(f"wide{w}", 256, w) for w in WGS]
    out, toks, lps = {}, {}, {}
    for rnd in range(5):
        for name, rows_knob, wgs in variants:
            _ffi.set_default_variant(sampler_wide_rows=rows_knob)
            _ffi.set_default_variant(sampler_wide_wgs=wgs)
            for (n, temp), smp in samplers.items():
                key = f"n{n}_T{temp}_{name}"
                for t in range(4):
                    smp.step_ptr(big.data_ptr(), V, t, sh)
                torch.cuda.synchronize()
                if rnd == 0:
                    toks.setdefault(f"n{n}_T{temp}", []).append(smp.tokens[:4].cpu().clone())
                    lps.setdefault(f"n{n}_T{temp}", []).append(smp.logprobs[:4].cpu().clone())
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for t in range(200):
                    smp.step_ptr(big.data_ptr(), V, t, sh)
                b.record()
                b.synchronize()
                out.setdefault(key, []).append(a.elapsed_time(b) / 200 * 1e3)
    _ffi.set_default_variant(sampler_wide_rows=256)  # the defaults
    _ffi.set_default_variant(sampler_wide_wgs=512)
    res = {k: round(sorted(x)[len(x) // 2], 2) for k, x in out.items()}
    res["tokens_equal"] = all(all(torch.equal(v[0], w) for w in v) for v in toks.values())
    res["logprob_maxdiff"] = max(float((w - v[0]).abs().max()) for v in lps.values() for w in v)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
