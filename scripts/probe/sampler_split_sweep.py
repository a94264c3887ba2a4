"""Split-mode sampler shape sweep on the product library: skyrl_variant ("sampler_split_wgs") x
skyrl_variant ("sampler_split_gran") (x skyrl_variant ("sampler_split_nt") with SWEEP_NT) at 64 and 128 rows x V = 151,936 bf16 (normal(0, 3) logits),
T = 1 and greedy. Interleaved rounds of 200 back-to-back launches through TokenSampler.step_ptr
(one foreign call per launch: ops.sample's Python checks cost ~15 us a call, more than a 64-row
launch), medians (us); tokens must not depend on the shape (the split partials fold exactly).
Prints one JSON line.
Run (GPU): python scripts/probe/sampler_split_sweep.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import _ffi  # noqa: E402
from skyrl_amd.config import SamplingParams  # noqa: E402
from skyrl_amd.sampler import TokenSampler  # noqa: E402

WGS = [int(v) for v in os.environ.get("SWEEP_WGS", "512,1024,2048").split(",")]
GRAN = [int(v) for v in os.environ.get("SWEEP_GRAN", "4096,8192,16384").split(",")]
NTS = [int(v) for v in os.environ.get("SWEEP_NT", "256").split(",")]


def main():
    dev = torch.device("cuda:0")
    V = 151936
    big = torch.empty((128, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    sh = torch.cuda.current_stream(dev).cuda_stream
    samplers = {(n, temp): TokenSampler(n, V, 200, dev, SamplingParams(temperature=temp), seed=1)
                for n in (64, 128) for temp in (1.0, 0.0)}
    out, toks = {}, {}
    for rnd in range(5):
        for nt, wgs, gran in [(a, b, c) for a in NTS for b in WGS for c in GRAN]:
            _ffi.set_default_variant(sampler_split_nt=nt)
            _ffi.set_default_variant(sampler_split_wgs=wgs)
            _ffi.set_default_variant(sampler_split_gran=gran)
            for (n, temp), smp in samplers.items():
                key = f"n{n}_T{temp}_nt{nt}_wgs{wgs}_gran{gran}"
                smp.step_ptr(big.data_ptr(), V, 3, sh)
                torch.cuda.synchronize()
                toks.setdefault(f"n{n}_T{temp}", []).append(smp.tokens[3].cpu().clone())
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for t in range(200):
                    smp.step_ptr(big.data_ptr(), V, t, sh)
                b.record()
                b.synchronize()
                out.setdefault(key, []).append(a.elapsed_time(b) / 200 * 1e3)
    _ffi.set_default_variant(sampler_split_nt=256)  # the defaults
    _ffi.set_default_variant(sampler_split_wgs=1024)
    _ffi.set_default_variant(sampler_split_gran=8192)
    res = {k: round(sorted(x)[len(x) // 2], 2) for k, x in out.items()}
    res["tokens_equal"] = all(all(torch.equal(v[0], w) for w in v) for v in toks.values())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
