"""top_p / min_p below the row-mode batch: the one-pass kernel (one workgroup per row,
skyrl_variant ("sampler_topp_fast") = 1, the default) against the two-kernel path (filter pre-pass +
MODE 2 sampler in split mode, = 0) at 32 / 64 / 128 / 256 / 512 rows x V = 151,936 bf16
(normal(0, 3) logits). Interleaved rounds of 100 back-to-back launches through TokenSampler.step_ptr,
medians (us); the two
paths must give the same tokens. Prints one JSON line. Run (GPU): python scripts/probe/topp_rows_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import _ffi  # noqa: E402
from skyrl_amd.config import SamplingParams  # noqa: E402
from skyrl_amd.sampler import TokenSampler  # noqa: E402

ROWS = [int(v) for v in os.environ.get("ROWS", "32,64,128,256,512").split(",")]
CASES = [(1.0, 0.95, 0.0), (0.6, 0.95, 0.0), (1.0, 1.0, 0.05)]


def main():
    dev = torch.device("cuda:0")
    V = 151936
    big = torch.empty((max(ROWS), V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    sh = torch.cuda.current_stream(dev).cuda_stream
    samplers = {(n, c): TokenSampler(n, V, 100, dev, SamplingParams(temperature=c[0], top_p=c[1], min_p=c[2]), seed=1)
                for n in ROWS for c in CASES}
    out, toks = {}, {}
    for rnd in range(5):
        for fast in (1, 0):
            _ffi.set_default_variant(sampler_topp_fast=fast)
            for (n, (temp, top_p, min_p)), smp in samplers.items():
                case = f"n{n}_T{temp}_p{top_p}_minp{min_p}"
                smp.step_ptr(big.data_ptr(), V, 3, sh)
                torch.cuda.synchronize()
                toks.setdefault(case, {})[fast] = smp.tokens[3].cpu().clone()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for t in range(100):
                    smp.step_ptr(big.data_ptr(), V, t, sh)
                b.record()
                b.synchronize()
                out.setdefault(f"{case}_fast{fast}", []).append(a.elapsed_time(b) / 100 * 1e3)
    _ffi.set_default_variant(sampler_topp_fast=1)
    res = {k: round(sorted(x)[len(x) // 2], 2) for k, x in out.items()}
    res["tokens_equal"] = all(torch.equal(d[0], d[1]) for d in toks.values())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
