"""Sampler per launch at the per-rank row counts of a strong-scaling job (512 / N rows x V =
151,936 bf16, rows R*V apart as in the bench's resident logits, T = 1 and greedy), for each
split setting (skyrl_variant sampler_split_rows / sampler_split_wgs): 200 launches replayed from a
HIP graph (the kernels alone; EAGER=1 also times them host-issued through
TokenSampler.step_ptr). Run under rocprofv3 --kernel-trace --stats for the kernels' own
durations. Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import _ffi  # noqa: E402
from skyrl_amd.config import SamplingParams  # noqa: E402
from skyrl_amd.sampler import TokenSampler  # noqa: E402

dev = torch.device("cuda:0")
V, R = 151936, 64
rows_list = [int(x) for x in os.environ.get("ROWS", "64,128,256,512").split(",")]
settings = [tuple(int(v) for v in (s + ":8192").split(":")[:3]) for s in
            os.environ.get("SETTINGS", "256:2048,1024:1024,1024:2048,1024:4096").split(",")]
eager_too = os.environ.get("EAGER") == "1"
reps = 200
out = {}
big = torch.empty((max(rows_list) * R, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
for nseq in rows_list:
    lg = big[: nseq * R]
    for rows_thr, wgs, gran in settings:
        if rows_thr <= nseq and (rows_thr, wgs, gran) != settings[0]:
            continue  # row mode: the same kernel as the first setting's
        _ffi.set_default_variant(sampler_split_rows=rows_thr)
        _ffi.set_default_variant(sampler_split_wgs=wgs)
        _ffi.set_default_variant(sampler_split_gran=gran)
        for name, sp in (("t1", SamplingParams()), ("greedy", SamplingParams(temperature=0.0))):
            smp = TokenSampler(nseq, V, R, dev, sp, seed=1)

            def launches(n, stream_handle):
                for t in range(n):
                    smp.step_ptr(lg.data_ptr() + 2 * V * (t % R), R * V, t % R, stream_handle)

            sh = torch.cuda.current_stream(dev).cuda_stream
            launches(10, sh)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            rec = {}
            if eager_too:
                a.record()
                launches(reps, sh)
                b.record()
                b.synchronize()
                rec["eager_us"] = round(a.elapsed_time(b) * 1e3 / reps, 2)
            side = torch.cuda.Stream(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                launches(reps, torch.cuda.current_stream(dev).cuda_stream)
            g.replay()
            torch.cuda.synchronize()
            a.record()
            for _ in range(3):
                g.replay()
            b.record()
            b.synchronize()
            us = a.elapsed_time(b) * 1e3 / (3 * reps)
            rec.update(graph_us=round(us, 2), TBps=round(nseq * V * 2 / (us * 1e-6) / 1e12, 2))
            out[f"{nseq}_{name}_rows{rows_thr}_wgs{wgs}_g{gran}"] = rec
            del g
_ffi.set_default_variant(sampler_split_rows=256)
_ffi.set_default_variant(sampler_split_wgs=1024)
_ffi.set_default_variant(sampler_split_gran=8192)
print(json.dumps(out), flush=True)
