"""Sampler per launch at the per-rank row counts of a strong-scaling job (512 / N rows x V =
151,936 bf16, rows R*V apart as in the bench's resident logits, T = 1 and greedy): 200
back-to-back launches eager (host-issued through TokenSampler.step_ptr) and the same 200
launches replayed from a HIP graph (no host issue cost). Run under rocprofv3 --kernel-trace
--stats for the kernels' own durations. Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd.config import SamplingParams  # noqa: E402
from skyrl_amd.sampler import TokenSampler  # noqa: E402

dev = torch.device("cuda:0")
V, R = 151936, 64
rows_list = [int(x) for x in os.environ.get("ROWS", "64,128,256,512").split(",")]
reps = 200
out = {}
big = torch.empty((max(rows_list) * R, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
for nseq in rows_list:
    lg = big[: nseq * R]
    for name, sp in (("t1", SamplingParams()), ("greedy", SamplingParams(temperature=0.0))):
        smp = TokenSampler(nseq, V, R, dev, sp, seed=1)
        sh = torch.cuda.current_stream(dev).cuda_stream

        def launches(n, stream_handle):
            for t in range(n):
                smp.step_ptr(lg.data_ptr() + 2 * V * (t % R), R * V, t % R, stream_handle)

        launches(10, sh)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        launches(reps, sh)
        b.record()
        b.synchronize()
        eager = a.elapsed_time(b) * 1e3 / reps
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
        graph = a.elapsed_time(b) * 1e3 / (3 * reps)
        nbytes = nseq * V * 2
        out[f"{nseq}_{name}"] = {"eager_us": round(eager, 2), "graph_us": round(graph, 2),
                                 "graph_TBps": round(nbytes / (graph * 1e-6) / 1e12, 2)}
        del g
print(json.dumps(out), flush=True)
