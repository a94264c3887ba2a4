"""T=1 sampler at 512 rows x V=151936 (bf16, resident): time per launch for a forced split
count (env SKYRL_SAMPLER_SPLITS, read once per process). The product build has no such
override: for the sweep, splits_for() in csrc/sampler.hip was temporarily patched to return
atoi(getenv("SKYRL_SAMPLER_SPLITS")) when set. Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd.config import SamplingParams  # noqa: E402
from skyrl_amd.sampler import TokenSampler  # noqa: E402

dev = torch.device("cuda:0")
N, V, R = 512, 151936, 1024
logits = torch.empty((N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
sh = torch.cuda.current_stream(dev).cuda_stream
res = {"splits": os.environ.get("SKYRL_SAMPLER_SPLITS", "auto")}
for name, sp in (("greedy", SamplingParams(temperature=0.0)), ("t1", SamplingParams())):
    smp = TokenSampler(N, V, R, dev, sp, seed=1)
    for t in range(10):
        smp.step_ptr(logits.data_ptr(), V, t, sh)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for t in range(200):
        smp.step_ptr(logits.data_ptr(), V, t % R, sh)
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) * 1e3 / 200
    res[name] = {"us": round(us, 2), "GBps": round(N * V * 2 / (us * 1e-6) / 1e9, 1)}
print(json.dumps(res), flush=True)
