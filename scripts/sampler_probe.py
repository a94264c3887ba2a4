"""Runs only the sampler (greedy and T=1) so PMC passes can isolate it."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from skyrl_amd.config import SamplingParams
from skyrl_amd.sampler import TokenSampler
dev = torch.device("cuda:0")
N, V, R = 512, 151936, 1024
logits = torch.empty((N * 64, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
sh = torch.cuda.current_stream(dev).cuda_stream
for sp in (SamplingParams(temperature=0.0), SamplingParams()):
    smp = TokenSampler(N, V, R, dev, sp, seed=1)
    for t in range(20):
        smp.step_ptr(logits.data_ptr() + 2 * V * (t % 64), 64 * V, t, sh)
torch.cuda.synchronize()
print("ok")
