"""Read+write ceiling probe: what structure reaches the highest copy bandwidth for the fused
training pass's traffic (16 x 1024 rows of V bf16 read, the same written). Measurement only."""
import ctypes
import os
import subprocess

import torch

here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join("/tmp", "librw_probe.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                       os.path.join(here, "rw_probe.hip"), "-o", so])
lib = ctypes.CDLL(so)
dev = torch.device("cuda:0")
V, rows = 151936, 16 * 1024
x = torch.empty(rows * V, dtype=torch.bfloat16, device=dev).normal_()
y = torch.empty_like(x)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
nbytes = 2 * rows * V * 2


def run(mode, param, nts, iters=5):
    def f():
        rc = lib.rw_probe(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_int64(rows), V, mode,
                          param, nts, st)
        assert rc == 0, rc
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        f()
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / iters
    print(f"mode={mode} param={param} nts={nts}: {ms:.3f} ms {nbytes / ms / 1e6:.0f} GB/s", flush=True)


for nts in (1, 0):
    for blocks in (2048, 4096, 16384):
        run(3, blocks, nts)
        run(0, blocks, nts)
        run(4, blocks, nts)
    run(1, 768, nts)
    run(1, 1024, nts)
    run(2, 384, nts)
    run(2, 256, nts)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(5):
    y.copy_(x)
b.record()
b.synchronize()
print(f"torch copy_: {nbytes / (a.elapsed_time(b) / 5) / 1e6:.0f} GB/s")
