"""Copy bandwidth vs working-set size (read+write bytes counted), to place the guide's 6.29 TB/s
float4-copy figure: at what size does a copy reach it on this box? Measurement only."""
import ctypes
import os
import subprocess

import torch

here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "librw_probe.so")  # built on the CPU side: this script with --build
if "--build" in os.sys.argv or not os.path.exists(so):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                           os.path.join(here, "rw_probe.hip"), "-o", so])
    if "--build" in os.sys.argv:
        raise SystemExit(0)
lib = ctypes.CDLL(so)
dev = torch.device("cuda:0")
V = 151936
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for rows in (64, 256, 1024, 4096, 16384):
    x = torch.empty(rows * V, dtype=torch.bfloat16, device=dev).normal_()
    y = torch.empty_like(x)
    nbytes = 2 * rows * V * 2
    iters = max(5, int(2e10 // nbytes))
    for mode, param in ((0, 16384), (0, 4096)):
        f = lambda: lib.rw_probe(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),  # noqa: E731
                                 ctypes.c_int64(rows), V, mode, param, 1, st)
        f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            f()
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / iters
        print(f"rows={rows} ({nbytes / 2**20:.0f} MiB rd+wr) mode={mode} param={param}: {ms * 1e3:.1f} us "
              f"{nbytes / ms / 1e6:.0f} GB/s", flush=True)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        y.copy_(x)
    b.record()
    b.synchronize()
    print(f"rows={rows} torch copy_: {nbytes / (a.elapsed_time(b) / iters) / 1e6:.0f} GB/s", flush=True)
    del x, y
