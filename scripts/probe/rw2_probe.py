"""Read / write / copy ceiling probe, second pass (scripts/probe/rw2_probe.hip). Measurement only.
Bytes counted: read-only n*16, write-only n*16, copies 2*n*16."""
import ctypes
import os
import subprocess

import torch

here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join("/tmp", "librw2_probe.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                       os.path.join(here, "rw2_probe.hip"), "-o", so])
lib = ctypes.CDLL(so)
dev = torch.device("cuda:0")
V, rows = 151936, 16 * 1024
x = torch.empty(rows * V, dtype=torch.bfloat16, device=dev).normal_()
y = torch.empty_like(x)
sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
nvec = rows * V // 8


def run(mode, param, nts, iters=5, label=""):
    def f():
        rc = lib.rw2_probe(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_int64(rows), V,
                           mode, param, nts, ctypes.c_void_p(sink.data_ptr()), st)
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
    nbytes = nvec * 16 * (1 if mode in (0, 1) else 2)
    print(f"{label:28s} mode={mode} param={param} nts={nts}: {ms:.3f} ms {nbytes / ms / 1e6:.0f} GB/s", flush=True)


import sys
EPOCH = [1]
if len(sys.argv) > 1 and sys.argv[1] == "split":
    def run_split(mode, nts, iters=5, label=""):
        def f():
            EPOCH[0] += 1
            rc = lib.rw2_probe(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_int64(rows), V,
                               mode, EPOCH[0], nts, ctypes.c_void_p(sink.data_ptr()), st)
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
        print(f"{label:28s} mode={mode} nts={nts}: {ms:.3f} ms {nvec * 32 / ms / 1e6:.0f} GB/s", flush=True)
    for nts in (1, 0):
        run(6, 0, nts, label="resident rows")
        run_split(10, nts, label="split rows P=4 x 256")
        run_split(11, nts, label="split rows P=2 x 512")
    assert torch.equal(x, y)
    run(2, 8192, 1, label="copy out of place")
    run(4, 32, 1, label="chunk copy")
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "pipe":
    for nts in (1, 0):
        run(6, 0, nts, label="resident rows")
        for g in (256, 512):
            run(8, g, nts, label="pipelined store,load")
            run(9, g, nts, label="pipelined load,store")
    run(2, 8192, 1, label="copy out of place")
    sys.exit(0)
for blocks in (1024, 2048, 4096, 8192):
    run(0, blocks, 1, label="read only")
for blocks in (2048, 8192):
    for nts in (0, 1):
        run(1, blocks, nts, label="write only")
for blocks in (2048, 8192):
    for nts in (0, 1):
        run(2, blocks, nts, label="copy out of place")
        run(3, blocks, nts, label="copy in place")
for ch in (16, 32):
    for nts in (0, 1):
        run(4, ch, nts, label="chunk copy")
        run(5, ch, nts, label="chunk copy in place")
for nts in (0, 1):
    run(6, 0, nts, label="resident rows")
    run(7, 0, nts, label="resident rows in place")
