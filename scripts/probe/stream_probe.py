"""Build + run the streaming-floor probe on the GPU box (measurement only)."""
import ctypes, os, statistics, subprocess, sys
import torch
here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "libprobe.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                       os.path.join(here, "stream_probe.hip"), "-o", so])
lib = ctypes.CDLL(so)
dev = torch.device("cuda:0")
N, V = 512, 151936
x = torch.empty((N * 64, V), dtype=torch.bfloat16, device=dev).normal_()  # 10 GB: every launch reads new data
out = torch.zeros(N, dtype=torch.int32, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
def run(mode, ld_rows):
    def f(t=[0]):
        t[0] += 1
        lib.probe(ctypes.c_void_p(x.data_ptr() + 2 * V * (t[0] % ld_rows)), ctypes.c_int64(ld_rows * V), N, V, mode,
                  ctypes.c_void_p(out.data_ptr()), st)
    for _ in range(5): f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        a.record(); [f() for _ in range(50)]; b.record(); b.synchronize(); ts.append(a.elapsed_time(b) / 50)
    return statistics.median(ts)
for mode, name in ((0, "512thr_row"), (1, "256thr_4split"), (2, "1024thr_row")):
    ms = run(mode, 64)
    print(name, f"{ms*1e3:.1f} us", f"{N*V*2/ms/1e6:.0f} GB/s")
# read+write ceiling: 5 GB copy (the fused training pass's traffic shape)
n = 16 * 1024 * V  # bf16 elements per micro-batch of dlogits
src = x.view(-1)[:n]
dst = torch.empty(n, dtype=torch.bfloat16, device=dev)
for nts in (0, 1):
    for blocks in (4096, 16384):
        def g():
            lib.probe_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), ctypes.c_int64(n // 8), nts,
                           blocks, st)
        g()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); [g() for _ in range(5)]; b.record(); b.synchronize()
        ms = a.elapsed_time(b) / 5
        print(f"copy nts={nts} blocks={blocks}", f"{ms:.3f} ms", f"{2 * n * 2 / ms / 1e6:.0f} GB/s")
