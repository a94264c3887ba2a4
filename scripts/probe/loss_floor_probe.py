"""Graph-node floor of the advantage+loss leg's shape (loss_floor_probe.hip); measurement only."""
import ctypes
import os
import subprocess

import torch

here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join("/tmp", "libloss_floor_probe.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                       os.path.join(here, "loss_floor_probe.hip"), "-o", so])
lib = ctypes.CDLL(so)
dev = torch.device("cuda:0")
N = 512 * 1024
t = [torch.randn(N, device=dev) for _ in range(5)]
rec = torch.zeros(8192, device=dev)
P = ctypes.c_void_p


def timed(modes, reps=20):
    side = torch.cuda.Stream(dev)

    def run():
        h = P(torch.cuda.current_stream(dev).cuda_stream)
        for m in modes:
            assert lib.floor_probe(P(t[0].data_ptr()), P(t[1].data_ptr()), P(t[2].data_ptr()), P(t[3].data_ptr()),
                                   P(t[4].data_ptr()), P(rec.data_ptr()), m, h) == 0
    with torch.cuda.stream(side):
        run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for _ in range(reps):
            run()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / (5 * reps), 2)


for rep in range(2):
    for name, modes in (("empty", (0,)), ("load4_store1", (1,)), ("load4_store1_records", (2,)),
                        ("fold_1block", (3,)), ("records+fold", (2, 3)), ("empty+empty", (0, 0))):
        print(f"{name}: {timed(modes)} us", flush=True)
