"""Times probe-only variants of sample_kernel (compile-time switches in sampler.hip, never set
in the product build) against the product kernel at the bench shape, to attribute its time.

Build (CPU side):  python scripts/probe/sampler_variants.py build
Run (GPU box):     python scripts/probe/sampler_variants.py run
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")
VARIANTS = {"base": [], "nohash": ["-DSKYRL_SV_NOHASH"], "nocand": ["-DSKYRL_SV_NOCAND"],
            "nohash_nocand": ["-DSKYRL_SV_NOHASH", "-DSKYRL_SV_NOCAND"]}


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared", "-Wno-unused-function",
             "-Wno-unused-parameter"]
    for name, defs in VARIANTS.items():
        out = os.path.join(HERE, f"libsv_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, *defs, os.path.join(CSRC, "capi.hip"),
                        os.path.join(CSRC, "sampler.hip"), "-o", out], check=True)
        print("built", out)


def run():
    sys.path.insert(0, ROOT)
    import torch
    dev = torch.device("cuda:0")
    N, V = 512, 151936
    logits = torch.empty((N * 8, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(N, dtype=torch.int64, device=dev)
    tok = torch.empty(N, dtype=torch.int32, device=dev)
    lp = torch.empty(N, dtype=torch.float32, device=dev)
    libs = {k: ctypes.CDLL(os.path.join(HERE, f"libsv_{k}.so")) for k in VARIANTS}
    s = torch.cuda.current_stream(dev)
    out = {}
    for temp in (1.0,):
        for rnd in range(5):
            for k, lib in libs.items():
                lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
                ws = torch.zeros(lib.skyrl_sample_workspace_bytes(N, V), dtype=torch.uint8, device=dev)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

                def call(t):
                    rc = lib.skyrl_sample(ctypes.c_void_p(logits.data_ptr() + 2 * V * (t % 8)), 1,
                                          ctypes.c_int64(8 * V), N, V, ctypes.c_float(temp), -1, ctypes.c_float(1.0),
                                          ctypes.c_float(0.0), ctypes.c_uint64(1), ctypes.c_void_p(ids.data_ptr()),
                                          ctypes.c_int64(t), ctypes.c_void_p(tok.data_ptr()),
                                          ctypes.c_void_p(lp.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                          ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0
                call(0)
                a.record(s)
                for t in range(20):
                    call(t)
                b.record(s)
                b.synchronize()
                out.setdefault(f"T{temp}_{k}", []).append(a.elapsed_time(b) / 20 * 1e3)
    print(json.dumps({k: round(sorted(v)[len(v) // 2], 1) for k, v in out.items()}))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
