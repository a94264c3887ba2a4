"""Attributes pass 1 of the one-pass top_p kernel (sample_topp_kernel) at the bench shape
[512, 151,936] bf16, T = 1, top_p = 0.95: probe-only builds of capi.hip + sampler.hip with
compile-time switches (never set in the product) and skyrl_variant's topp_probe = 1 as the default
(pass 1 alone): the LDS count histogram removed (nohist), the recorded race removed (norace),
both (neither), the race without its LDS records (norec), against the unchanged pass 1 (base) and the unfiltered T = 1 kernel (one read of
the row). Interleaved rounds in one process; medians.

Build (CPU side):  python scripts/probe/topp_variants.py build
Run (GPU box):     python scripts/probe/topp_variants.py run
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")
VARIANTS = {"base": [], "nohist": ["-DSKYRL_TP_NOHIST"], "norace": ["-DSKYRL_TP_NORACE"],
            "neither": ["-DSKYRL_TP_NOHIST", "-DSKYRL_TP_NORACE"], "norec": ["-DSKYRL_TP_NOREC"]}


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared", "-Wno-unused-function",
             "-Wno-unused-parameter", "-DSKYRL_TP_PROBE0=1"]
    for name, defs in VARIANTS.items():
        out = os.path.join(HERE, f"libtp_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, *defs, os.path.join(CSRC, "capi.hip"),
                        os.path.join(CSRC, "sampler.hip"), "-o", out], check=True)
        print("built", out)


def run():
    sys.path.insert(0, ROOT)
    import torch
    dev = torch.device("cuda:0")
    N, V = 512, 151936
    logits = torch.empty((N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(N, dtype=torch.int64, device=dev)
    tok = torch.empty(N, dtype=torch.int32, device=dev)
    lp = torch.empty(N, dtype=torch.float32, device=dev)
    libs = {k: ctypes.CDLL(os.path.join(HERE, f"libtp_{k}.so")) for k in VARIANTS}
    s = torch.cuda.current_stream(dev)
    out = {}
    for rnd in range(7):
        for k, lib in libs.items():
            lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
            ws = torch.zeros(lib.skyrl_sample_workspace_bytes(N, V), dtype=torch.uint8, device=dev)
            for name, top_p in (("top_p0.95", 0.95), ("unfiltered", 1.0)):
                if name == "unfiltered" and k != "base":
                    continue
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

                def call(t):
                    rc = lib.skyrl_sample(ctypes.c_void_p(logits.data_ptr()), 1, ctypes.c_int64(V), N, V,
                                          ctypes.c_float(1.0), -1, ctypes.c_float(top_p), ctypes.c_float(0.0),
                                          ctypes.c_uint64(1), ctypes.c_void_p(ids.data_ptr()), ctypes.c_int64(t),
                                          ctypes.c_void_p(tok.data_ptr()), ctypes.c_void_p(lp.data_ptr()),
                                          ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0
                call(0)
                a.record(s)
                for t in range(20):
                    call(t)
                b.record(s)
                b.synchronize()
                out.setdefault(f"{name}_{k}", []).append(a.elapsed_time(b) / 20 * 1e3)
    print(json.dumps({k: round(sorted(v)[len(v) // 2], 2) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
