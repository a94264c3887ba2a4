"""The split-mode sampler (rows < 256: each row over several 256-thread workgroups) built for 4
waves per SIMD (the product: 110 VGPRs, no spills) against 5 (96 VGPRs, a few spills), at the
per-rank batch sizes of a strong-scaling job (64 / 128 rows x V = 151,936 bf16, T = 1 and greedy):
one capi.hip + sampler.hip library per setting, interleaved rounds of 200 back-to-back launches,
medians. Build: python scripts/probe/split_wpe.py build; run (GPU): ... run."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")
WPE = (4, 5)


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared", "-Wno-unused-function",
             "-Wno-unused-parameter"]
    for w in WPE:
        out = os.path.join(HERE, f"libwpe{w}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, f"-DSKYRL_SPLIT_WPE={w}", os.path.join(CSRC, "capi.hip"),
                        os.path.join(CSRC, "sampler.hip"), "-o", out], check=True)
        print("built", out)


def run():
    sys.path.insert(0, ROOT)
    import torch
    dev = torch.device("cuda:0")
    V = 151936
    big = torch.empty((128, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(128, dtype=torch.int64, device=dev)
    tok = torch.empty(128, dtype=torch.int32, device=dev)
    lp = torch.empty(128, dtype=torch.float32, device=dev)
    libs = {w: ctypes.CDLL(os.path.join(HERE, f"libwpe{w}.so")) for w in WPE}
    s = torch.cuda.current_stream(dev)
    out = {}
    for rnd in range(5):
        for w, lib in libs.items():
            lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
            for n in (64, 128):
                ws = torch.zeros(lib.skyrl_sample_workspace_bytes(n, V), dtype=torch.uint8, device=dev)
                for temp in (1.0, 0.0):
                    def call(t):
                        rc = lib.skyrl_sample(ctypes.c_void_p(big.data_ptr()), 1, ctypes.c_int64(V), n, V,
                                              ctypes.c_float(temp), -1, ctypes.c_float(1.0), ctypes.c_float(0.0),
                                              ctypes.c_uint64(1), ctypes.c_void_p(ids.data_ptr()), ctypes.c_int64(t),
                                              ctypes.c_void_p(tok.data_ptr()), ctypes.c_void_p(lp.data_ptr()),
                                              ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(s.cuda_stream))
                        assert rc == 0
                    for t in range(5):
                        call(t)
                    ref = tok[:n].clone()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    for t in range(200):
                        call(t)
                    b.record(s)
                    b.synchronize()
                    out.setdefault(f"n{n}_T{temp}_wpe{w}", []).append(a.elapsed_time(b) / 200 * 1e3)
                    out.setdefault(f"n{n}_T{temp}_wpe{w}_tok", []).append(int(ref.sum()))
    res = {k: (round(sorted(v)[len(v) // 2], 2) if not k.endswith("_tok") else v[0]) for k, v in out.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
