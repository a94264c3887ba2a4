"""The T = 1 sampler with its seed (the first two vectors' exact scores and the workgroup barrier
that shares the best as the bar) before the streaming loop (SKYRL_SEED_IN_LOOP=0, r04's form)
against inside the loop's first iteration, after the next iteration's loads are issued (=1), at
512 rows (row mode, the bench's decode step) and 64 / 128 rows (split mode): one capi.hip +
sampler.hip library per setting, interleaved rounds of 200 back-to-back launches, medians; the
tokens of both must be equal. Build: python scripts/probe/sampler_seed.py build; run (GPU): ... run."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")
WPE = (0, 1)


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared", "-Wno-unused-function",
             "-Wno-unused-parameter"]
    for w in WPE:
        out = os.path.join(HERE, f"libseed{w}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, f"-DSKYRL_SEED_IN_LOOP={w}", os.path.join(CSRC, "capi.hip"),
                        os.path.join(CSRC, "sampler.hip"), "-o", out], check=True)
        print("built", out)


def run():
    sys.path.insert(0, ROOT)
    import torch
    dev = torch.device("cuda:0")
    V = 151936
    big = torch.empty((512, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(512, dtype=torch.int64, device=dev)
    tok = torch.empty(512, dtype=torch.int32, device=dev)
    lp = torch.empty(512, dtype=torch.float32, device=dev)
    libs = {w: ctypes.CDLL(os.path.join(HERE, f"libseed{w}.so")) for w in WPE}
    s = torch.cuda.current_stream(dev)
    out = {}
    for rnd in range(5):
        for w, lib in libs.items():
            lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
            for n in (64, 128, 512):
                ws = torch.zeros(lib.skyrl_sample_workspace_bytes(n, V), dtype=torch.uint8, device=dev)
                for temp in (1.0,):
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
                    out.setdefault(f"n{n}_T{temp}_seed{w}", []).append(a.elapsed_time(b) / 200 * 1e3)
                    out.setdefault(f"n{n}_T{temp}_seed{w}_tok", []).append(int(ref.sum()))
    res = {k: (round(sorted(v)[len(v) // 2], 2) if not k.endswith("_tok") else v[0]) for k, v in out.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
