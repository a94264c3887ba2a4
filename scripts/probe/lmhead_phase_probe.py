"""Where does a fused lm_head + sampler tile (512 x 151,936 x 1536) spend its time? Build on the CPU
side with `python scripts/probe/lmhead_phase_probe.py build`, run on the GPU box with `... run`:
median per-tile spans of the K loop, the image write, sampler pass 1, the candidate evaluation
and the fold, for T = 1 and greedy (us)."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(here))
SO = os.path.join(here, "liblphase.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                           "-Wno-unused-function", "-Wno-unused-parameter",
                           os.path.join(here, "lmhead_phase_probe.hip"), "-o", SO])
    print("built", SO)


def run():
    import torch
    lib = ctypes.CDLL(SO, mode=ctypes.RTLD_LOCAL)
    dev = torch.device("cuda:0")
    M, H, V = 512, 1536, 151936
    w = (torch.randn(V, H, device=dev) * (3.0 / H ** 0.5)).to(torch.bfloat16)
    h = torch.randn(M, H, device=dev).to(torch.bfloat16)
    tok = torch.empty(M, dtype=torch.int32, device=dev)
    lp = torch.empty(M, dtype=torch.float32, device=dev)
    lib.skyrl_lmhead_sample_workspace_bytes.restype = ctypes.c_size_t
    ws = torch.zeros(lib.skyrl_lmhead_sample_workspace_bytes(M, V), dtype=torch.uint8, device=dev)
    ids = torch.arange(M, dtype=torch.int64, device=dev)
    P = ctypes.c_void_p
    st = P(torch.cuda.current_stream().cuda_stream)
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    out = {}
    for temp in (1.0, 0.0):
        def launch(step):
            rc = lib.skyrl_lmhead_sample(P(h.data_ptr()), ctypes.c_int64(H), P(w.data_ptr()), ctypes.c_int64(H), M, V, H,
                                         ctypes.c_float(temp), ctypes.c_uint64(1), P(ids.data_ptr()), ctypes.c_int64(step),
                                         P(tok.data_ptr()), P(lp.data_ptr()), P(ws.data_ptr()), st)
            assert rc == 0
        for i in range(5):
            launch(i)
        torch.cuda.synchronize()
        for rep in range(2):
            launch(10 + rep)
            torch.cuda.synchronize()
            assert lib.probe_read(buf.ctypes.data_as(P), ctypes.c_size_t(buf.nbytes)) == 0
            ntiles = 2 * ((V + 255) // 256)
            t = buf.reshape(-1, 8)[:ntiles, :6].astype(np.int64)
            rel = (t - t[:, 0].min()) / 100.0
            med = lambda a, b: round(float(np.median(rel[:, b] - rel[:, a])), 2)  # noqa: E731
            rec = {"span_us": round(float(rel[:, 5].max()), 1), "k_loop": med(0, 1), "image": med(1, 2),
                   "epilogue_total": med(2, 5)}
            if temp > 0:
                rec.update({"pass1": med(2, 3), "candidates": med(3, 4), "fold": med(4, 5)})
            out.setdefault(f"T{temp}", []).append(rec)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
