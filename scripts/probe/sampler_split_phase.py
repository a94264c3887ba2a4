"""Where does a split-mode sampler launch (few rows x 151,936 bf16, each row cut over several
workgroups, the last arriver folding) spend its time? Probe build of sampler.hip
(SKYRL_SAMPLER_PHASE_PROBE: s_memrealtime per workgroup at entry, after the first iteration +
seeding, end of wave 0's stream, after the block fold, after the arrival, and before the token
write in the last arriver). `python scripts/probe/sampler_split_phase.py build` here, `... run`
on the GPU box. Prints one JSON object (us)."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(here))
SO = os.path.join(here, "libsphase.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                           "-Wno-unused-function", "-Wno-unused-parameter",
                           os.path.join(here, "sampler_phase_probe.hip"), "-o", SO])
    print("built", SO)


def run():
    import torch
    sys.path.insert(0, ROOT)
    lib = ctypes.CDLL(SO, mode=ctypes.RTLD_LOCAL)
    dev = torch.device("cuda:0")
    V = 151936
    P = ctypes.c_void_p
    st = P(torch.cuda.current_stream().cuda_stream)
    lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
    out = {}
    for N in [int(x) for x in os.environ.get("ROWS", "64,128").split(",")]:
        logits = torch.empty((4, N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
        ids = torch.arange(N, dtype=torch.int64, device=dev)
        tok = torch.empty(N, dtype=torch.int32, device=dev)
        lp = torch.empty(N, dtype=torch.float32, device=dev)
        ws = torch.zeros(lib.skyrl_sample_workspace_bytes(N, V), dtype=torch.uint8, device=dev)
        buf = np.zeros(4096 * 8, dtype=np.uint64)
        for temp in (1.0, 0.0):
            def launch(i):
                rc = lib.skyrl_sample(P(logits[i % 4].data_ptr()), 1, ctypes.c_int64(V), N, V, ctypes.c_float(temp),
                                      -1, ctypes.c_float(1.0), ctypes.c_float(0.0), ctypes.c_uint64(1),
                                      P(ids.data_ptr()), ctypes.c_int64(i), P(tok.data_ptr()), P(lp.data_ptr()),
                                      P(ws.data_ptr()), st)
                assert rc == 0
            for i in range(6):
                launch(i)
            torch.cuda.synchronize()
            recs = []
            for rep in range(4):
                buf[:] = 0
                assert lib.probe_clear() == 0
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                launch(10 + rep)
                b.record()
                torch.cuda.synchronize()
                assert lib.probe_read(buf.ctypes.data_as(P), ctypes.c_size_t(buf.nbytes)) == 0
                t = buf.reshape(-1, 8).astype(np.int64)
                live = t[:, 0] > 0
                t = t[live]
                t0 = t[:, 0].min()
                rel = (t[:, :6] - t0) / 100.0
                last = t[:, 4] > 0
                pct = lambda x: [round(float(np.percentile(x, q)), 2) for q in (10, 50, 90, 100)]  # noqa: E731
                recs.append({
                    "event_us": round(a.elapsed_time(b) * 1e3, 2), "wgs": int(live.sum()),
                    "entry_p10_p50_p90_max": pct(rel[:, 0]),
                    "first_iter_seed_p50": round(float(np.median(rel[:, 1] - rel[:, 0])), 2),
                    "stream_p50": round(float(np.median(rel[:, 2] - rel[:, 1])), 2),
                    "block_fold_p50": round(float(np.median(rel[:, 3] - rel[:, 2])), 2),
                    "store_arrive_p50": round(float(np.median(rel[:, 5] - rel[:, 3])), 2),
                    "arrive_p10_p50_p90_max": pct(rel[:, 5]),
                    "last_merge_p50": round(float(np.median(rel[last, 4] - rel[last, 5])), 2),
                    "token_write_max": round(float(rel[last, 4].max()), 2),
                    "wg_total_p50": round(float(np.median(rel[:, 5] - rel[:, 0])), 2)})
            out[f"{N}_T{temp}"] = recs
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
