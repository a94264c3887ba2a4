"""Where does a row-mode sampler launch (512 x 151,936 bf16) spend its time? Build on the CPU side
with `python scripts/probe/sampler_phase_probe.py build`, run on the GPU box with `... run`:
prints the launch span, the dispatch skew of the workgroups, the median per-workgroup phase
spans and the spread of the workgroup end times (us)."""
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
    N, V = 512, 151936
    logits = torch.empty((4, N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(N, dtype=torch.int64, device=dev)
    tok = torch.empty(N, dtype=torch.int32, device=dev)
    lp = torch.empty(N, dtype=torch.float32, device=dev)
    lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
    ws = torch.zeros(lib.skyrl_sample_workspace_bytes(N, V), dtype=torch.uint8, device=dev)
    P = ctypes.c_void_p
    st = P(torch.cuda.current_stream().cuda_stream)

    def launch(i, temp):
        rc = lib.skyrl_sample(P(logits[i % 4].data_ptr()), 1, ctypes.c_int64(V), N, V, ctypes.c_float(temp), -1,
                              ctypes.c_float(1.0), ctypes.c_float(0.0), ctypes.c_uint64(1), P(ids.data_ptr()),
                              ctypes.c_int64(i), P(tok.data_ptr()), P(lp.data_ptr()), P(ws.data_ptr()), st)
        assert rc == 0

    buf = np.zeros(4096 * 8, dtype=np.uint64)
    out = {}
    for temp, var in ((1.0, 0), (1.0, 1), (0.0, 0), (0.0, 1)):
        lib.probe_set_row(var)
        for i in range(6):
            launch(i, temp)
        torch.cuda.synchronize()
        for rep in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(10 + rep, temp)
            b.record()
            torch.cuda.synchronize()
            assert lib.probe_read(buf.ctypes.data_as(P), ctypes.c_size_t(buf.nbytes)) == 0
            t = buf.reshape(-1, 8)[:N].astype(np.int64)
            t0 = t[:, 0].min()
            rel = (t[:, :5] - t0) / 100.0
            med = lambda a, b: round(float(np.median(rel[:, b] - rel[:, a])), 2)  # noqa: E731
            cu = t[:, 7]
            rec = {"event_us": round(a.elapsed_time(b) * 1e3, 1), "span_us": round(float(rel[:, 4].max()), 2),
                   "start_skew_p50_p100": [round(float(np.median(rel[:, 0])), 2), round(float(rel[:, 0].max()), 2)],
                   "first_iter_and_seed": med(0, 1), "stream_wave0": med(1, 2), "wave_join": med(2, 3),
                   "merge_to_write": med(3, 4), "wg_total_p50": med(0, 4),
                   "end_p10_p50_p90_max": [round(float(np.percentile(rel[:, 4], q)), 2) for q in (10, 50, 90, 100)],
                   "wgs_per_cu_max": int(np.bincount(cu.astype(np.int64)).max()), "cus": int(len(np.unique(cu)))}
            xcc = t[:, 6] & 0xF
            rec["end_median_by_xcc"] = {int(x): round(float(np.median(rel[xcc == x, 4])), 2) for x in np.unique(xcc)}
            rec["end_max_by_xcc"] = {int(x): round(float(rel[xcc == x, 4].max()), 2) for x in np.unique(xcc)}
            # the two workgroups sharing a CU: end-time difference
            pairs = []
            key = xcc * 1000 + cu
            for k in np.unique(key):
                e = np.sort(rel[key == k, 4])
                if len(e) == 2:
                    pairs.append(e[1] - e[0])
            rec["cu_pair_end_gap_p50_p90"] = [round(float(np.median(pairs)), 2), round(float(np.percentile(pairs, 90)), 2)] if pairs else None
            rec["blockid_mod8_end_median"] = {int(m): round(float(np.median(rel[np.arange(N) % 8 == m, 4])), 2) for m in range(8)}
            out.setdefault(f"T{temp}_v{var}", []).append(rec)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
