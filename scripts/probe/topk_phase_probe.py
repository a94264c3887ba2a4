"""Where does the one-pass top_k sampler (sample_topk_kernel, 512 x 151,936 bf16, top_k 50,
top_p 0.9) spend its time? Build with `python scripts/probe/sampler_phase_probe.py build` (the
same phase-stamp build of sampler.hip), run here with `run`: median per-workgroup spans of the
prologue (first loads + radix select of the bound), the pass, the on-chip selection and the
filters + decision, and the spread of the workgroup end times (us)."""
import ctypes
import json
import os
import sys

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(here))
SO = os.path.join(here, "libsphase.so")


def run():
    import torch
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

    def launch(i):
        rc = lib.skyrl_sample(P(logits[i % 4].data_ptr()), 1, ctypes.c_int64(V), N, V, ctypes.c_float(1.0), 50,
                              ctypes.c_float(0.9), ctypes.c_float(0.0), ctypes.c_uint64(1), P(ids.data_ptr()),
                              ctypes.c_int64(i), P(tok.data_ptr()), P(lp.data_ptr()), P(ws.data_ptr()), st)
        assert rc == 0

    buf = np.zeros(4096 * 8, dtype=np.uint64)
    for i in range(6):
        launch(i)
    torch.cuda.synchronize()
    for rep in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        launch(10 + rep)
        b.record()
        torch.cuda.synchronize()
        assert lib.probe_read(buf.ctypes.data_as(P), ctypes.c_size_t(buf.nbytes)) == 0
        t = buf.reshape(-1, 8)[:N].astype(np.int64)
        t0 = t[:, 0].min()
        rel = (t[:, :6] - t0) / 100.0
        med = lambda a, b: round(float(np.median(rel[:, b] - rel[:, a])), 2)  # noqa: E731
        print(json.dumps({"event_us": round(a.elapsed_time(b) * 1e3, 1), "span_us": round(float(rel[:, 4].max()), 2),
                          "start_p50_max": [round(float(np.median(rel[:, 0])), 2), round(float(rel[:, 0].max()), 2)],
                          "prologue_bound": med(0, 1), "pass": med(1, 2), "wave_join": med(2, 5), "select_radix": med(5, 3), "compact_rank_filter_decide": med(3, 4),
                          "wg_total_p50": med(0, 4),
                          "end_p10_p50_p90_max": [round(float(np.percentile(rel[:, 4], q)), 2) for q in (10, 50, 90, 100)]}),
              flush=True)


if __name__ == "__main__":
    run()
