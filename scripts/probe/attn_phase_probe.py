"""Per-wave timeline of the paged decode kernel on the ragged rollout mix vs uniform contexts.
Build on the CPU side with `python scripts/probe/attn_phase_probe.py build`, run on the GPU box
with `... run`. For each case prints: launch span, entry skew, first-block latency, per-wave
token rate (early vs late waves), the number of live waves over time, and per-CU work vs end
time. One JSON line per case. Probe only."""
import ctypes
import json
import math
import os
import subprocess
import sys

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(here))
SO = os.path.join(here, "libaphase.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                           "-Wno-unused-function", "-Wno-unused-parameter",
                           os.path.join(here, "attn_phase_probe.hip"), "-o", SO])
    print("built", SO)


def run():
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, here)
    from attn_chunk_sweep import D, NH, NKV, setup

    lib = ctypes.CDLL(SO, mode=ctypes.RTLD_LOCAL)
    lib.skyrl_paged_decode_workspace_bytes.restype = ctypes.c_size_t
    dev = torch.device("cuda:0")
    P = ctypes.c_void_p
    buf = np.zeros(8192 * 8, dtype=np.uint64)
    cases = [("ragged_np1", (512, 17, 1536), 1, 64), ("uniform_np1", (512, 1280, 1280), 1, 64),
             ("ragged_c512", (512, 17, 1536), 3, 512), ("ragged_c256", (512, 17, 1536), 6, 256)]
    for name, shape, nparts, pmin in cases:
        q, kc, vc, bt, ctx, max_ctx = setup(dev, *shape)
        nseq = q.shape[0]
        out = torch.empty_like(q)
        ws = torch.empty(max(16, lib.skyrl_paged_decode_workspace_bytes(nseq, NH, D, nparts)), dtype=torch.uint8,
                         device=dev)
        st = P(torch.cuda.current_stream().cuda_stream)

        def launch():
            rc = lib.skyrl_paged_decode(P(q.data_ptr()), ctypes.c_int64(q.stride(0)), P(kc.data_ptr()),
                                        P(vc.data_ptr()), P(bt.data_ptr()), ctypes.c_int64(bt.stride(0)),
                                        P(ctx.data_ptr()), nseq, NH, NKV, D, ctypes.c_float(1 / math.sqrt(D)), pmin,
                                        nparts, P(out.data_ptr()), ctypes.c_int64(out.stride(0)),
                                        P(ws.data_ptr()) if nparts > 1 else None, st)
            assert rc == 0

        for _ in range(10):
            launch()
        torch.cuda.synchronize()
        for rep in range(2):
            assert lib.probe_clear() == 0
            torch.cuda.synchronize()
            for _ in range(20):  # warm: the buffer keeps the last launch's stamps
                launch()
            torch.cuda.synchronize()
            assert lib.probe_read(buf.ctypes.data_as(P), ctypes.c_size_t(buf.nbytes)) == 0
            t = buf.reshape(-1, 8).astype(np.int64)
            live = t[:, 0] != 0
            t = t[live]
            t0 = t[:, 0].min()
            us = lambda x: (x - t0) / 100.0  # noqa: E731
            start, first, end = us(t[:, 0]), us(t[:, 1]), us(t[:, 2])
            tokens = t[:, 6]
            cu = (t[:, 7] & 0xffffffff) | ((t[:, 7] >> 32) << 16)  # (xcc, cu) key
            dur = end - start
            rate = tokens / np.maximum(dur, 1e-3)  # tokens per us per wave
            span = float(end.max())
            grid = np.linspace(0, span, 21)
            livewaves = [int(((start <= x) & (end > x)).sum()) for x in grid[:-1]]
            bytes_tok = NKV * D * 4 / NKV  # K+V bytes per token per kv head
            live_bytes = [float(tokens[(start <= x) & (end > x)].sum()) for x in grid[:-1]]
            keys, inv = np.unique(cu, return_inverse=True)
            cu_tokens = np.bincount(inv, weights=tokens)
            cu_end = np.zeros(len(keys))
            np.maximum.at(cu_end, inv, end)
            long_ = tokens >= np.percentile(tokens, 90)
            rec = {"case": name, "rep": rep, "waves": int(len(t)), "span_us": round(span, 2),
                   "entry_skew_us": round(float(start.max()), 2),
                   "first_block_us_p50": round(float(np.median(first - start)), 2),
                   "first_block_us_p90": round(float(np.percentile(first - start, 90)), 2),
                   "wave_end_us_p10_p50_p90": [round(float(np.percentile(end, q_)), 2) for q_ in (10, 50, 90)],
                   "long_waves_rate_tok_per_us_p50": round(float(np.median(rate[long_])), 2),
                   "long_waves_dur_us_p50": round(float(np.median(dur[long_])), 2),
                   "all_waves_rate_p50": round(float(np.median(rate)), 2),
                   "live_waves_over_time": livewaves,
                   "live_MB_over_time": [round(b * bytes_tok / 1e6, 1) for b in live_bytes],
                   "cus": int(len(keys)),
                   "cu_tokens_p10_p50_p90_max": [round(float(np.percentile(cu_tokens, q_))) for q_ in (10, 50, 90, 100)],
                   "cu_end_us_p10_p50_p90_max": [round(float(np.percentile(cu_end, q_)), 2) for q_ in (10, 50, 90, 100)],
                   "corr_cu_tokens_end": round(float(np.corrcoef(cu_tokens, cu_end)[0, 1]), 3),
                   "xcc_tokens": [int(x) for x in np.bincount((t[:, 7] >> 32).astype(np.int64), weights=tokens)]}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
