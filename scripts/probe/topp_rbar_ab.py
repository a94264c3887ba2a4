"""A/B of the top_p kernel's pass-1 bar (csrc/sampler.hip SKYRL_TP_RBAR) at the bench shape
[512, 151,936] bf16: R = 1 the best exact score so far (r05 product), R > 1 the R-th largest of
the waves' best scores (pass 1 certifies unless the row's R best elements are all cut). Probe
builds of capi.hip + sampler.hip; per variant: the mean time of both launches over decode steps
0..19 (fresh noise per step), the rows left to pass 2, and the tokens / logprobs against R = 1.

Build (CPU side):  python scripts/probe/topp_rbar_ab.py build
Run (GPU box):     python scripts/probe/topp_rbar_ab.py run
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")
P, ML = "-DSKYRL_TP_PROBE0=2", "-DSKYRL_MP_LIST=1"
# r1: the product as built (the exactness reference); ml: min_p alone decided from pass 1's list of
# the elements within T |ln min_p| of the running max (SKYRL_MP_LIST); p2: pass 1 + the cut alone
VARIANTS = {"r1": [], "ml": [ML], "r1p2": [P], "mlp2": [ML, P]}
CASES = {"minp0.05_T1": (1.0, 1.0, 0.05), "minp0.05_T0.6": (0.6, 1.0, 0.05), "minp0.1_T1": (1.0, 1.0, 0.1),
         "p0.95_minp0.05_T1": (1.0, 0.95, 0.05)}
FILT = 1024 * 4  # the RowFilter array's offset (sampler.hip kCounterBytes); RowFilter = 5 x 4 B


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared", "-Wno-unused-function",
             "-Wno-unused-parameter"]
    procs = []
    for name, defs in VARIANTS.items():
        out = os.path.join(HERE, f"libtprb_{name}.so")
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", *flags, *defs, os.path.join(CSRC, "capi.hip"),
                                       os.path.join(CSRC, "sampler.hip"), "-o", out]))
    for p in procs:
        assert p.wait() == 0
    print("built", list(VARIANTS))


def run():
    import torch
    dev = torch.device("cuda:0")
    N, V = 512, 151936
    torch.manual_seed(0)
    logits = torch.empty((N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(N, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    libs = {k: ctypes.CDLL(os.path.join(HERE, f"libtprb_{k}.so")) for k in VARIANTS}
    out = {}
    for case, (temp, top_p, min_p) in CASES.items():
        ref = {}
        for rnd in range(3):
            for k, lib in libs.items():
                lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
                ws = torch.zeros(lib.skyrl_sample_workspace_bytes(N, V), dtype=torch.uint8, device=dev)
                tok = torch.empty(N, dtype=torch.int32, device=dev)
                lp = torch.empty(N, dtype=torch.float32, device=dev)

                def call(t):
                    rc = lib.skyrl_sample(ctypes.c_void_p(logits.data_ptr()), 1, ctypes.c_int64(V), N, V,
                                          ctypes.c_float(temp), -1, ctypes.c_float(top_p), ctypes.c_float(min_p),
                                          ctypes.c_uint64(3), ctypes.c_void_p(ids.data_ptr()), ctypes.c_int64(t),
                                          ctypes.c_void_p(tok.data_ptr()), ctypes.c_void_p(lp.data_ptr()),
                                          ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0
                call(0)
                times, left, same = [], [], True
                for t in range(20):
                    for _ in range(2):
                        call(t)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    for _ in range(5):
                        call(t)
                    b.record(s)
                    b.synchronize()
                    times.append(a.elapsed_time(b) / 5 * 1e3)
                    ff = ws[FILT:FILT + 20 * N].view(torch.int32).view(N, 5)
                    left.append(int((ff[:, 1] != 1).sum()))
                    if k.endswith("why") and rnd == 0:
                        for c in ff[:, 1][ff[:, 1] != 1].cpu().tolist():
                            why = out.setdefault(f"{case}_{k}_reasons", {})
                            why[str(c)] = why.get(str(c), 0) + 1
                    if rnd == 0 and not k.endswith("p2"):
                        cur = (tok.cpu().clone(), lp.cpu().clone())
                        if k == "r1":
                            ref[t] = cur
                        else:
                            same &= bool(torch.equal(cur[0], ref[t][0])) and bool(
                                torch.equal(cur[1].view(torch.int32), ref[t][1].view(torch.int32)))
                rec = out.setdefault(f"{case}_{k}", {"us": [], "rows_left": left})
                if k.endswith("p2") and rnd == 0:  # (COUNT builds) per-row means of the last step
                    rec["events_per_row"] = round(float(tok.float().mean()), 1)
                    rec["scores_per_row"] = round(float(lp.mean()), 1)
                rec["us"].append(round(sum(times) / len(times), 2))
                if not k.endswith("p2"):  # mean time of the steps pass 1 decided whole / not
                    z = [x for x, n in zip(times, left) if n == 0]
                    nz = [x for x, n in zip(times, left) if n]
                    rec.setdefault("us_steps_none_left", []).append(round(sum(z) / len(z), 2) if z else None)
                    rec.setdefault("us_steps_some_left", []).append(round(sum(nz) / len(nz), 2) if nz else None)
                if rnd == 0 and k != "r1" and not k.endswith("p2"):
                    rec["bit_exact_vs_r1"] = same
        print(json.dumps({k: v for k, v in out.items() if k.startswith(case)}), flush=True)
    for name, v in out.items():
        if name.endswith("_reasons"):
            continue
        v["us_median"] = sorted(v["us"])[len(v["us"]) // 2]
        v["rows_left_mean"] = round(sum(v["rows_left"]) / len(v["rows_left"]), 2)
        v["steps_with_pass2"] = sum(1 for x in v["rows_left"] if x)
        del v["rows_left"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
