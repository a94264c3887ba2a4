"""A/B of a compile-time switch of the T > 0 sampler (sampler.hip), at 512 rows (row mode, the
bench's decode step) and 64 / 128 rows (split mode) x V = 151,936 bf16, T = 1 and T = 0.7, top_p 0.95 at T = 1 and 0.6, and min_p 0.05: one
capi.hip + sampler.hip library per value of AB_DEFINE (default SKYRL_LAZY_BAR) in AB_VALUES
(default 0,1), or one library per set of AB_SETS ("name:DEF=v,DEF2=w|name2:..."), interleaved
rounds of 200 back-to-back launches, medians; the tokens of every value must be equal (the
switches change speed only). Rows in AB_ROWS (default 64,128,512).
Build: python scripts/probe/sampler_ab.py build; run (GPU): python scripts/probe/sampler_ab.py run"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")
DEF = os.environ.get("AB_DEFINE", "SKYRL_LAZY_BAR")
ROWS = [int(v) for v in os.environ.get("AB_ROWS", "64,128,512").split(",")]
if os.environ.get("AB_SETS"):  # name:DEF=v,DEF2=w|name2:...
    SETS = {}
    for item in os.environ["AB_SETS"].split("|"):
        name, defs = item.split(":")
        SETS[name] = [f"-D{d}" for d in defs.split(",") if d]
else:
    SETS = {f"{DEF}{v}": [f"-D{DEF}={v}"] for v in os.environ.get("AB_VALUES", "0,1").split(",")}
VALS = list(SETS)


def lib_path(v):
    return os.path.join(HERE, f"libab_{v}.so")


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared", "-Wno-unused-function",
             "-Wno-unused-parameter"]
    for v in VALS:
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, *SETS[v], os.path.join(CSRC, "capi.hip"),
                        os.path.join(CSRC, "sampler.hip"), "-o", lib_path(v)], check=True)
        print("built", lib_path(v))


def run():
    sys.path.insert(0, ROOT)
    import torch
    dev = torch.device("cuda:0")
    V = 151936
    big = torch.empty((512, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(512, dtype=torch.int64, device=dev)
    tok = torch.empty(512, dtype=torch.int32, device=dev)
    lp = torch.empty(512, dtype=torch.float32, device=dev)
    libs = {v: ctypes.CDLL(lib_path(v)) for v in VALS}
    s = torch.cuda.current_stream(dev)
    out, toks = {}, {}
    for rnd in range(5):
        for v, lib in libs.items():
            lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
            for n in ROWS:
                ws = torch.zeros(lib.skyrl_sample_workspace_bytes(n, V), dtype=torch.uint8, device=dev)
                for temp, top_p, min_p in ((1.0, 1.0, 0.0), (0.7, 1.0, 0.0), (1.0, 0.95, 0.0), (0.6, 0.95, 0.0), (1.0, 1.0, 0.05)):
                    def call(t):
                        rc = lib.skyrl_sample(ctypes.c_void_p(big.data_ptr()), 1, ctypes.c_int64(V), n, V,
                                              ctypes.c_float(temp), -1, ctypes.c_float(top_p), ctypes.c_float(min_p),
                                              ctypes.c_uint64(1), ctypes.c_void_p(ids.data_ptr()), ctypes.c_int64(t),
                                              ctypes.c_void_p(tok.data_ptr()), ctypes.c_void_p(lp.data_ptr()),
                                              ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(s.cuda_stream))
                        assert rc == 0
                    call(3)
                    torch.cuda.synchronize()
                    toks.setdefault(f"n{n}_T{temp}_p{top_p}_m{min_p}", {})[v] = tok[:n].cpu().clone()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    for t in range(200):
                        call(t)
                    b.record(s)
                    b.synchronize()
                    out.setdefault(f"n{n}_T{temp}_p{top_p}_m{min_p}_{v}", []).append(a.elapsed_time(b) / 200 * 1e3)
    res = {k: round(sorted(x)[len(x) // 2], 2) for k, x in out.items()}
    res["tokens_equal"] = all(all(torch.equal(d[VALS[0]], d[v]) for v in VALS) for d in toks.values())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
