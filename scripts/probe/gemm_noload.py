"""Times the lm_head GEMM loop structures (skyrl_variant lmhead_pipe 4 vs 11) with and without
operand copies: the probe library is built with -DSKYRL_GEMM_NOLOAD (the K loop re-reads the
prologue's LDS tiles; results are garbage, timing is the loop's compute/LDS/barrier cost).

Build (CPU side, after `make -C skyrl_amd/csrc`):  python scripts/probe/gemm_noload.py build
Run (GPU box):                                     python scripts/probe/gemm_noload.py run
"""
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "skyrl_amd", "csrc")


VARIANTS = {"noload": "-DSKYRL_GEMM_NOLOAD"}


def build():
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mcode-object-version=5",
             "-Wno-unused-function", "-Wno-unused-parameter"]
    others = [o for o in glob.glob(os.path.join(ROOT, "build", "obj", "*.o")) if not o.endswith("lmhead_gemm.o")]
    for name, flag in VARIANTS.items():
        obj = f"/tmp/lmhead_gemm_{name}.o"
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, flag, "-c", os.path.join(CSRC, "lmhead_gemm.hip"), "-o", obj],
                       check=True)
        out = os.path.join(HERE, f"libgemm_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", obj, *others, "-o", out],
                       check=True)
        print("built", out)


def run():
    sys.path.insert(0, ROOT)
    import torch
    sys.argv = [sys.argv[0]]
    from skyrl_amd import _ffi
    import importlib.util
    spec = importlib.util.spec_from_file_location("lsb", os.path.join(HERE, "lmhead_sample_bench.py"))
    lsb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lsb)
    shapes = ((8192, 151936), (512, 151936))
    lsb.PIPES = (12, 14)
    print(json.dumps({"lib": "product"}), flush=True)
    lsb.gemm_sweep(shapes)
    for name in VARIANTS:
        _ffi._lib = None
        _ffi.LIB_PATH = os.path.join(HERE, f"libgemm_{name}.so")
        print(json.dumps({"lib": name}), flush=True)
        lsb.gemm_sweep(shapes)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
