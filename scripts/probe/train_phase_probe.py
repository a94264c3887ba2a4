"""Where does a row of the fused training pass spend its time? Builds train_phase_probe.hip and
prints the median per-row phase spans and the per-CU gap between consecutive rows (us)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

here = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(here))
sys.path.insert(0, ROOT)
so = "/tmp/libtphase.so"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                       os.path.join(here, "train_phase_probe.hip"), "-o", so])
lib = ctypes.CDLL(so, mode=ctypes.RTLD_LOCAL)
from skyrl_amd import _ffi, ppo_utils  # noqa: E402
from skyrl_amd.config import AlgorithmConfig  # noqa: E402

dev = torch.device("cuda:0")
mb, R, V = 16, 1024, 151936
x = torch.empty((mb, R, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
dx = torch.empty_like(x)
g = torch.Generator(device=dev).manual_seed(1)
labels = torch.randint(0, V, (mb, R), device=dev, generator=g)
old = torch.randn(mb, R, device=dev, generator=g) - 12
adv = torch.randn(mb, R, device=dev, generator=g)
mask = torch.ones(mb, R, device=dev)
ref = old + 0.01
lp = torch.empty(mb, R, device=dev)
ent = torch.empty(mb, R, device=dev)
loss = torch.empty((), device=dev)
met = torch.empty(8, device=dev)
ws = torch.zeros(_ffi.query("skyrl_policy_train_workspace_bytes", mb, R), dtype=torch.uint8, device=dev)
params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=True)
P = ctypes.c_void_p
fn = lib.skyrl_policy_train_fwd
fn.restype = ctypes.c_int
I64, I32 = ctypes.c_int64, ctypes.c_int32
fn.argtypes = [P, ctypes.c_int, I64, I64, I32, I32, I32, P, I64, I64, ctypes.c_float, P, P, P, P,
               ctypes.POINTER(_ffi.PPOParams), P, P, P, P, P, I64, I64, P, P]
st = P(torch.cuda.current_stream().cuda_stream)


def launch():
    rc = fn(P(x.data_ptr()), 1, x.stride(0), x.stride(1), mb, R, V, P(labels.data_ptr()), labels.stride(0),
            labels.stride(1), 1.0, P(old.data_ptr()), P(adv.data_ptr()), P(mask.data_ptr()), P(ref.data_ptr()),
            ctypes.byref(params), P(loss.data_ptr()), P(met.data_ptr()), P(lp.data_ptr()), P(ent.data_ptr()),
            P(dx.data_ptr()), R * V, V, P(ws.data_ptr()), st)
    assert rc == 0


for _ in range(5):
    launch()
torch.cuda.synchronize()
buf = np.zeros(16384 * 8, dtype=np.uint64)
for rep in range(3):
    launch()
    torch.cuda.synchronize()
    assert lib.probe_read(buf.ctypes.data_as(P), ctypes.c_size_t(buf.nbytes)) == 0
    t = buf.reshape(-1, 8).astype(np.int64)
    span = lambda a, b: np.median((t[:, b] - t[:, a]) / 100.0)  # noqa: E731
    cu = t[:, 7]
    gaps = []
    for c in np.unique(cu):
        rows = t[cu == c]
        rows = rows[np.argsort(rows[:, 0])]
        gaps.extend(((rows[1:, 0] - rows[:-1, 4]) / 100.0).tolist())
    total = (t[:, 4].max() - t[:, 0].min()) / 100.0
    print(f"rep {rep}: launch span {total:.1f} us; per row: sweep1 {span(0, 1):.2f}, barrier1 {span(1, 2):.2f}, "
          f"loss terms+barrier2 {span(2, 3):.2f}, sweep2 {span(3, 4):.2f}, row total {span(0, 4):.2f}; "
          f"gap to the next row on the CU: median {np.median(gaps):.2f} p90 {np.percentile(gaps, 90):.2f}; "
          f"rows per CU {len(t) / len(np.unique(cu)):.1f}")
