"""Phase timeline of the product form of the GRPO-inside-the-loss launch (skyrl_grpo_ppo_loss_fwd
with the pack scores, SKYRL_LOSS_DEFER_FOLD, no advantages output): phase 5 = after the score
barrier, 1 = token pass done, 6 = records stored. Measurement only."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

here = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(here))
sys.path.insert(0, ROOT)
VARIANT = sys.argv[1] if len(sys.argv) > 1 else ""  # "", NOSTATS, NOMATH (timing-only probe builds)
so = f"/tmp/libphase_fused{VARIANT}.so"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC"]
                      + ([f"-DSKYRL_PROBE_{VARIANT}"] if VARIANT else []) +
                      ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "skyrl_amd", "csrc"),
                       os.path.join(here, "phase_probe.hip"), os.path.join(ROOT, "skyrl_amd", "csrc", "grpo.hip"), "-o", so])
lib = ctypes.CDLL(so, mode=ctypes.RTLD_LOCAL)
from skyrl_amd import _ffi, ppo_utils  # noqa: E402
from skyrl_amd.config import AlgorithmConfig  # noqa: E402

dev = torch.device("cuda:0")
N, R = 512, 1024
g = torch.Generator(device=dev).manual_seed(0)
lp = -2 + 0.1 * torch.randn(N, R, device=dev, generator=g)
old = lp + 0.05 * torch.randn(N, R, device=dev, generator=g)
ref = lp + 0.05 * torch.randn(N, R, device=dev, generator=g)
adv = torch.empty(N, R, device=dev)
mask = torch.ones(N, R, device=dev)
rmask = torch.ones(N, R, device=dev, dtype=torch.int64)
rew = torch.zeros(N, R, device=dev)
rew[:, -1] = (torch.rand(N, device=dev, generator=g) < 0.3).float()
params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=False)
loss = torch.empty(1, device=dev)
metrics = torch.empty(8, device=dev)
glp = torch.empty(N, R, device=dev)
rows = mask.sum(-1)
scores = rew.sum(-1)
ws = torch.zeros(_ffi.query("skyrl_ppo_loss_workspace_bytes", N, R), dtype=torch.uint8, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = ctypes.c_void_p
fn = lib.skyrl_grpo_ppo_loss_fwd
fn.restype = ctypes.c_int
I32 = ctypes.c_int32
fn.argtypes = [P, P, P, ctypes.c_int, I32, ctypes.c_float, I32, P, P, P, P, P, P, I32, I32, P, P, P, P, P, P, I32,
               P, P]


def launch():
    rc = fn(P(rew.data_ptr()), P(scores.data_ptr()), None, _ffi.I64, N // 8, 1e-6, 1, P(lp.data_ptr()),
            P(old.data_ptr()), P(mask.data_ptr()), P(ref.data_ptr()), None, P(rows.data_ptr()), N, R,
            ctypes.byref(params), None, P(loss.data_ptr()), P(metrics.data_ptr()), P(glp.data_ptr()), None,
            _ffi.LOSS_DEFER_FOLD, P(ws.data_ptr()), st)
    assert rc == 0


for _ in range(20):
    launch()
torch.cuda.synchronize()
buf = np.zeros(8192 * 8, dtype=np.uint64)
for rep in range(3):
    lib.probe_clear()
    torch.cuda.synchronize()
    for _ in range(1 if rep == 0 else 30):  # rep 0 cold (after a sync), later reps warm (last of 30)
        launch()
    torch.cuda.synchronize()
    assert lib.probe_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) == 0
    t = buf.reshape(-1, 8).astype(np.int64)
    t = t[: int(np.nonzero(t[:, 0])[0].max()) + 1]
    t0 = t[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731  (s_memrealtime: 100 MHz)
    med = lambda k: np.median((t[:, k] - t[:, 0]) / 100)  # noqa: E731
    print(f"{VARIANT or 'default'} rep {rep}: {len(t)} blocks: entries {us(t[:, 0]).min():.2f}..{us(t[:, 0]).max():.2f} us; "
          f"median span to barrier {med(5):.2f}, token pass {med(1):.2f}, records {med(6):.2f}; "
          f"last barrier {us(t[:, 5]).max():.2f}, last token pass {us(t[:, 1]).max():.2f}, "
          f"last records {us(t[:, 6]).max():.2f}", flush=True)
