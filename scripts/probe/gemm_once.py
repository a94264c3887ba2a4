"""Launch only the lm_head MFMA GEMM (STORE epilogue) at the decode shape, for PMC passes."""
import sys

import torch

sys.path.insert(0, ".")
from skyrl_amd import _ffi, ops  # noqa: E402

dev = torch.device("cuda")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 512
pipe = int(sys.argv[2]) if len(sys.argv) > 2 else -1
H, V = 1536, 151936
w = (torch.randn(V, H, device=dev) * 0.08).to(torch.bfloat16)
h = torch.randn(M, H, device=dev).to(torch.bfloat16)
z = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
_ffi.set_default_variant(lmhead_pipe=pipe)
for _ in range(20):
    ops.lmhead_gemm(h, w, out=z)
torch.cuda.synchronize()
print("ok")
