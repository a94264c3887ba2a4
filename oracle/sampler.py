"""ctypes binding of oracle/_build/libsampler_ref.so (TEST INFRASTRUCTURE ONLY: the checker
for skyrl_sample; imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline)."""

import ctypes
import os

import torch

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libsampler_ref.so")
_fn = None
_support = None


def load():
    global _fn
    if _fn is None:
        f = ctypes.CDLL(_LIB).sampler_ref
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _fn = f
    return _fn


def sample(logits_cpu: torch.Tensor, temperature=1.0, top_k=-1, top_p=1.0, min_p=0.0, seed=0, seq_ids=None, step=0):
    """[nseq, V] bf16/f32 CPU logits -> (tokens int32, logprobs f32), one thread, index order."""
    f = load()
    n, V = logits_cpu.shape
    bf = logits_cpu.dtype == torch.bfloat16
    raw = logits_cpu.contiguous().view(torch.int16) if bf else logits_cpu.contiguous().float()
    tok = torch.empty(n, dtype=torch.int32)
    lp = torch.empty(n, dtype=torch.float32)
    keys = torch.empty(V, dtype=torch.int32)
    ids = torch.arange(n, dtype=torch.int64) if seq_ids is None else seq_ids.to(torch.int64).contiguous()
    f(raw.data_ptr(), int(bf), V, n, V, float(temperature), int(top_k), float(top_p), float(min_p),
      ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), ids.data_ptr(), int(step), tok.data_ptr(), lp.data_ptr(),
      keys.data_ptr())
    return tok, lp


def support(logits_cpu: torch.Tensor, temperature=1.0, top_k=-1, top_p=1.0, min_p=0.0) -> torch.Tensor:
    """[nseq, V] bf16/f32 CPU logits -> bool [nseq, V]: the filtered support (the finite
    entries of tx's apply_top_k_batch / apply_top_p_batch output)."""
    global _support
    if _support is None:
        f = ctypes.CDLL(_LIB).sampler_ref_support
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        _support = f
    n, V = logits_cpu.shape
    bf = logits_cpu.dtype == torch.bfloat16
    raw = logits_cpu.contiguous().view(torch.int16) if bf else logits_cpu.contiguous().float()
    keep = torch.empty(n, V, dtype=torch.uint8)
    _support(raw.data_ptr(), int(bf), V, n, V, float(temperature), int(top_k), float(top_p), float(min_p),
             keep.data_ptr())
    return keep.bool()
