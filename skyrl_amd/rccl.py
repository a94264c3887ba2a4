"""RCCL communicator through the C ABI (``skyrl_comm_*`` in include/skyrl_hip.h).

The trainer's own exchanges go through torch.distributed (``comm.py``), whose "nccl" backend is
the same RCCL. This binding exercises the C-ABI surface a non-Python host would bind (SURVEY
§8(b): ``skyrl_comm_{init, allreduce, broadcast}``) and gives Python callers collectives that
are independent of a torch process group: one communicator per process and GPU, every call
stream-ordered on the current torch stream, nothing allocated per call.

Reference call sites (skyrl-train/skyrl_train/): all-reduce = metric reduction
(distributed/strategy.py:70-95) and the DP gradient mean (distributed/fsdp_strategy.py:216-226);
reduce-scatter = FSDP2's fp32 gradient reduce-scatter (fsdp_strategy.py:253-271); broadcast =
learner -> rollout weights (weight_sync/broadcast_strategy.py:98-191).
"""

from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.distributed as dist

from . import _ffi

SUM, MAX, MIN, AVG = 0, 1, 2, 3
_OPS = {"sum": SUM, "max": MAX, "min": MIN, "avg": AVG}
_DTYPES = {torch.float32: _ffi.F32, torch.bfloat16: _ffi.BF16, torch.int64: _ffi.I64, torch.int32: _ffi.I32,
           torch.uint8: _ffi.U8}


def _dt(t: torch.Tensor) -> int:
    if t.dtype not in _DTYPES:
        raise TypeError(f"RCCL collectives take {sorted(str(d) for d in _DTYPES)}, got {t.dtype}")
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("RCCL collectives take contiguous device tensors")
    return _DTYPES[t.dtype]


def _op(op) -> int:
    if isinstance(op, str):
        if op not in _OPS:
            raise ValueError(f"op must be one of {sorted(_OPS)}")
        return _OPS[op]
    return int(op)


class RcclComm:
    """One RCCL communicator (nranks, rank) on the current HIP device."""

    def __init__(self, nranks: int, rank: int, unique_id: bytes):
        if len(unique_id) != self.unique_id_bytes():
            raise ValueError(f"unique_id must be {self.unique_id_bytes()} bytes")
        buf = ctypes.create_string_buffer(unique_id, len(unique_id))
        handle = ctypes.c_void_p()
        _ffi.call("skyrl_comm_init", ctypes.cast(buf, ctypes.c_void_p), int(nranks), int(rank), ctypes.byref(handle))
        self._h = handle
        self.nranks, self.rank = int(nranks), int(rank)

    @staticmethod
    def unique_id_bytes() -> int:
        return int(_ffi.query("skyrl_comm_unique_id_bytes"))

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(RcclComm.unique_id_bytes())
        _ffi.call("skyrl_comm_get_unique_id", ctypes.cast(buf, ctypes.c_void_p))
        return buf.raw

    @classmethod
    def from_group(cls, group=None) -> "RcclComm":
        """Rank 0 of a torch process group (any backend) makes the id; the group carries it."""
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(world, rank, obj[0])

    def size(self):
        n, r = ctypes.c_int32(), ctypes.c_int32()
        _ffi.call("skyrl_comm_size", self._h, ctypes.byref(n), ctypes.byref(r))
        return n.value, r.value

    @staticmethod
    def _stream(t: torch.Tensor, stream: Optional[torch.cuda.Stream]):
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        return ctypes.c_void_p(s.cuda_stream)

    def all_reduce(self, t: torch.Tensor, op="sum", out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        out = t if out is None else out
        if out.shape != t.shape or out.dtype != t.dtype:
            raise ValueError("all_reduce: out must match the input")
        _ffi.call("skyrl_comm_allreduce", ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()), t.numel(),
                  _dt(t), _op(op), self._h, self._stream(t, stream))
        return out

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op="sum", stream=None) -> torch.Tensor:
        if inp.numel() != out.numel() * self.nranks or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: input must hold nranks * out.numel() elements of out's dtype")
        _dt(out)
        _ffi.call("skyrl_comm_reduce_scatter", ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                  out.numel(), _dt(inp), _op(op), self._h, self._stream(out, stream))
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None) -> torch.Tensor:
        if out.numel() != inp.numel() * self.nranks or inp.dtype != out.dtype:
            raise ValueError("all_gather: output must hold nranks * input.numel() elements of the input's dtype")
        _dt(out)
        _ffi.call("skyrl_comm_allgather", ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                  inp.numel(), _dt(inp), self._h, self._stream(out, stream))
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        _ffi.call("skyrl_comm_broadcast", ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()), t.numel(),
                  _dt(t), int(root), self._h, self._stream(t, stream))
        return t

    def close(self) -> None:
        """Destroy the communicator (collective: every rank calls it). Not done from __del__: at
        interpreter exit the other ranks may be gone and the destroy would wait for them."""
        if self._h:
            _ffi.call("skyrl_comm_destroy", self._h)
            self._h = ctypes.c_void_p()
