"""Host launchers of the decode-loop kernels (csrc/attention.hip) through the C ABI.

The rollout engine calls these once per layer per step; they check shapes on the host
before any launch (a wrong stride would otherwise read out of bounds on the device) and
raise if the HIP library is missing — there is no CPU fallback on the product path.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

from .. import _ffi
from ..ops import _ptr, _require_gpu, _stream

BLOCK_SIZE = 16  # tokens per KV-cache block (the kernels' fixed tile)


def rope_kv_write(qkv: torch.Tensor, positions: torch.Tensor, slot_mapping: torch.Tensor, cos_sin: torch.Tensor,
                  nh: int, nkv: int, head_dim: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
                  q_out: Optional[torch.Tensor] = None, k_out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rotate q/k of the fused projection ``qkv`` [T, (nh+2nkv)*D] (bf16, unit last stride),
    write k/v into one layer's paged cache at ``slot_mapping`` and return rotated q [T, nh, D]."""
    dev = _require_gpu(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache)
    T = qkv.shape[0]
    width = (nh + 2 * nkv) * head_dim
    if qkv.dtype != torch.bfloat16 or qkv.dim() != 2 or qkv.shape[1] != width or qkv.stride(1) != 1:
        raise ValueError(f"qkv must be bf16 [T, {width}] with unit column stride, got {tuple(qkv.shape)}")
    if positions.dtype != torch.int64 or slot_mapping.dtype != torch.int64 or positions.numel() != T \
            or slot_mapping.numel() != T:
        raise ValueError("positions and slot_mapping must be int64 [T]")
    if cos_sin.dtype != torch.float32 or cos_sin.dim() != 2 or cos_sin.shape[1] != head_dim:
        raise ValueError(f"cos_sin must be f32 [max_pos, {head_dim}]")
    nb = k_cache.shape[0]
    if k_cache.shape != (nb, nkv, BLOCK_SIZE, head_dim) or v_cache.shape != (nb, nkv, head_dim, BLOCK_SIZE) \
            or not (k_cache.is_contiguous() and v_cache.is_contiguous()):
        raise ValueError("k_cache must be [blocks, nkv, 16, D] and v_cache [blocks, nkv, D, 16], contiguous")
    if q_out is None:
        q_out = torch.empty((T, nh, head_dim), dtype=torch.bfloat16, device=dev)
    if k_out is not None and (k_out.shape != (T, nkv, head_dim) or not k_out.is_contiguous()):
        raise ValueError("k_out must be contiguous [T, nkv, D]")
    _ffi.call("skyrl_rope_kv_write", _ptr(qkv), qkv.stride(0), T, nh, nkv, head_dim, _ptr(positions),
              _ptr(slot_mapping), _ptr(cos_sin), _ptr(q_out), _ptr(k_out), _ptr(k_cache), _ptr(v_cache), _stream(dev))
    return q_out


def add_rmsnorm(delta: Optional[torch.Tensor], hidden: torch.Tensor, weight: torch.Tensor, eps: float,
                out: torch.Tensor) -> torch.Tensor:
    """hidden += delta (bf16, in place; delta may be None), out = RMSNorm(hidden) * weight."""
    dev = _require_gpu(hidden, weight, out, delta)
    n, H = hidden.shape
    for t in (hidden, out) + ((delta,) if delta is not None else ()):
        if t.dtype != torch.bfloat16 or t.shape != (n, H) or not t.is_contiguous():
            raise ValueError(f"add_rmsnorm: expected contiguous bf16 [{n}, {H}]")
    if weight.dtype != torch.bfloat16 or weight.shape != (H,):
        raise ValueError("add_rmsnorm: weight must be bf16 [H]")
    _ffi.call("skyrl_add_rmsnorm", _ptr(delta), _ptr(hidden), _ptr(weight), n, H, float(eps), _ptr(out), _stream(dev))
    return out


def silu_mul(gate_up: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up of the fused [n, 2I] gate|up projection -> bf16 [n, I]."""
    dev = _require_gpu(gate_up)
    n, I2 = gate_up.shape
    if gate_up.dtype != torch.bfloat16 or not gate_up.is_contiguous() or I2 % 8:
        raise ValueError("silu_mul: gate_up must be contiguous bf16 [n, 2I] with I % 4 == 0")
    if out is None:
        out = torch.empty((n, I2 // 2), dtype=torch.bfloat16, device=dev)
    _ffi.call("skyrl_silu_mul", _ptr(gate_up), n, I2 // 2, _ptr(out), _stream(dev))
    return out


MIN_PARTITION = 64  # context tokens: below this a wave's fixed cost outweighs its KV stream


def choose_nparts(nseq: int, nkv: int, max_ctx: int, target_waves: int = 1024, min_split: int = 1) -> int:
    """Waves per (sequence, kv head) for about ``target_waves`` waves in flight (256 CUs x 4;
    measured: fewer, longer waves beat finer splits down to that count), never more than
    max_ctx / MIN_PARTITION. ``min_split`` > 1 forces a split even when the batch alone fills
    the chip: at 512 ragged rollout contexts U[17,1536] 2-4 splits measured 4.0-4.3 TB/s vs
    3.8 unsplit, but at 512 uniform contexts of 1280 2 splits lose 10% (5.05 vs 5.65 TB/s),
    so the default stays 1 (scripts/probe/attn_ragged_sweep.py). The kernel splits each
    sequence's own context over that many waves (at least MIN_PARTITION tokens each), so the
    choice only sizes the grid: two calls whose nparts differ only by this cap compute
    identical splits."""
    want = max(min_split, math.ceil(target_waves / max(1, nseq * nkv)))
    return max(1, min(want, math.ceil(max(max_ctx, 1) / MIN_PARTITION)))


def balanced_waves(nkv: int, total_blocks_hint: Optional[int] = None, target_waves: int = 1024) -> int:
    """Waves per kv head for paged_decode_balanced: about ``target_waves`` in flight (one per SIMD)."""
    w = max(1, target_waves // max(1, nkv))
    return w if total_blocks_hint is None else max(1, min(w, total_blocks_hint))


class DecodeWorkspace:
    """Grows-only fp32 scratch for the partition merge (reused every layer and step)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = torch.empty(0, dtype=torch.uint8, device=self.device)

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 2 * self.buf.numel()), dtype=torch.uint8, device=self.device)
        return self.buf


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                 context_lens: torch.Tensor, max_ctx: int, scale: float, out: Optional[torch.Tensor] = None,
                 workspace: Optional[DecodeWorkspace] = None, nparts: Optional[int] = None,
                 part_min: int = MIN_PARTITION) -> torch.Tensor:
    """softmax(scale * q K^T) V for one query token per sequence over its paged context.

    q: bf16 [n, nh, D]; block_tables: int32 [n, max_blocks]; context_lens: int32 [n] (>= 1,
    <= max_ctx, and max_blocks * 16 >= max_ctx). Each context is split on device over at most
    ``nparts`` waves per kv head of at least ``part_min`` tokens. Returns bf16 [n, nh, D]."""
    dev = _require_gpu(q, k_cache, v_cache, block_tables, context_lens)
    n, nh, D = q.shape
    nb, nkv = k_cache.shape[0], k_cache.shape[1]
    if q.dtype != torch.bfloat16 or q.stride(2) != 1 or q.stride(1) != D:
        raise ValueError("q must be bf16 [n, nh, D] with contiguous heads")
    if k_cache.shape != (nb, nkv, BLOCK_SIZE, D) or v_cache.shape != (nb, nkv, D, BLOCK_SIZE):
        raise ValueError("cache shapes do not match q")
    if block_tables.dtype != torch.int32 or block_tables.dim() != 2 or block_tables.shape[0] != n \
            or block_tables.stride(1) != 1:
        raise ValueError("block_tables must be int32 [n, max_blocks] with unit column stride")
    if context_lens.dtype != torch.int32 or context_lens.numel() != n or not context_lens.is_contiguous():
        raise ValueError("context_lens must be contiguous int32 [n]")
    if block_tables.shape[1] * BLOCK_SIZE < max_ctx:
        raise ValueError("block_tables too narrow for max_ctx")
    if out is None:
        out = torch.empty((n, nh, D), dtype=torch.bfloat16, device=dev)
    if n == 0:
        return out
    nparts = nparts or choose_nparts(n, nkv, max_ctx)
    ws = None
    if nparts > 1:
        nbytes = _ffi.query("skyrl_paged_decode_workspace_bytes", n, nh, D, nparts)
        ws = (workspace or DecodeWorkspace(dev)).get(nbytes)
    _ffi.call("skyrl_paged_decode", _ptr(q), q.stride(0), _ptr(k_cache), _ptr(v_cache), _ptr(block_tables),
              block_tables.stride(0), _ptr(context_lens), n, nh, nkv, D, float(scale), part_min, nparts, _ptr(out),
              out.stride(0), _ptr(ws), _stream(dev))
    return out


def paged_decode_balanced(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                          block_tables: torch.Tensor, context_lens: torch.Tensor, scale: float,
                          out: Optional[torch.Tensor] = None, workspace: Optional[DecodeWorkspace] = None,
                          waves: Optional[int] = None) -> torch.Tensor:
    """paged_decode with the work split by cache blocks: every wave streams the same number of
    blocks across sequence boundaries (plan + attention + merge on the device), so a ragged
    batch streams at the uniform batch's rate. Same arguments and result as paged_decode
    (no max_ctx / split arguments: the plan reads context_lens on the device)."""
    dev = _require_gpu(q, k_cache, v_cache, block_tables, context_lens)
    n, nh, D = q.shape
    nb, nkv = k_cache.shape[0], k_cache.shape[1]
    if q.dtype != torch.bfloat16 or q.stride(2) != 1 or q.stride(1) != D:
        raise ValueError("q must be bf16 [n, nh, D] with contiguous heads")
    if k_cache.shape != (nb, nkv, BLOCK_SIZE, D) or v_cache.shape != (nb, nkv, D, BLOCK_SIZE):
        raise ValueError("cache shapes do not match q")
    if block_tables.dtype != torch.int32 or block_tables.dim() != 2 or block_tables.shape[0] != n \
            or block_tables.stride(1) != 1:
        raise ValueError("block_tables must be int32 [n, max_blocks] with unit column stride")
    if context_lens.dtype != torch.int32 or context_lens.numel() != n or not context_lens.is_contiguous():
        raise ValueError("context_lens must be contiguous int32 [n]")
    if out is None:
        out = torch.empty((n, nh, D), dtype=torch.bfloat16, device=dev)
    if n == 0:
        return out
    waves = waves or balanced_waves(nkv)
    nbytes = _ffi.query("skyrl_paged_decode_balanced_workspace_bytes", n, nh, D, waves)
    ws = (workspace or DecodeWorkspace(dev)).get(nbytes)
    _ffi.call("skyrl_paged_decode_balanced", _ptr(q), q.stride(0), _ptr(k_cache), _ptr(v_cache), _ptr(block_tables),
              block_tables.stride(0), _ptr(context_lens), n, nh, nkv, D, float(scale), waves, _ptr(out),
              out.stride(0), _ptr(ws), _stream(dev))
    return out
