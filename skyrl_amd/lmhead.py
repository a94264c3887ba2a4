"""lm_head-fused logprob + entropy: the [T,V] logits are never materialized.

Reference: HFModelWrapper.forward (skyrl_train/model_wrapper.py:308-363). The model's lm_head
writes bf16 logits [n,S,V]. ``logits.div_(temperature)`` runs in bf16. Then
``logprobs_from_logits`` (utils/torch_utils.py:115-177) and ``chunked_entropy_from_logits``
(:59-111) read the logits. Their backward writes bf16 dlogits, which the lm_head backward GEMMs
read.

Here V is cut into chunks of ``chunk`` columns (one reused bf16 [T, chunk] buffer, about the
size of the 256 MiB Infinity Cache):

  forward   per chunk: z = h @ W_c^T (hipBLASLt, into the reused buffer), then
            skyrl_lmhead_chunk_fwd merges z into the per-token softmax state; the last chunk's
            launch writes logp / entropy / lse.
  backward  per chunk: recompute z, skyrl_lmhead_chunk_bwd writes dz (bf16, reused buffer), then
            dh += dz @ W_c (fp32 accumulation in the GEMM) and dW_c = dz^T @ h.

The GEMMs are plain library GEMMs. The softmax statistics, the label gather, the temperature
division and the dlogits are the HIP kernels, so the per-element numerics equal the unfused
``ops.logprobs_and_entropy`` on the same bf16 logits. The trade is one extra GEMM in the
backward (the recompute) against the bf16 logits and dlogits round trips through HBM, and
O(T*chunk) instead of O(T*V) activation memory.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _ffi
from .ops import _ptr, _require_gpu, _stream

# Chunk buffer budget. Measured at T=8192, H=1536, V=151936 (docs: DESIGN.md §9): 16384-column
# chunks (256 MiB) beat 4096/8192 (fewer, larger GEMMs). A two-stream pipeline that overlaps the
# chunk kernels with the next GEMM measured 18-30 % SLOWER (the memory-bound kernel steals CU slots
# from a GEMM that already saturates the chip), so the chunks run back to back on one stream.
MALL_BUDGET_BYTES = 256 << 20


def default_chunk(T: int, V: int) -> int:
    """Largest multiple of 256 columns whose bf16 [T, chunk] buffer fits the budget."""
    c = MALL_BUDGET_BYTES // max(1, 2 * T)
    c = max(2048, min(65536, c // 256 * 256))
    return min(c, V)


def _labels_flat(labels: torch.Tensor, T: int, dev) -> Tuple[torch.Tensor, int]:
    lab = labels.to(device=dev, dtype=torch.int64)
    if lab.dim() == 1 and lab.numel() == T:
        return lab, lab.stride(0)
    lab = lab.reshape(T)
    return lab, lab.stride(0)


class LMHeadLogprob(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, weight, labels, temperature, compute_entropy, chunk):
        dev = _require_gpu(hidden, weight, labels)
        if hidden.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
            raise TypeError("lm_head fused logprob takes bf16 hidden states and bf16 weight")
        if temperature <= 0:
            raise ValueError("temperature must be > 0")
        H = hidden.shape[-1]
        V = weight.shape[0]
        if weight.dim() != 2 or weight.shape[1] != H:
            raise ValueError(f"weight must be [V, {H}], got {tuple(weight.shape)}")
        h = hidden.reshape(-1, H)
        if h.stride(-1) != 1:
            h = h.contiguous()
        T = h.shape[0]
        lab, lstride = _labels_flat(labels, T, dev)
        vc = int(chunk) if chunk else default_chunk(T, V)
        logp = torch.empty(T, dtype=torch.float32, device=dev)
        ent = torch.empty(T, dtype=torch.float32, device=dev) if compute_entropy else None
        lse = torch.empty(T, dtype=torch.float32, device=dev)
        if T > 0:
            zbuf = torch.empty(T * min(vc, V), dtype=torch.bfloat16, device=dev)
            state = torch.empty(_ffi.query("skyrl_lmhead_state_bytes", T), dtype=torch.uint8, device=dev)
            s = _stream(dev)
            for v0 in range(0, V, vc):
                w = min(vc, V - v0)
                z = zbuf[: T * w].view(T, w)
                torch.mm(h, weight[v0:v0 + w].t(), out=z)
                _ffi.call("skyrl_lmhead_chunk_fwd", _ptr(z), w, T, w, v0, _ptr(lab), lstride, float(temperature),
                          _ptr(state), int(v0 == 0), int(v0 + w >= V), _ptr(logp), _ptr(ent), _ptr(lse), s)
        ctx.save_for_backward(h, weight, lab, lse, ent if ent is not None else lse)
        ctx.meta = (hidden.shape, float(temperature), vc, lstride, ent is not None)
        shape = labels.shape
        return logp.view(shape), (ent.view(shape) if ent is not None else None)

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        h, weight, lab, lse, ent = ctx.saved_tensors
        hshape, temperature, vc, lstride, has_ent = ctx.meta
        T, H = h.shape
        V = weight.shape[0]
        dev = h.device
        glp = (torch.zeros(T, dtype=torch.float32, device=dev) if g_logp is None
               else g_logp.reshape(T).to(torch.float32).contiguous())
        gent = None
        if has_ent and g_ent is not None:
            gent = g_ent.reshape(T).to(torch.float32).contiguous()
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dh = torch.zeros(T, H, dtype=torch.float32, device=dev) if need_h else None
        dw = torch.empty_like(weight) if need_w else None
        if T > 0 and (need_h or need_w):
            n = T * min(vc, V)
            zbuf = torch.empty(n, dtype=torch.bfloat16, device=dev)
            dzbuf = torch.empty(n, dtype=torch.bfloat16, device=dev)
            s = _stream(dev)
            for v0 in range(0, V, vc):
                w = min(vc, V - v0)
                wc = weight[v0:v0 + w]
                z = zbuf[: T * w].view(T, w)
                dz = dzbuf[: T * w].view(T, w)
                torch.mm(h, wc.t(), out=z)
                _ffi.call("skyrl_lmhead_chunk_bwd", _ptr(z), w, T, w, v0, _ptr(lab), lstride, temperature,
                          _ptr(lse), _ptr(ent if gent is not None else None), _ptr(glp), _ptr(gent), _ptr(dz), w, s)
                if need_h:
                    _acc_mm(dh, dz, wc)
                if need_w:
                    torch.mm(dz.t(), h, out=dw[v0:v0 + w])
        elif need_w:
            dw.zero_()
        dhid = dh.to(h.dtype).view(hshape) if need_h else None
        return dhid, dw, None, None, None, None


_ADDMM_F32 = [None]  # whether aten::addmm.dtype_out (bf16 x bf16 + f32 -> f32) runs on this build


def _acc_mm(acc: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """acc (f32) += a @ b (bf16), accumulated in fp32 inside the GEMM where the build allows."""
    if _ADDMM_F32[0] is not False:
        try:
            torch.ops.aten.addmm.dtype_out(acc, a, b, torch.float32, out=acc)
            _ADDMM_F32[0] = True
            return
        except (RuntimeError, NotImplementedError):
            _ADDMM_F32[0] = False
    acc.add_(torch.mm(a, b, out_dtype=torch.float32))


def lmhead_logprobs_and_entropy(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor,
                                temperature: float = 1.0, compute_entropy: bool = True,
                                chunk: Optional[int] = None):
    """logp, entropy of softmax((hidden @ weight^T) in bf16 / temperature) at ``labels``.

    hidden [..., H] bf16, weight [V, H] bf16 (the HF lm_head.weight layout), labels [...] int.
    Returns f32 tensors shaped like ``labels`` (entropy None when not requested); both are
    differentiable w.r.t. hidden and weight.
    """
    return LMHeadLogprob.apply(hidden, weight, labels, float(temperature), bool(compute_entropy), chunk)
