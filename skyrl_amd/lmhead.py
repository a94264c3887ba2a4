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

Forward-only calls (the old / ref log-prob passes: no grad needed) take neither: they run
``skyrl_lmhead_logprob_fwd``, our MFMA GEMM with the online softmax in its epilogue (the persistent
tile kernel), so no logits, not even a chunk, leave the registers.
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


def _epilogue_form_ok(h: torch.Tensor, weight: torch.Tensor) -> bool:
    """The GEMM-epilogue kernel's operand rules (skyrl_lmhead_logprob_fwd): bf16, unit K stride,
    K % 64 == 0, 16-B aligned rows."""
    K = h.shape[-1]
    return (h.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and h.dim() == 2 and weight.dim() == 2
            and weight.shape[1] == K and K % 64 == 0 and h.stride(1) == 1 and weight.stride(1) == 1
            and h.stride(0) % 8 == 0 and weight.stride(0) % 8 == 0
            and h.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0)


def lmhead_logprobs_and_entropy(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor,
                                temperature: float = 1.0, compute_entropy: bool = True,
                                chunk: Optional[int] = None):
    """logp, entropy of softmax((hidden @ weight^T) in bf16 / temperature) at ``labels``.

    hidden [..., H] bf16, weight [V, H] bf16 (the HF lm_head.weight layout), labels [...] int.
    Returns f32 tensors shaped like ``labels`` (entropy None when not requested); both are
    differentiable w.r.t. hidden and weight. Without grad (no-grad mode or no operand that needs
    one) and with ``chunk`` unset, the GEMM-epilogue kernel computes them.
    """
    needs_grad = torch.is_grad_enabled() and (hidden.requires_grad or weight.requires_grad)
    if not needs_grad and chunk is None and temperature > 0:
        from . import ops
        H = hidden.shape[-1]
        h = hidden.reshape(-1, H)
        if h.stride(-1) != 1:
            h = h.contiguous()
        if _epilogue_form_ok(h, weight) and h.is_cuda and weight.is_cuda:
            lab, _ = _labels_flat(labels, h.shape[0], h.device)
            lp, ent = ops.lmhead_logprob_fwd(h, weight, lab, temperature=float(temperature),
                                             compute_entropy=bool(compute_entropy))
            shape = labels.shape
            return lp.view(shape), (ent.view(shape) if ent is not None else None)
    return LMHeadLogprob.apply(hidden, weight, labels, float(temperature), bool(compute_entropy), chunk)


# ---------------------------------------------------------------- tensor-parallel vocab shards
def _tp_world(group) -> int:
    import torch.distributed as dist

    if group is None and not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def _shard_states(h, weight, lab, lstride, v_start, temperature, vc) -> torch.Tensor:
    """Per-token softmax state (m, S, W, label logit; 16 B) of this rank's vocab shard: the
    chunk kernel over the shard's columns with v0 = global column and no finalize."""
    T, V = h.shape[0], weight.shape[0]
    dev = h.device
    state = torch.empty(max(16, _ffi.query("skyrl_lmhead_state_bytes", T)), dtype=torch.uint8, device=dev)
    if T > 0:
        zbuf = torch.empty(T * min(vc, V), dtype=torch.bfloat16, device=dev)
        s = _stream(dev)
        for c0 in range(0, V, vc):
            w = min(vc, V - c0)
            z = zbuf[: T * w].view(T, w)
            torch.mm(h, weight[c0:c0 + w].t(), out=z)
            _ffi.call("skyrl_lmhead_chunk_fwd", _ptr(z), w, T, w, v_start + c0, _ptr(lab), lstride, temperature,
                      _ptr(state), int(c0 == 0), 0, None, None, None, s)
    return state


def _gather_states(state: torch.Tensor, T: int, group) -> Tuple[torch.Tensor, int]:
    """All-gather the ranks' per-token softmax states (16 B per token each, rank order): one
    small collective instead of the reference's three all-reduces (max, sum-exp, label logit)."""
    import torch.distributed as dist

    st = state[: T * 16].view(torch.float32).view(T, 4)
    world = _tp_world(group)
    if world == 1:
        return st, 1
    if dist.get_backend(group) == "gloo":  # CPU rehearsal backend: stage through host memory
        bufs = [torch.empty(T, 4, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(bufs, st.cpu(), group=group)
        return torch.cat(bufs, dim=0).to(state.device), world
    bufs = [torch.empty_like(st) for _ in range(world)]
    dist.all_gather(bufs, st.contiguous(), group=group)
    return torch.cat(bufs, dim=0), world


def _merge(states: torch.Tensor, n: int, T: int, compute_entropy: bool, dev):
    logp = torch.empty(T, dtype=torch.float32, device=dev)
    ent = torch.empty(T, dtype=torch.float32, device=dev) if compute_entropy else None
    lse = torch.empty(T, dtype=torch.float32, device=dev)
    _ffi.call("skyrl_lmhead_state_merge", _ptr(states), n, T, _ptr(logp), _ptr(ent), _ptr(lse), _stream(dev))
    return logp, ent, lse


def _shard_bwd(h, weight, lab, lstride, v_start, temperature, vc, lse, ent, glp, gent, need_h, need_w, z_of=None):
    """dh (f32 partial over this shard) and dW_shard; z_of(v0, w) gives precomputed logits
    columns instead of the recompute GEMM (the logits-input variant passes it, weight=None)."""
    T = lse.shape[0]
    V = weight.shape[0] if weight is not None else z_of.V
    dev = lse.device
    H = h.shape[1] if h is not None else 0
    dh = torch.zeros(T, H, dtype=torch.float32, device=dev) if need_h else None
    dw = torch.zeros_like(weight) if need_w else None
    dzs = []
    if T > 0:
        n = T * min(vc, V)
        zbuf = torch.empty(n, dtype=torch.bfloat16, device=dev) if z_of is None else None
        dzbuf = torch.empty(n, dtype=torch.bfloat16, device=dev) if z_of is None else None
        s = _stream(dev)
        for c0 in range(0, V, vc):
            w = min(vc, V - c0)
            if z_of is None:
                z = zbuf[: T * w].view(T, w)
                torch.mm(h, weight[c0:c0 + w].t(), out=z)
                ldz = w
                dz = dzbuf[: T * w].view(T, w)
            else:
                z, ldz = z_of(c0, w)
                dz = z_of.grad[:, c0:c0 + w]
            _ffi.call("skyrl_lmhead_chunk_bwd", _ptr(z), ldz, T, w, v_start + c0, _ptr(lab), lstride, temperature,
                      _ptr(lse), _ptr(ent if gent is not None else None), _ptr(glp), _ptr(gent), _ptr(dz),
                      dz.stride(0), s)
            if need_h:
                _acc_mm(dh, dz, weight[c0:c0 + w])
            if need_w:
                torch.mm(dz.t(), h, out=dw[c0:c0 + w])
    return dh, dw


class VocabParallelLMHeadLogprob(torch.autograd.Function):
    """lm_head-fused logprob + entropy with the vocabulary sharded over a tensor-parallel group.

    Replaces the Megatron path's vocab-parallel lm_head -> logits.div_(T) ->
    from_parallel_logits_to_logprobs / DistributedLogprob (distributed/megatron/model_utils.py:
    64-136, 250-321) + vocab_parallel_entropy (:548-590). Each rank holds rows
    [vocab_start, vocab_start + V_shard) of the lm_head weight; the logits are never
    materialized on any rank. Forward: local chunks (v0 = global column, no finalize), one
    all-gather of the 16-B per-token states, a merge kernel. Backward: the local chunks' dz
    with the merged lse/entropy, dW for the local shard, and dh all-reduced over the group (the
    input-gradient reduction of a vocab-parallel lm_head)."""

    @staticmethod
    def forward(ctx, hidden, weight, labels, temperature, compute_entropy, chunk, vocab_start, group):
        dev = _require_gpu(hidden, weight, labels)
        if hidden.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
            raise TypeError("lm_head fused logprob takes bf16 hidden states and bf16 weight")
        if temperature <= 0:
            raise ValueError("temperature must be > 0")
        H = hidden.shape[-1]
        V = weight.shape[0]
        if weight.dim() != 2 or weight.shape[1] != H or V == 0:
            raise ValueError(f"weight shard must be [V_shard > 0, {H}], got {tuple(weight.shape)}")
        h = hidden.reshape(-1, H)
        if h.stride(-1) != 1:
            h = h.contiguous()
        T = h.shape[0]
        lab, lstride = _labels_flat(labels, T, dev)
        vc = int(chunk) if chunk else default_chunk(T, V)
        state = _shard_states(h, weight, lab, lstride, int(vocab_start), float(temperature), vc)
        states, n = _gather_states(state, T, group)
        logp, ent, lse = _merge(states, n, T, compute_entropy, dev)
        ctx.save_for_backward(h, weight, lab, lse, ent if ent is not None else lse)
        ctx.meta = (hidden.shape, float(temperature), vc, lstride, ent is not None, int(vocab_start), group)
        shape = labels.shape
        return logp.view(shape), (ent.view(shape) if ent is not None else None)

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        import torch.distributed as dist

        h, weight, lab, lse, ent = ctx.saved_tensors
        hshape, temperature, vc, lstride, has_ent, v_start, group = ctx.meta
        T = h.shape[0]
        dev = h.device
        glp = (torch.zeros(T, dtype=torch.float32, device=dev) if g_logp is None
               else g_logp.reshape(T).to(torch.float32).contiguous())
        gent = g_ent.reshape(T).to(torch.float32).contiguous() if (has_ent and g_ent is not None) else None
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dh, dw = _shard_bwd(h, weight, lab, lstride, v_start, temperature, vc, lse, ent, glp, gent, need_h, need_w)
        if need_h and _tp_world(group) > 1:
            if dist.get_backend(group) == "gloo":
                host = dh.cpu()
                dist.all_reduce(host, group=group)
                dh.copy_(host)
            else:
                dist.all_reduce(dh, group=group)
        dhid = dh.to(h.dtype).view(hshape) if need_h else None
        return dhid, dw, None, None, None, None, None, None


def vocab_parallel_lmhead_logprobs_and_entropy(hidden: torch.Tensor, weight_shard: torch.Tensor,
                                               labels: torch.Tensor, vocab_start: int, group=None,
                                               temperature: float = 1.0, compute_entropy: bool = True,
                                               chunk: Optional[int] = None):
    """lmhead_logprobs_and_entropy with lm_head rows [vocab_start, vocab_start + V_shard) on this
    rank of ``group`` (all ranks pass the same hidden and labels; labels are global ids).
    Every rank returns the full-vocabulary logp / entropy."""
    return VocabParallelLMHeadLogprob.apply(hidden, weight_shard, labels, float(temperature), bool(compute_entropy),
                                            chunk, int(vocab_start), group)


class _LogitsShard:
    """z_of(v0, w) over materialized vocab-parallel logits rows (bf16 [T, V_shard])."""

    def __init__(self, logits: torch.Tensor, grad: Optional[torch.Tensor] = None):
        self.logits, self.grad, self.V = logits, grad, logits.shape[1]

    def __call__(self, c0, w):
        return self.logits[:, c0:c0 + w], self.logits.stride(0)


class DistributedLogprob(torch.autograd.Function):
    """The reference's DistributedLogprob (megatron/model_utils.py:64-136) over materialized bf16
    vocab-parallel logits [..., V_shard], on the HIP chunk kernels: the shard is one chunk
    (no GEMM), states all-gathered and merged as above. Backward: dlogits for the local shard
    (1[v = target] - softmax) * grad, bf16 like the logits."""

    @staticmethod
    def forward(ctx, vocab_parallel_logits, target, vocab_start_index, vocab_end_index, group, inference_only):
        dev = _require_gpu(vocab_parallel_logits, target)
        if vocab_parallel_logits.dtype != torch.bfloat16:
            raise TypeError("DistributedLogprob takes bf16 vocab-parallel logits")
        Vs = vocab_parallel_logits.shape[-1]
        if vocab_end_index - vocab_start_index != Vs:
            raise ValueError(f"vocab range [{vocab_start_index}, {vocab_end_index}) does not match the shard width {Vs}")
        z = vocab_parallel_logits.reshape(-1, Vs)
        if z.stride(-1) != 1:
            z = z.contiguous()
        T = z.shape[0]
        lab, lstride = _labels_flat(target, T, dev)
        state = torch.empty(max(16, _ffi.query("skyrl_lmhead_state_bytes", T)), dtype=torch.uint8, device=dev)
        if T > 0:
            _ffi.call("skyrl_lmhead_chunk_fwd", _ptr(z), z.stride(0), T, Vs, int(vocab_start_index), _ptr(lab),
                      lstride, 1.0, _ptr(state), 1, 0, None, None, None, _stream(dev))
        states, n = _gather_states(state, T, group)
        logp, _, lse = _merge(states, n, T, False, dev)
        if not inference_only:
            ctx.save_for_backward(z, lab, lse)
            ctx.meta = (vocab_parallel_logits.shape, lstride, int(vocab_start_index))
        return logp.view(target.shape)

    @staticmethod
    def backward(ctx, g):
        z, lab, lse = ctx.saved_tensors
        shape, lstride, v_start = ctx.meta
        T, Vs = z.shape
        glp = g.reshape(T).to(torch.float32).contiguous()
        grad = torch.empty(T, Vs, dtype=torch.bfloat16, device=z.device)
        _shard_bwd(None, None, lab, lstride, v_start, 1.0, Vs, lse, None, glp, None, False, False,
                   z_of=_LogitsShard(z, grad))
        return grad.view(shape), None, None, None, None, None


def from_parallel_logits_to_logprobs(vocab_parallel_logits: torch.Tensor, target: torch.Tensor,
                                     vocab_start_index: int, vocab_end_index: int, tp_group=None,
                                     inference_only: bool = False) -> torch.Tensor:
    """model_utils.py:250-321 without context parallelism: targets rolled by -1, logprobs of
    [B, S] logits shards, the last position dropped -> [B, S-1]."""
    target = target.roll(shifts=-1, dims=-1)
    lp = DistributedLogprob.apply(vocab_parallel_logits, target, vocab_start_index, vocab_end_index, tp_group,
                                  inference_only)
    return lp[:, :-1]
