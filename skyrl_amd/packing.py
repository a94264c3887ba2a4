"""Sample packing for the learner forward (reference: HFModelWrapper.forward with
use_sample_packing, model_wrapper.py:272-330; on by default, `config.py:457`).

The reference removes the padding with flash-attn's `unpad_input`. It runs the HF model on one
[1, nnz] row with per-sequence position ids and no attention mask, and flash_attention_2's
varlen kernel keeps the sequences apart. flash-attn is not part of this image. Here the same
packed row runs through PyTorch's varlen flash attention (`torch.nn.attention.varlen`, the
ROCm flash kernels). It is registered with HF as the attention implementation "skyrl_varlen":

  * packed calls (cu_seq_lens_q in the layer kwargs) go to varlen_attn, causal, one segment
    per sequence;
  * calls without them (padded batches, generation) fall through to HF's SDPA attention and
    SDPA mask, so a model switched to "skyrl_varlen" still runs unpacked batches unchanged.

The cu_seq_lens / max_length kwargs are passed into the model call. HF forwards them to every
attention layer, including the recompute under gradient checkpointing.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

IMPL = "skyrl_varlen"
_REGISTERED = [False]


def _varlen_attention(module, query, key, value, attention_mask, dropout=0.0, scaling=None, **kwargs):
    from transformers.integrations.sdpa_attention import sdpa_attention_forward

    cu = kwargs.get("cu_seq_lens_q")
    if cu is None:
        return sdpa_attention_forward(module, query, key, value, attention_mask, dropout=dropout, scaling=scaling,
                                      **kwargs)
    from torch.nn.attention.varlen import varlen_attn

    if query.shape[0] != 1:
        raise ValueError("packed attention expects one packed row")
    D = query.shape[-1]
    if scaling is not None and abs(scaling - D ** -0.5) > 1e-6 * D ** -0.5:
        raise ValueError("varlen attention uses the 1/sqrt(head_dim) scale")
    q = query[0].transpose(0, 1)  # [T, Hq, D]
    k = key[0].transpose(0, 1)
    v = value[0].transpose(0, 1)
    if q.dtype not in (torch.bfloat16, torch.float16):  # fp32 rope output under autocast: SDPA would cast too
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.bfloat16
        q, k, v = q.to(dt), k.to(dt), v.to(dt)
    mx = int(kwargs["max_length_q"])
    out = varlen_attn(q.contiguous(), k.contiguous(), v.contiguous(), cu, cu, mx, mx, is_causal=True)
    return out.unsqueeze(0), None  # [1, T, Hq, D]


def _varlen_mask(*args, **kwargs):
    """No mask for packed calls (attention_mask None); HF's SDPA mask otherwise."""
    from transformers.masking_utils import sdpa_mask

    if kwargs.get("attention_mask") is None:
        return None
    return sdpa_mask(*args, **kwargs)


def enable_sample_packing(model) -> None:
    """Switch an HF model to the "skyrl_varlen" attention (idempotent)."""
    if not _REGISTERED[0]:
        from transformers import AttentionInterface
        from transformers.masking_utils import AttentionMaskInterface

        AttentionInterface.register(IMPL, _varlen_attention)
        AttentionMaskInterface.register(IMPL, _varlen_mask)
        _REGISTERED[0] = True
    cfg = model.config
    cfg._attn_implementation = IMPL


@dataclass
class Packed:
    input_ids: torch.Tensor  # [1, nnz]
    position_ids: torch.Tensor  # [1, nnz]
    cu_seqlens: torch.Tensor  # int32 [n+1]
    max_len: int
    packed_of: torch.Tensor  # int64 [n*S]: packed index of each padded position (valid where att == 1)


def pack(seq: torch.Tensor, att: torch.Tensor) -> Packed:
    """unpad_input of the reference: the attention_mask == 1 tokens in row-major order, with
    position ids counting from 0 within each sequence (model_wrapper.py:272-289)."""
    flat = att.reshape(-1).bool()
    idx = flat.nonzero().squeeze(1)
    lens = att.sum(1, dtype=torch.int32)
    cu = torch.zeros(len(lens) + 1, dtype=torch.int32, device=seq.device)
    torch.cumsum(lens, 0, out=cu[1:])
    pos = att.long().cumsum(-1) - 1
    packed_of = flat.long().cumsum(0) - 1
    return Packed(seq.reshape(-1)[idx][None], pos.reshape(-1)[idx][None], cu, int(lens.max().item()), packed_of)


def packed_hidden_states(base_model, seq: torch.Tensor, att: torch.Tensor, R: int) -> torch.Tensor:
    """Hidden states of the positions whose logits predict the last R tokens ([n, R, H]: padded
    positions [-R-1:-1]), computed on the packed row. Positions that are padding come back as
    the hidden state of packed token 0 (their logprobs are masked downstream, as the
    reference's pad_input zeros)."""
    p = pack(seq, att)
    out = base_model(input_ids=p.input_ids, position_ids=p.position_ids, attention_mask=None,
                     cu_seq_lens_q=p.cu_seqlens, cu_seq_lens_k=p.cu_seqlens, max_length_q=p.max_len,
                     max_length_k=p.max_len).last_hidden_state[0]
    n, S = seq.shape
    cols = torch.arange(S - R - 1, S - 1, device=seq.device)
    flat_pos = (torch.arange(n, device=seq.device)[:, None] * S + cols[None]).reshape(-1)
    valid = att.reshape(-1)[flat_pos].bool()
    gidx = torch.where(valid, p.packed_of[flat_pos], torch.zeros_like(flat_pos))
    return out.index_select(0, gidx).view(n, R, -1)
