"""skyrl_train.utils.torch_utils surface over the HIP logprob/entropy kernels.

logprobs_from_logits / chunked_entropy_from_logits keep the reference names and argument
meaning (utils/torch_utils.py:59-177) but run one fused HIP pass over the vocabulary
(skyrl_amd.ops.LogprobEntropyFunction): fp32 logsumexp + label gather (the flash-attn CE
semantics the reference uses on GPU) and the entropy in fp32 from the same pass.
"""

from __future__ import annotations

from typing import Optional

import torch

from . import ops


def masked_mean(tensor: torch.Tensor, mask: Optional[torch.Tensor], dim=None) -> torch.Tensor:
    """torch_utils.py:180-184"""
    if mask is None:
        return tensor.mean(axis=dim)
    return (tensor * mask).sum(axis=dim) / mask.sum(axis=dim).clamp(min=1.0)


def safe_exp_delta(delta: torch.Tensor, clip: float = 20.0, out_dtype=None) -> torch.Tensor:
    """torch_utils.py:187-192"""
    y = torch.clamp(delta.to(torch.float32), -clip, clip).exp()
    return y.to(out_dtype or delta.dtype)


def logprobs_from_logits(logits: torch.Tensor, labels: torch.Tensor, inplace_backward: bool = True,
                         temperature: float = 1.0) -> torch.Tensor:
    """Per-token log p(label): fp32 output, differentiable w.r.t. logits (HIP fwd/bwd)."""
    lp, _ = ops.logprobs_and_entropy(logits, labels, temperature, compute_entropy=False)
    return lp


def logprobs_and_entropy(logits: torch.Tensor, labels: torch.Tensor, temperature: float = 1.0,
                         entropy_requires_grad: bool = False):
    """One vocabulary pass for both outputs (the fused form HFModelWrapper.forward needs)."""
    return ops.logprobs_and_entropy(logits, labels, temperature, compute_entropy=entropy_requires_grad)


def chunked_entropy_from_logits(logits: torch.Tensor, requires_grad: bool = False,
                                attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """-sum p log p over the vocab per position (fp32), zeroed where attention_mask == 0."""
    if attention_mask is not None and tuple(attention_mask.shape) != tuple(logits.shape[:2]):
        raise ValueError(
            f"attention_mask shape {tuple(attention_mask.shape)} does not match logits shape "
            f"(batch_size={logits.shape[0]}, seqlen={logits.shape[1]})."
        )
    labels = torch.zeros(logits.shape[:-1], dtype=torch.int64, device=logits.device)
    _, ent = ops.logprobs_and_entropy(logits, labels, 1.0, compute_entropy=requires_grad)
    if attention_mask is not None:
        ent = ent * attention_mask
    return ent
