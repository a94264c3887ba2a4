"""CPU restatement of the reference's hot-path algorithms (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline; the product path
(skyrl_amd/) never imports it.

Each function restates the algorithm of one reference function (cited file:line under
/root/reference/skyrl-train/skyrl_train/) with torch-CPU or numpy operations in the same
order and dtype as the reference, so results agree to fp32 rounding. Parity of this
module is pinned by tests/test_oracle_golden.py against golden vectors produced by the
real reference (tools/gen_golden.py) and the reference's own known-answer tests.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

# --------------------------------------------------------------------------- utils
def masked_mean(t: torch.Tensor, mask: Optional[torch.Tensor], dim=None) -> torch.Tensor:
    """utils/torch_utils.py:180-184"""
    if mask is None:
        return t.mean(axis=dim)
    return (t * mask).sum(axis=dim) / mask.sum(axis=dim).clamp(min=1.0)


def safe_exp_delta(delta: torch.Tensor, clip: float = 20.0, out_dtype=None) -> torch.Tensor:
    """utils/torch_utils.py:187-192"""
    y = torch.clamp(delta.to(torch.float32), -clip, clip).exp()
    return y.to(out_dtype or delta.dtype)


# --------------------------------------------------------------------------- a6 KL
def approx_kl(lp: torch.Tensor, base: torch.Tensor, mask: Optional[torch.Tensor] = None, kind: str = "k3"):
    """utils/ppo_utils.py:88-124 (no grad)"""
    with torch.no_grad():
        if kind == "k1":
            k = lp - base
        elif kind == "abs":
            k = (lp - base).abs()
        elif kind == "k2":
            k = 0.5 * (lp - base).square()
        elif kind == "k3":
            kl = torch.clamp(base - lp, min=-20, max=20)
            k = torch.clamp(torch.exp(kl) - kl - 1, min=-10, max=10)
        else:
            raise ValueError(kind)
        if mask is not None:
            k = k * mask
    return k


# --------------------------------------------------------------------------- a4 GRPO
def grpo_advantage(rewards: torch.Tensor, mask: torch.Tensor, index: Sequence, eps: float = 1e-6,
                   norm_by_std: bool = True) -> torch.Tensor:
    """utils/ppo_utils.py:1132-1182, restated: per-uid mean / unbiased std of row sums."""
    scores = rewards.sum(dim=-1).clone()
    groups: Dict = {}
    for i, uid in enumerate(index):
        groups.setdefault(uid.item() if hasattr(uid, "item") else uid, []).append(i)
    stats = {}
    for uid, rows in groups.items():
        vals = scores[rows]
        if len(rows) == 1:
            stats[uid] = (torch.tensor(0.0), torch.tensor(1.0))
        else:
            stats[uid] = (vals.mean(), vals.std())
    out = scores.clone()
    for uid, rows in groups.items():
        mu, sd = stats[uid]
        for i in rows:
            out[i] = (scores[i] - mu) / (sd + eps) if norm_by_std else scores[i] - mu
    return out.unsqueeze(-1) * mask


def normalize_advantages(adv: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """utils/ppo_utils.py:127-145 (advantage_batch_normalize, trainer.py:275-276): the mean is
    over EVERY element (unmasked), the squared deviations are masked and divided by the mask
    sum, rstd = clamp(., 1e-8).rsqrt(); the result is not re-masked."""
    num = mask.sum()
    mean = adv.mean()
    ss = ((adv - mean).pow(2) * mask).sum()
    rstd = (ss / num).clamp(min=1e-8).rsqrt()
    return (adv - mean) * rstd


# --------------------------------------------------------------------------- a5 GAE
def masked_whiten(values: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """utils/ppo_utils.py:148-172 (unbiased masked variance)"""
    mean = masked_mean(values, mask)
    centered = values - mean
    var = masked_mean(centered**2, mask)
    msum = mask.sum()
    if msum == 0:
        raise ValueError("At least one element in the mask has to be 1.")
    if msum == 1:
        raise ValueError("The sum of the mask is one, which can cause a division by zero.")
    var = var * (msum / (msum - 1))
    return (values - mean) * torch.rsqrt(var + 1e-8)


def gae(rewards: torch.Tensor, values: torch.Tensor, mask: torch.Tensor, gamma: float, lambd: float):
    """utils/ppo_utils.py:1101-1129: unmasked reverse recursion, then masked whitening."""
    R = rewards.shape[-1]
    last = torch.zeros(rewards.shape[0], dtype=rewards.dtype)
    adv = torch.empty_like(rewards)
    for t in range(R - 1, -1, -1):
        nv = values[:, t + 1] if t < R - 1 else torch.zeros_like(last)
        delta = rewards[:, t] + gamma * nv - values[:, t]
        last = delta + gamma * lambd * last
        adv[:, t] = last
    ret = adv + values
    return masked_whiten(adv, mask), ret


# --------------------------------------------------------------------------- a7 loss
def ppo_policy_loss(lp, old, adv, *, eps_low=0.2, eps_high=0.2, clip_c=3.0, dual_clip=False,
                    reduction="token_mean", mask=None, max_seq_len=None):
    """utils/ppo_utils.py:548-586 + reduce_loss :984-1009. Differentiable in lp."""
    ratio = safe_exp_delta(lp - old, clip=20.0, out_dtype=lp.dtype)
    surr1 = ratio * adv
    surr2 = ratio.clamp(1 - eps_low, 1 + eps_high) * adv
    loss = -torch.min(surr1, surr2)
    clip_ratio = masked_mean((-surr2 > -surr1).float(), mask).mean().detach().item()
    if dual_clip:
        pg3 = -adv * clip_c
        loss = torch.where(adv < 0, torch.min(pg3, loss), loss)
    if reduction == "token_mean":
        out = masked_mean(loss, mask)
    elif reduction == "sequence_mean":
        out = masked_mean(loss, mask, dim=-1).mean()
    elif reduction == "seq_mean_token_sum_norm":
        seq = (loss * mask).sum(-1) / max_seq_len if mask is not None else loss.sum(-1) / max_seq_len
        out = seq.mean()
    else:
        raise ValueError(reduction)
    return out, {"clip_ratio": clip_ratio}


def policy_loss_assembly(lp, old, adv, mask, ref, entropy, *, use_kl_loss=True, kl_type="k3", kl_coef=0.001,
                         use_entropy_loss=False, ent_coef=0.01, **loss_kw):
    """workers/worker.py:801-876: final = pg + kl*coef - H*coef*[use_entropy_loss]."""
    pg, m = ppo_policy_loss(lp, old, adv, mask=mask, **loss_kw)
    with torch.set_grad_enabled(use_entropy_loss and entropy is not None and entropy.requires_grad):
        ent = masked_mean(entropy, mask) if entropy is not None else torch.tensor(0.0)
    ent_term = ent * ent_coef if use_entropy_loss else torch.tensor(0.0)
    if use_kl_loss:
        kl = approx_kl(lp, ref, mask, kl_type)
        kl = masked_mean(kl, mask, dim=-1).mean()
    else:
        kl = torch.tensor(0.0)
    final = pg + kl * kl_coef - ent_term
    return final, {"policy_loss": pg.item(), "policy_kl": kl.item(), "policy_entropy": ent.item(),
                   "clip_ratio": m["clip_ratio"], "final_loss": final.item()}


def critic_loss(values, old_values, returns, mask, value_clip):
    """utils/ppo_utils.py:175-193"""
    if value_clip is not None:
        vclip = old_values + (values - old_values).clamp(-value_clip, value_clip)
        s1 = (vclip - returns) ** 2
        s2 = (values - returns) ** 2
        loss = torch.max(s1, s2)
        clipfrac = masked_mean((s1 > s2).float(), mask).mean().detach().item()
    else:
        clipfrac = None
        loss = (values - returns) ** 2
    return 0.5 * masked_mean(loss, mask, dim=-1).mean(), clipfrac


def reward_kl_penalty(rewards, lp, base, mask, kind, coef):
    """trainer.py:981-1035 -> (rewards, avg_kl, avg_kl_max)"""
    kl = approx_kl(lp, base, mask, kind)
    kl_max = torch.max(kl.abs(), dim=-1)[0]
    kl_mean = masked_mean(kl, mask, dim=-1)
    return rewards - kl * max(0, coef), kl_mean.mean().item(), kl_max.mean().item()


# --------------------------------------------------------------------------- a2/a3 logprob
def logprobs_from_logits(logits: torch.Tensor, labels: torch.Tensor, temperature: float = 1.0):
    """model_wrapper.py:314 (div_ in the logits dtype) + torch_utils.py:158-177 fp32 path
    (the flash CE semantics: fp32 logsumexp of the upcast logits minus the label logit)."""
    x = logits / temperature if temperature != 1.0 else logits
    x = x.to(torch.float32)
    lab = torch.gather(x, -1, labels.unsqueeze(-1)).squeeze(-1)
    return lab - torch.logsumexp(x, dim=-1)


def entropy_from_logits(logits: torch.Tensor, temperature: float = 1.0, in_dtype: bool = False):
    """torch_utils.py:59-111. in_dtype=True restates the reference exactly (math in the
    logits dtype, bf16 for a bf16 model); False computes the same quantity in fp32."""
    x = logits / temperature if temperature != 1.0 else logits
    if not in_dtype:
        x = x.to(torch.float32)
    lp = torch.log_softmax(x, dim=-1)
    return -(lp.exp() * lp).sum(-1)


# --------------------------------------------------------------------------- a9 pack
def pack(prompts: List[List[int]], responses: List[List[int]], rewards: List[List[float]],
         loss_masks: List[List[float]], logprobs: Optional[List[List[float]]], pad_id: int, pad: int = 0):
    """dataset/preprocess.py:28-132 + trainer.pad_batch (trainer.py:872-907), numpy."""
    N = len(prompts)
    P = max(len(p) for p in prompts)
    R = max(len(r) for r in responses)
    S = P + R
    Np = N + pad
    seq = np.full((Np, S), pad_id, dtype=np.int64)
    att = np.zeros((Np, S), dtype=np.int64)
    rm = np.zeros((Np, R), dtype=np.int64)
    rw = np.zeros((Np, R), dtype=np.float32)
    lm = np.zeros((Np, R), dtype=np.float32)
    lp = np.zeros((Np, R), dtype=np.float32) if logprobs else None
    for i in range(Np):
        s = i if i < N else i - N
        p, r = prompts[s], responses[s]
        seq[i, P - len(p):P] = p
        att[i, P - len(p):P] = 1
        seq[i, P:P + len(r)] = r
        att[i, P:P + len(r)] = 1
        rm[i, :len(r)] = 1
        rw[i, :len(rewards[s])] = rewards[s]
        if i < N:
            lm[i, :len(loss_masks[s])] = loss_masks[s]
        if lp is not None:
            lp[i, :len(logprobs[s])] = logprobs[s]
    return seq, att, rm, rw, lm, lp
