"""Secondary registry entries (not on the accelerated path): torch restatements.

The reference registers these under the same names (skyrl_train/utils/ppo_utils.py:
589-981 losses, :1013-1098 estimators, off_policy_correction_utils.py:7-296). They are
reached only through the registry when a config selects them; SURVEY.md §8(a) keeps them
out of this tier's HIP scope, so they run as plain torch ops on whatever device their
inputs live on. The hot-path names (grpo, gae, regular, dual_clip) never route here.
"""

from __future__ import annotations

from collections import defaultdict
from typing import Dict, Optional, Tuple

import torch

from .torch_utils import masked_mean, safe_exp_delta


def _reduce(loss, mask, reduction, max_seq_len):
    from .ppo_utils import reduce_loss

    return reduce_loss(loss, mask, reduction, max_seq_len)


# ----------------------------------------------------------------------------- off-policy correction
def _is_ratio(old, rollout):
    return safe_exp_delta(old - rollout, clip=20.0, out_dtype=old.dtype)


def off_policy_terms(old, rollout, mask, opc) -> Tuple[Optional[torch.Tensor], Dict[str, float], torch.Tensor]:
    """(tis multiplier or None, metrics, corrected loss mask): off_policy_correction_utils.py:200-258."""
    if opc.tis_ratio_type is None and opc.sequence_mask_metric is None:
        return None, {}, mask
    r = _is_ratio(old, rollout)
    metrics = {
        "is_ratio_mean": masked_mean(r, mask).mean().item(),
        "is_ratio_std": (r * mask).std().item(),
        "is_ratio_max": (r * mask).max().item(),
        "is_ratio_min": (r * mask).min().item(),
    }
    valid = mask > 0
    hi = (r > opc.outlier_token_is_threshold_high) & valid if opc.outlier_token_is_threshold_high is not None \
        else torch.zeros_like(valid)
    lo = (r < opc.outlier_token_is_threshold_low) & valid if opc.outlier_token_is_threshold_low is not None \
        else torch.zeros_like(valid)
    ok = ((~hi & ~lo) | (mask == 0)).all(dim=-1, keepdim=True)
    n = float(ok.shape[0])
    metrics["outlier_seq_masked_ratio"] = ((~ok.squeeze(-1)).sum() / n).item()
    metrics["outlier_seq_over_high_ratio"] = (hi.any(-1).sum() / n).item()
    metrics["outlier_seq_under_low_ratio"] = (lo.any(-1).sum() / n).item()
    mask = mask * ok.float()
    tis = None
    logr = old - rollout
    if opc.tis_ratio_type == "token":
        cap = opc.token_tis_ratio_clip_high
        capped = (r > cap) & (mask > 0)
        metrics["tis_token_clip_high_ratio"] = (capped.sum() / (mask > 0).sum().clamp(min=1)).item()
        tis = torch.clamp(r, max=cap).detach()
    elif opc.tis_ratio_type == "sequence":
        sr = safe_exp_delta((logr * mask).sum(-1, keepdim=True), clip=20.0, out_dtype=old.dtype)
        cap = opc.sequence_tis_ratio_clip_high
        metrics["tis_seq_clip_high_ratio"] = ((sr > cap).sum() / sr.shape[0]).item()
        tis = torch.clamp(sr, max=cap).detach()
    elif opc.tis_ratio_type is not None:
        raise ValueError(f"Unknown tis_ratio_type: {opc.tis_ratio_type}")
    metric = opc.sequence_mask_metric
    if metric is not None:
        s = (logr * mask).sum(-1, keepdim=True)
        if metric == "geometric":
            q = safe_exp_delta(s / mask.sum(-1, keepdim=True).clamp(min=1.0), clip=20.0, out_dtype=old.dtype)
            hi_c, lo_c, tag = opc.geo_mask_high, opc.geo_mask_low, "geo_sequence_mask"
        elif metric == "product":
            q = safe_exp_delta(s, clip=20.0, out_dtype=old.dtype)
            hi_c, lo_c, tag = opc.product_mask_high, opc.product_mask_low, "product_sequence_mask"
        else:
            raise ValueError(f"Unknown sequence_mask_metric: {metric}")
        over, under = q > hi_c, q < lo_c
        keep = ~over & ~under
        n = float(q.shape[0])
        metrics[f"{tag}_masked_ratio"] = ((~keep).sum() / n).item()
        metrics[f"{tag}_over_high_ratio"] = (over.sum() / n).item()
        metrics[f"{tag}_under_low_ratio"] = (under.sum() / n).item()
        mask = mask * keep.float()
    return tis, metrics, mask


def apply_off_policy_correction(loss, old, rollout, mask, opc):
    if rollout is None:
        return loss, mask, {}
    tis, metrics, mask = off_policy_terms(old, rollout, mask, opc)
    if tis is not None:
        loss = loss * tis
    return loss, mask, metrics


# ----------------------------------------------------------------------------- losses
def gspo_policy_loss(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    seq_lr = masked_mean(log_probs - old_log_probs, loss_mask, dim=-1).unsqueeze(-1)
    tok = torch.clamp(log_probs - log_probs.detach() + seq_lr.detach(), max=10)
    ratio = torch.exp(tok)
    s1 = ratio * advantages
    s2 = ratio.clamp(1 - config.eps_clip_low, 1 + config.eps_clip_high) * advantages
    loss = -torch.min(s1, s2)
    m = {"clip_ratio": masked_mean((-s2 > -s1).float(), loss_mask).mean().item()}
    loss, loss_mask, extra = apply_off_policy_correction(loss, old_log_probs, rollout_logprobs, loss_mask,
                                                         config.off_policy_correction)
    m.update(extra)
    return _reduce(loss, loss_mask, config.loss_reduction, config.max_seq_len), m


def sapo_policy_loss(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    tp = torch.as_tensor(config.sapo.tau_pos, dtype=advantages.dtype, device=advantages.device)
    tn = torch.as_tensor(config.sapo.tau_neg, dtype=advantages.dtype, device=advantages.device)
    ratio = torch.exp(torch.clamp(log_probs - old_log_probs, min=-20.0, max=20.0))
    tau = torch.where(advantages > 0, tp, tn)
    gate = torch.sigmoid(tau * (ratio - 1.0)) * (4.0 / tau)
    loss = -gate * advantages
    m = {"clip_ratio": 0.0}
    loss, loss_mask, extra = apply_off_policy_correction(loss, old_log_probs, rollout_logprobs, loss_mask,
                                                         config.off_policy_correction)
    m.update(extra)
    return _reduce(loss, loss_mask, config.loss_reduction, config.max_seq_len), m


def compute_policy_loss_cispo(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    ratio = safe_exp_delta(log_probs - old_log_probs, clip=20.0, out_dtype=log_probs.dtype)
    lo, hi = 1 - config.cispo.cispo_eps_clip_low, 1 + config.cispo.cispo_eps_clip_high
    loss = -advantages * torch.clamp(ratio, lo, hi).detach() * log_probs
    m = {"clip_ratio": masked_mean(((ratio < lo) | (ratio > hi)).float(), loss_mask).mean().item()}
    loss, loss_mask, extra = apply_off_policy_correction(loss, old_log_probs, rollout_logprobs, loss_mask,
                                                         config.off_policy_correction)
    m.update(extra)
    return _reduce(loss, loss_mask, config.loss_reduction, config.max_seq_len), m


def compute_policy_loss_clip_cov(log_probs, old_log_probs, advantages, config, loss_mask=None,
                                 rollout_logprobs=None):
    cc = config.clip_cov
    ratio = torch.exp(log_probs - old_log_probs)
    l1 = -advantages * ratio
    l2 = -advantages * torch.clamp(ratio, 1 - config.eps_clip_low, 1 + config.eps_clip_high)
    clipped = (l2 > l1) & (loss_mask > 0)
    cov = (advantages - masked_mean(advantages, loss_mask)) * (log_probs - masked_mean(log_probs.detach(), loss_mask))
    cov[loss_mask == 0] = -torch.inf
    cov[clipped] = -torch.inf
    k = max(int(cc.clip_ratio * loss_mask.sum().item()), 1)
    cand = torch.nonzero((cov < cc.clip_cov_ub) & (cov > cc.clip_cov_lb) & (loss_mask > 0))
    corr = torch.ones_like(advantages)
    if len(cand) > 0:
        cand = cand[torch.randperm(len(cand))[: min(k, len(cand))]]
        corr[cand[:, 0], cand[:, 1]] = 0
    frac = masked_mean((corr == 0).float(), loss_mask)
    loss = _reduce(torch.maximum(l1, l2) * corr, loss_mask, config.loss_reduction, config.max_seq_len)
    return loss, {"clip_ratio": frac.item()}


def compute_policy_loss_kl_cov(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    kc = config.kl_cov
    nk = log_probs - old_log_probs
    ratio = torch.exp(nk)
    l1 = -advantages * ratio
    lkl = -advantages * ratio + kc.ppo_kl_coef * nk.abs()
    out = l1.clone()
    valid = loss_mask > 0
    vidx = torch.nonzero(valid.reshape(-1), as_tuple=True)[0]
    a = advantages[valid].detach().reshape(-1).cpu()
    lp = log_probs[valid].detach().reshape(-1).cpu()
    if len(a) > 0:
        cov = (a - a.mean()) * (lp - lp.mean())
        k = max(1, int(len(cov) * kc.kl_cov_frac))
        top = torch.topk(cov, min(k, len(cov)), largest=True).indices
        if len(top) > 0:
            sel = vidx[top.to(vidx.device)]
            R = advantages.shape[1]
            out[sel // R, sel % R] = lkl[sel // R, sel % R]
    return _reduce(out, loss_mask, config.loss_reduction, config.max_seq_len), {"clip_ratio": 0.0}


def cross_entropy_loss(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    el = -log_probs
    loss = (el * loss_mask).sum() if loss_mask is not None else el.sum()
    return loss, {"clip_ratio": 0.0}


def importance_sampling_loss(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    r = torch.exp(log_probs - old_log_probs)
    el = -(r * advantages)
    if loss_mask is not None:
        loss = (el * loss_mask).sum()
        mr = (r * loss_mask).sum() / loss_mask.sum()
    else:
        loss = el.sum()
        mr = r.mean()
    return loss, {"importance_ratio": mr.item()}


# ----------------------------------------------------------------------------- estimators
def _whiten(values, mask):
    from .ppo_utils import masked_whiten

    return masked_whiten(values, mask)


def compute_reinforce_plus_plus_outcome_advantage(token_level_rewards, response_mask, gamma, **kwargs):
    with torch.no_grad():
        ret = torch.zeros_like(token_level_rewards)
        run = 0
        for t in reversed(range(token_level_rewards.shape[1])):
            run = token_level_rewards[:, t] + gamma * run
            ret[:, t] = run
            run = run * response_mask[:, t]
        adv = _whiten(ret, response_mask) * response_mask
    return adv, ret


def compute_rloo_outcome_advantage(token_level_rewards, response_mask, index, **kwargs):
    scores = token_level_rewards.sum(dim=-1)
    groups = defaultdict(list)
    with torch.no_grad():
        for i in range(scores.shape[0]):
            groups[index[i]].append(i)
        out = scores.clone()
        for rows in groups.values():
            n = len(rows)
            if n == 1:
                out[rows[0]] = 0.0
                continue
            mu = torch.mean(torch.stack([scores[i] for i in rows]))
            for i in rows:
                out[i] = (scores[i] - mu) * (n / (n - 1))
        out = out.unsqueeze(-1) * response_mask
    return out, out
