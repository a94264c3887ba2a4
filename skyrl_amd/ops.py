"""torch-facing wrappers of the HIP hot path (device tensors in, device tensors out).

Each function validates shapes/dtypes/devices on the host, takes the current HIP stream,
and calls one C-ABI entry point (skyrl_amd._ffi). Nothing here computes on the CPU: a
CPU tensor, a missing GPU or a missing library is an error, never a fallback.
"""

from __future__ import annotations

import ctypes
from typing import Dict, Optional, Sequence, Tuple

import torch

from . import _ffi
from ._ffi import BF16, F32, I32, I64, U8
from ._ffi import set_default_variant, variant  # noqa: F401  (per-call kernel variants, skyrl_variant)

_MASK_DTYPES = {torch.float32: F32, torch.int64: I64, torch.int32: I32, torch.bool: U8, torch.uint8: U8}
KL_TYPES = {"k1": 0, "abs": 1, "k2": 2, "k3": 3}
LOSS_REDUCTIONS = {"token_mean": 0, "sequence_mean": 1, "seq_mean_token_sum_norm": 2}


# ---------------------------------------------------------------------------- plumbing
def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_gpu(*tensors: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "skyrl_amd HIP path requires device tensors (got a tensor on "
                f"{t.device}); there is no CPU fallback"
            )
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} vs {t.device}")
    if dev is None:
        raise RuntimeError("no device tensor given")
    return dev


def _f32c(t: Optional[torch.Tensor], name: str) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    return t.contiguous()


class _Workspaces:
    """Zero-initialised scratch per (device, stream, kind); grows, never shrinks.

    Kernels with an in-launch last-arriver counter (ppo loss, critic loss, reward KL,
    sampler) rely on the counter words being zero at allocation; the kernel re-arms them.
    """

    def __init__(self):
        self._bufs: Dict[Tuple, torch.Tensor] = {}

    def get(self, device: torch.device, kind: str, nbytes: int) -> torch.Tensor:
        stream = torch.cuda.current_stream(device).cuda_stream
        key = (device.index, stream, kind)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            nbytes = max(int(nbytes), 256)
            buf = torch.zeros(nbytes, dtype=torch.uint8, device=device)
            self._bufs[key] = buf
        return buf


WORKSPACES = _Workspaces()


# ---------------------------------------------------------------------------- a4 GRPO
def groups_from_index(index: Sequence) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """Map the reference's per-row uid list (`index`) to CSR groups (host, O(N)).

    Mirrors the grouping of compute_grpo_outcome_advantage (ppo_utils.py:1160-1163):
    rows sharing a uid form one group, in first-appearance order.
    """
    order: Dict = {}
    members = []
    for i, uid in enumerate(index):
        key = uid.item() if hasattr(uid, "item") else uid
        g = order.get(key)
        if g is None:
            g = order[key] = len(members)
            members.append([])
        members[g].append(i)
    off = [0]
    rows = []
    for m in members:
        rows.extend(m)
        off.append(len(rows))
    return torch.tensor(off, dtype=torch.int32), torch.tensor(rows, dtype=torch.int32), len(members)


def contiguous_group_size(group_off: torch.Tensor, group_rows: torch.Tensor, num_groups: int) -> int:
    """G if the CSR groups are rows [g*G, (g+1)*G) for every g (the trainer's layout), else 0."""
    n = int(group_rows.numel())
    if num_groups <= 0 or n % num_groups:
        return 0
    G = n // num_groups
    if G > 16:
        return 0
    off = group_off.cpu()
    rows = group_rows.cpu()
    if torch.equal(rows, torch.arange(n, dtype=rows.dtype)) and torch.equal(
            off, torch.arange(0, n + 1, G, dtype=off.dtype)):
        return G
    return 0


def grpo_advantage(
    token_level_rewards: torch.Tensor,
    response_mask: torch.Tensor,
    group_off: Optional[torch.Tensor],
    group_rows: Optional[torch.Tensor],
    num_groups: int,
    epsilon: float = 1e-6,
    norm_by_std: bool = True,
    scores_out: Optional[torch.Tensor] = None,
    scores: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """a4 GRPO advantage. ``scores`` (f32 [N], the per-row reward sums pack_experience returns
    with ``return_row_sums``) skips the reward reads; the result is the same as computing them."""
    dev = _require_gpu(token_level_rewards, response_mask, scores)
    rew = _f32c(token_level_rewards, "token_level_rewards")
    if rew.dim() != 2 or response_mask.shape != rew.shape:
        raise ValueError(f"rewards {tuple(rew.shape)} and response_mask {tuple(response_mask.shape)} must match [N,R]")
    mask = response_mask.contiguous()
    if mask.dtype not in _MASK_DTYPES:
        raise TypeError(f"unsupported response_mask dtype {mask.dtype}")
    N, R = rew.shape
    if group_off is None and group_rows is None:  # contiguous groups of N / num_groups rows
        goff = grows = None
        aligned = all(t.data_ptr() % 16 == 0 for t in (rew, mask))
        if not (aligned and R % 4 == 0 and num_groups > 0 and N % num_groups == 0 and N // num_groups <= 16):
            G = N // max(num_groups, 1)  # the CSR kernel covers what the index-free one cannot
            goff = torch.arange(0, N + 1, max(G, 1), dtype=torch.int32, device=dev)[: num_groups + 1]
            grows = torch.arange(N, dtype=torch.int32, device=dev)
    else:
        goff = group_off.to(device=dev, dtype=torch.int32)
        grows = group_rows.to(device=dev, dtype=torch.int32)
    sc = None
    if scores is not None:
        sc = _f32c(scores.detach(), "scores")
        if tuple(sc.shape) != (N,):
            raise ValueError(f"scores shape {tuple(sc.shape)} != {(N,)}")
    out = torch.empty((N, R), dtype=torch.float32, device=dev)
    _ffi.call(
        "skyrl_grpo_advantage", _ptr(rew), _ptr(sc), _ptr(mask), _MASK_DTYPES[mask.dtype], _ptr(goff), _ptr(grows),
        int(num_groups), N, R, float(epsilon), int(bool(norm_by_std)), _ptr(out), _ptr(scores_out), _stream(dev),
    )
    return out


def normalize_advantages(advantages: torch.Tensor, response_mask: torch.Tensor, group=None) -> torch.Tensor:
    """advantage_batch_normalize (ppo_utils.py:127-145, trainer.py:275-276): (adv - mean) * rstd
    with the unmasked mean over every element and rstd = rsqrt(clamp(sum((adv - mean)^2 * mask) /
    sum(mask), 1e-8)), returned as a new tensor (the reference does not re-mask). Two launches:
    the five fp64 sums (sum a, sum m, sum a m, sum a^2 m, count), then the apply pass. With a
    data-parallel `group` (each rank holding its rows of one global batch, as the reference
    normalizes the whole batch on the driver) the sums are SUM-all-reduced between them: one
    collective of 5 fp64 scalars, no host sync."""
    dev = _require_gpu(advantages, response_mask)
    adv = _f32c(advantages.detach(), "advantages")
    mask = response_mask.contiguous()
    if mask.dtype not in _MASK_DTYPES:
        raise TypeError(f"unsupported response_mask dtype {mask.dtype}")
    if mask.shape != adv.shape:
        raise ValueError(f"advantages {tuple(adv.shape)} and response_mask {tuple(mask.shape)} must match")
    sums = torch.empty(5, dtype=torch.float64, device=dev)
    ws = WORKSPACES.get(dev, "adv_norm", _ffi.query("skyrl_adv_norm_workspace_bytes"))
    _ffi.call("skyrl_adv_norm_stats", _ptr(adv), _ptr(mask), _MASK_DTYPES[mask.dtype], adv.numel(), _ptr(sums),
              _ptr(ws), _stream(dev))
    if group is not None and torch.distributed.get_world_size(group) > 1:
        torch.distributed.all_reduce(sums, group=group)
    out = torch.empty_like(adv)
    _ffi.call("skyrl_adv_norm_apply", _ptr(adv), adv.numel(), _ptr(sums), _ptr(out), _stream(dev))
    return out


# ---------------------------------------------------------------------------- a5 GAE
def gae_advantage_return(
    token_level_rewards: torch.Tensor,
    values: torch.Tensor,
    response_mask: torch.Tensor,
    gamma: float,
    lambd: float,
    check: bool = True,
) -> Tuple[torch.Tensor, torch.Tensor]:
    dev = _require_gpu(token_level_rewards, values, response_mask)
    rew = _f32c(token_level_rewards, "token_level_rewards")
    val = _f32c(values, "values")
    mask = response_mask.contiguous()
    if mask.dtype not in _MASK_DTYPES:
        raise TypeError(f"unsupported response_mask dtype {mask.dtype}")
    if rew.dim() != 2 or val.shape != rew.shape or mask.shape != rew.shape:
        raise ValueError("rewards, values and response_mask must all be [N,R]")
    N, R = rew.shape
    adv = torch.empty_like(rew)
    ret = torch.empty_like(rew)
    ws = WORKSPACES.get(dev, "gae", _ffi.query("skyrl_gae_workspace_bytes", N))
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    _ffi.call(
        "skyrl_gae_advantage_return", _ptr(rew), _ptr(val), _ptr(mask), _MASK_DTYPES[mask.dtype], N, R,
        float(gamma), float(lambd), _ptr(adv), _ptr(ret), _ptr(ws), _ptr(status), _stream(dev),
    )
    if check:  # the reference raises from masked_var (ppo_utils.py:157-163); one sync
        st = int(status.item())
        if st == 1:
            raise ValueError("At least one element in the mask has to be 1.")
        if st == 2:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
    return adv, ret


# ---------------------------------------------------------------------------- a6 KL
def approx_kl(
    log_probs: torch.Tensor,
    log_probs_base: torch.Tensor,
    loss_mask: Optional[torch.Tensor] = None,
    kl_estimator_type: str = "k3",
) -> torch.Tensor:
    if kl_estimator_type not in KL_TYPES:
        raise ValueError(f"Invalid KL estimator type: {kl_estimator_type}")
    dev = _require_gpu(log_probs, log_probs_base, loss_mask)
    lp = _f32c(log_probs, "log_probs")
    base = _f32c(log_probs_base, "log_probs_base")
    if base.shape != lp.shape:
        raise ValueError("log_probs and log_probs_base must have the same shape")
    mask = None
    mdt = F32
    if loss_mask is not None:
        mask = loss_mask.contiguous()
        if mask.shape != lp.shape:
            mask = mask.expand_as(lp).contiguous()
        mdt = _MASK_DTYPES[mask.dtype]
    out = torch.empty_like(lp)
    _ffi.call(
        "skyrl_approx_kl", _ptr(lp), _ptr(base), _ptr(mask), mdt, lp.numel(), KL_TYPES[kl_estimator_type],
        _ptr(out), _stream(dev),
    )
    return out


def reward_kl_penalty(
    rewards: torch.Tensor,
    action_log_probs: torch.Tensor,
    base_action_log_probs: torch.Tensor,
    loss_mask: torch.Tensor,
    kl_estimator_type: str,
    kl_coef: float,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (new rewards, device tensor [avg_kl, avg_kl_max])."""
    dev = _require_gpu(rewards, action_log_probs, base_action_log_probs, loss_mask)
    rew = _f32c(rewards, "rewards")
    lp = _f32c(action_log_probs, "action_log_probs")
    base = _f32c(base_action_log_probs, "base_action_log_probs")
    mask = loss_mask.to(torch.float32).contiguous()
    N, R = rew.shape
    out = torch.empty_like(rew)
    metrics = torch.empty(2, dtype=torch.float32, device=dev)
    ws = WORKSPACES.get(dev, "reward_kl", _ffi.query("skyrl_reward_kl_workspace_bytes", N))
    _ffi.call(
        "skyrl_reward_kl_penalty", _ptr(rew), _ptr(lp), _ptr(base), _ptr(mask), N, R,
        KL_TYPES[kl_estimator_type], float(kl_coef), _ptr(out), _ptr(metrics), _ptr(ws), _stream(dev),
    )
    return out, metrics


# ---------------------------------------------------------------------------- a7 PPO loss
def make_ppo_params(
    *,
    eps_clip_low: float = 0.2,
    eps_clip_high: float = 0.2,
    clip_ratio_c: float = 3.0,
    policy_loss_type: str = "regular",
    loss_reduction: str = "token_mean",
    max_seq_len: Optional[float] = None,
    use_kl_loss: bool = False,
    kl_estimator_type: str = "k3",
    kl_loss_coef: float = 0.0,
    use_entropy_loss: bool = False,
    entropy_loss_coef: float = 0.0,
    has_entropy: bool = False,
) -> _ffi.PPOParams:
    if policy_loss_type not in ("regular", "dual_clip"):
        raise ValueError(f"HIP PPO loss supports 'regular' and 'dual_clip', got {policy_loss_type!r}")
    if loss_reduction not in LOSS_REDUCTIONS:
        raise ValueError(
            "loss_reduction must be either 'token_mean', 'sequence_mean', or 'seq_mean_token_sum_norm'"
        )
    if loss_reduction == "seq_mean_token_sum_norm" and max_seq_len is None:
        raise AssertionError("max_seq_len must be provided for seq_mean_token_sum_norm loss reduction")
    if kl_estimator_type not in KL_TYPES:
        raise ValueError(f"Invalid KL estimator type: {kl_estimator_type}")
    return _ffi.PPOParams(
        float(eps_clip_low), float(eps_clip_high), float(clip_ratio_c), int(policy_loss_type == "dual_clip"),
        LOSS_REDUCTIONS[loss_reduction], float(max_seq_len or 0.0), int(bool(use_kl_loss)),
        KL_TYPES[kl_estimator_type], float(kl_loss_coef), int(bool(use_entropy_loss)), float(entropy_loss_coef),
        int(bool(has_entropy)),
    )


FOLD_TIMEOUT_SLOT = 6  # metrics[6] = 1: an in-launch fold's bounded spin timed out (loss/metrics NaN)


def check_loss_metrics(metrics) -> None:
    """Raise when a loss launch's cross-workgroup exchange timed out (metrics[6] != 0): the
    in-launch fold of skyrl_ppo_loss_fwd / skyrl_grpo_ppo_loss_fwd (loss and metrics NaN, the
    gradients written), or a split row's state exchange in skyrl_policy_train_fwd (that row's
    outputs NaN). Training must not go on silently. ``metrics`` is one [8] vector or rows of
    them, device or host; one host read."""
    m = torch.as_tensor(metrics)
    flag = m.reshape(-1, m.shape[-1])[:, FOLD_TIMEOUT_SLOT]
    if bool((flag != 0).any()):
        raise RuntimeError("fused PPO loss: a cross-workgroup exchange (loss fold or split-row softmax state) "
                           "timed out (metrics[6] = 1; the affected outputs are NaN)")


def _loss_workspace(dev, n, R, defer):
    nbytes = _ffi.query("skyrl_ppo_loss_workspace_bytes", n, R)
    if defer:  # the records live until this call's backward: a workspace of its own (no zeroing needed)
        return torch.empty(nbytes, dtype=torch.uint8, device=dev)
    return WORKSPACES.get(dev, "ppo", nbytes)


def _loss_backward(ctx, grad_loss):
    if ctx.used:  # the gradients are rescaled in place
        raise RuntimeError("the fused PPO loss supports a single backward pass")
    ctx.used = True
    glp, gent, loss, metrics = ctx.saved_tensors
    g = grad_loss.detach().to(torch.float32).reshape(1).contiguous()
    if ctx.defer:  # fold the forward's records into loss/metrics + rescale, one launch
        _ffi.call("skyrl_ppo_loss_finish", _ptr(g), _ptr(glp), _ptr(gent), glp.shape[0], glp.shape[1],
                  ctypes.byref(ctx.params), _ptr(loss), _ptr(metrics), _ptr(ctx.ws), _stream(glp.device))
    else:
        _ffi.call("skyrl_ppo_loss_bwd", _ptr(g), glp.numel(), _ptr(glp), _ptr(gent), _stream(glp.device))
    return glp, gent


def _loss_finish_now(n, R, params, loss, metrics, ws, dev):
    """A deferred forward whose backward will not run (no grad): fold now."""
    _ffi.call("skyrl_ppo_loss_finish", None, None, None, n, R, ctypes.byref(params), _ptr(loss), _ptr(metrics),
              _ptr(ws), _stream(dev))


class PPOLossFunction(torch.autograd.Function):
    """Fused policy loss (+KL(ref) +entropy term): ONE HIP launch computes the loss, the
    metrics and the final dL/dlogp (and dL/dentropy) for a unit upstream gradient; the
    backward rescales them in place only when the upstream gradient is not 1.

    forward returns (loss 0-d, metrics f32[8] device). Gradients flow to log_probs and,
    when params.use_entropy_loss, to entropy. The KL term has no gradient (reference:
    compute_approx_kl is @torch.no_grad(), ppo_utils.py:87).

    defer_fold: the forward writes gradients and per-block records only, and the backward's
    single launch (skyrl_ppo_loss_finish) folds them into loss/metrics and rescales: one
    launch less and no in-launch fold. loss/metrics are then valid after backward (the
    reference reads them there, workers/worker.py:876-894); when no backward can follow
    (grad disabled or no differentiable input) the fold runs at once. One backward per call
    (the gradients are rescaled in place).
    """

    @staticmethod
    def forward(ctx, log_probs, old_log_probs, advantages, loss_mask, ref_log_probs, entropy, params,
                loss_mask_row_sum, defer_fold=False):
        dev = _require_gpu(log_probs, old_log_probs, advantages, loss_mask, ref_log_probs, entropy)
        lp = _f32c(log_probs.detach(), "log_probs")
        old = _f32c(old_log_probs.detach(), "old_log_probs")
        adv = _f32c(advantages.detach(), "advantages")
        mask = None if loss_mask is None else loss_mask.detach().to(torch.float32).contiguous()
        ref = None if ref_log_probs is None else _f32c(ref_log_probs.detach(), "ref_log_probs")
        ent = None if entropy is None else _f32c(entropy.detach(), "entropy")
        if lp.dim() != 2:
            raise ValueError(f"log_probs must be [n,R], got {tuple(lp.shape)}")
        for name, t in (("old_log_probs", old), ("advantages", adv), ("loss_mask", mask), ("ref", ref), ("entropy", ent)):
            if t is not None and t.shape != lp.shape:
                raise ValueError(f"{name} shape {tuple(t.shape)} != log_probs shape {tuple(lp.shape)}")
        n, R = lp.shape
        rows = None
        if loss_mask_row_sum is not None:
            rows = _f32c(loss_mask_row_sum.detach(), "loss_mask_row_sum")
            if tuple(rows.shape) != (n,):
                raise ValueError(f"loss_mask_row_sum shape {tuple(rows.shape)} != {(n,)}")
        loss = torch.empty((), dtype=torch.float32, device=dev)
        metrics = torch.empty(_ffi.M_COUNT, dtype=torch.float32, device=dev)
        glp = torch.empty_like(lp)
        want_ent = bool(params.use_entropy_loss) and entropy is not None and ctx.needs_input_grad[5]
        gent = torch.empty_like(lp) if want_ent else None
        defer = bool(defer_fold)
        ws = _loss_workspace(dev, n, R, defer)
        _ffi.call(
            "skyrl_ppo_loss_fwd", _ptr(lp), _ptr(old), _ptr(adv), _ptr(mask), _ptr(ref), _ptr(ent), _ptr(rows), n, R,
            ctypes.byref(params), _ptr(loss), _ptr(metrics), _ptr(glp), _ptr(gent),
            _ffi.LOSS_DEFER_FOLD if defer else 0, _ptr(ws), _stream(dev),
        )
        if defer and not (ctx.needs_input_grad[0] or ctx.needs_input_grad[5]):
            _loss_finish_now(n, R, params, loss, metrics, ws, dev)
            defer = False
        ctx.save_for_backward(glp, gent, loss, metrics)
        ctx.mark_non_differentiable(metrics)
        ctx.used, ctx.defer, ctx.n, ctx.params, ctx.ws = False, defer, n, params, ws
        return loss, metrics

    @staticmethod
    def backward(ctx, grad_loss, grad_metrics):
        glp, gent = _loss_backward(ctx, grad_loss)
        return glp, None, None, None, None, gent, None, None, None


class GRPOPPOLossFunction(torch.autograd.Function):
    """GRPO advantage (contiguous groups) + the fused policy loss for a batch that is one
    micro-batch: ``skyrl_grpo_ppo_loss_fwd``, ONE launch when the layout allows (see the
    header), with outputs bit-identical to ``grpo_advantage`` followed by ``ppo_loss``.
    forward returns (advantages [n,R], loss 0-d, metrics f32[8]); gradients flow to
    log_probs (and entropy), exactly as ``PPOLossFunction`` (defer_fold included)."""

    @staticmethod
    def forward(ctx, token_level_rewards, response_mask, num_groups, epsilon, norm_by_std, log_probs, old_log_probs,
                loss_mask, ref_log_probs, entropy, params, loss_mask_row_sum, scores=None, defer_fold=False,
                want_advantages=True, mask_within_response=False):
        dev = _require_gpu(token_level_rewards, response_mask, log_probs, old_log_probs, loss_mask, ref_log_probs,
                           entropy, scores)
        rew = _f32c(token_level_rewards.detach(), "token_level_rewards")
        rmask = response_mask.detach().contiguous()
        if rmask.dtype not in _MASK_DTYPES:
            raise TypeError(f"unsupported response_mask dtype {rmask.dtype}")
        lp = _f32c(log_probs.detach(), "log_probs")
        old = _f32c(old_log_probs.detach(), "old_log_probs")
        mask = None if loss_mask is None else loss_mask.detach().to(torch.float32).contiguous()
        ref = None if ref_log_probs is None else _f32c(ref_log_probs.detach(), "ref_log_probs")
        ent = None if entropy is None else _f32c(entropy.detach(), "entropy")
        if lp.dim() != 2:
            raise ValueError(f"log_probs must be [n,R], got {tuple(lp.shape)}")
        for name, t in (("token_level_rewards", rew), ("response_mask", rmask), ("old_log_probs", old),
                        ("loss_mask", mask), ("ref", ref), ("entropy", ent)):
            if t is not None and t.shape != lp.shape:
                raise ValueError(f"{name} shape {tuple(t.shape)} != log_probs shape {tuple(lp.shape)}")
        n, R = lp.shape
        rows = None if loss_mask_row_sum is None else _f32c(loss_mask_row_sum.detach(), "loss_mask_row_sum")
        sc = None
        if scores is not None:
            sc = _f32c(scores.detach(), "scores")
            if tuple(sc.shape) != (n,):
                raise ValueError(f"scores shape {tuple(sc.shape)} != {(n,)}")
        want_ent = bool(params.use_entropy_loss) and entropy is not None and ctx.needs_input_grad[9]
        # the C entry's one-launch conditions (skyrl_grpo_ppo_loss_fwd); the two-launch form needs
        # the advantages buffer and the response mask
        need_total = params.loss_reduction == 0 or want_ent
        one_launch = rows is not None and n * ((R + 1023) // 1024) <= 2048 and not (need_total and n > 1024)
        want_adv = bool(want_advantages) or not one_launch
        adv = torch.empty_like(lp) if want_adv else None
        # without the advantages output the response mask is not read when the caller guarantees
        # loss_mask == 0 outside the response (pack's layout): then every loss token uses its row's
        # advantage, exactly what adv * response_mask gives it
        rm_arg = rmask if (want_adv or not mask_within_response) else None
        loss = torch.empty((), dtype=torch.float32, device=dev)
        metrics = torch.empty(_ffi.M_COUNT, dtype=torch.float32, device=dev)
        glp = torch.empty_like(lp)
        gent = torch.empty_like(lp) if want_ent else None
        defer = bool(defer_fold)
        ws = _loss_workspace(dev, n, R, defer)
        _ffi.call(
            "skyrl_grpo_ppo_loss_fwd", _ptr(rew), _ptr(sc), _ptr(rm_arg), _MASK_DTYPES[rmask.dtype], int(num_groups),
            float(epsilon), int(bool(norm_by_std)), _ptr(lp), _ptr(old), _ptr(mask), _ptr(ref), _ptr(ent), _ptr(rows),
            n, R, ctypes.byref(params), _ptr(adv), _ptr(loss), _ptr(metrics), _ptr(glp), _ptr(gent),
            _ffi.LOSS_DEFER_FOLD if defer else 0, _ptr(ws), _stream(dev),
        )
        if defer and not (ctx.needs_input_grad[5] or ctx.needs_input_grad[9]):
            _loss_finish_now(n, R, params, loss, metrics, ws, dev)
            defer = False
        ctx.save_for_backward(glp, gent, loss, metrics)
        if adv is not None:
            ctx.mark_non_differentiable(adv, metrics)
        else:
            ctx.mark_non_differentiable(metrics)
        ctx.used, ctx.defer, ctx.n, ctx.params, ctx.ws = False, defer, n, params, ws
        return (adv if want_advantages else None), loss, metrics

    @staticmethod
    def backward(ctx, grad_adv, grad_loss, grad_metrics):
        glp, gent = _loss_backward(ctx, grad_loss)
        return None, None, None, None, None, glp, None, None, None, gent, None, None, None, None, None, None


def grpo_ppo_loss(token_level_rewards, response_mask, num_groups, log_probs, old_log_probs, loss_mask, params,
                  ref_log_probs=None, entropy=None, loss_mask_row_sum=None, epsilon=1e-6, norm_by_std=True,
                  scores=None, defer_fold=False, want_advantages=True, mask_within_response=False):
    """GRPO advantage + fused loss in one call; returns (advantages, loss, metrics). Layouts
    the C entry's contiguous form cannot take (R % 4 != 0, groups > 16 rows, unaligned
    buffers) run the two HIP calls, with the CSR GRPO kernel. ``scores``: the per-row reward
    sums (pack_experience(return_row_sums=True)); ``defer_fold``: see PPOLossFunction.
    ``want_advantages=False`` skips the advantages output (returned as None) on the one-launch
    layout; with ``mask_within_response`` (the caller guarantees loss_mask is 0 outside the
    response, as pack's output is) the response mask is not read either."""
    n, R = log_probs.shape
    ng = int(num_groups)
    if ng > 0 and n % ng == 0:
        tens = (token_level_rewards, response_mask, log_probs, old_log_probs, loss_mask, ref_log_probs, entropy,
                scores)
        contiguous_ok = R % 4 == 0 and n // ng <= 16 and all(
            t is None or (t.is_contiguous() and t.data_ptr() % 16 == 0) for t in tens)
        if not contiguous_ok:
            adv = grpo_advantage(token_level_rewards, response_mask, None, None, ng, epsilon, norm_by_std,
                                 scores=scores)
            loss, metrics = ppo_loss(log_probs, old_log_probs, adv, loss_mask, params, ref_log_probs, entropy,
                                     loss_mask_row_sum, defer_fold=defer_fold)
            return (adv if want_advantages else None), loss, metrics
    return GRPOPPOLossFunction.apply(token_level_rewards, response_mask, num_groups, epsilon, norm_by_std, log_probs,
                                     old_log_probs, loss_mask, ref_log_probs, entropy, params, loss_mask_row_sum,
                                     scores, defer_fold, want_advantages, mask_within_response)


def ppo_loss(log_probs, old_log_probs, advantages, loss_mask, params, ref_log_probs=None, entropy=None,
             loss_mask_row_sum=None, defer_fold=False):
    """Fused loss; returns (loss 0-d tensor, metrics device tensor [8]). ``loss_mask_row_sum``
    (f32 [n], per-row sums of ``loss_mask``, as pack_experience emits them) saves one launch.
    One backward per call. ``defer_fold`` moves the loss/metric fold into the backward launch
    (loss and metrics valid after backward; see PPOLossFunction)."""
    return PPOLossFunction.apply(log_probs, old_log_probs, advantages, loss_mask, ref_log_probs, entropy, params,
                                 loss_mask_row_sum, defer_fold)


# ---------------------------------------------------------------------------- a8 critic loss
class CriticLossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, values, old_values, returns, loss_mask, value_clip):
        dev = _require_gpu(values, old_values, returns, loss_mask)
        v = _f32c(values.detach(), "values")
        ov = None if old_values is None else _f32c(old_values.detach(), "old_values")
        ret = _f32c(returns.detach(), "returns")
        mask = None if loss_mask is None else loss_mask.detach().to(torch.float32).contiguous()
        n, R = v.shape
        loss = torch.empty((), dtype=torch.float32, device=dev)
        clipfrac = torch.empty(1, dtype=torch.float32, device=dev)
        gv = torch.empty_like(v)
        ws = WORKSPACES.get(dev, "critic", _ffi.query("skyrl_critic_loss_workspace_bytes", n, R))
        vc = -1.0 if value_clip is None else float(value_clip)
        _ffi.call(
            "skyrl_critic_loss_fwd", _ptr(v), _ptr(ov), _ptr(ret), _ptr(mask), n, R, vc, _ptr(loss),
            _ptr(clipfrac), _ptr(gv), _ptr(ws), _stream(dev),
        )
        ctx.save_for_backward(gv)
        ctx.mark_non_differentiable(clipfrac)
        return loss, clipfrac

    @staticmethod
    def backward(ctx, grad_loss, grad_clip):
        (gv,) = ctx.saved_tensors
        out = torch.empty_like(gv)
        g = grad_loss.detach().to(torch.float32).reshape(1).contiguous()
        _ffi.call("skyrl_scale_by_device_scalar", _ptr(g), _ptr(gv), _ptr(out), gv.numel(), _stream(gv.device))
        return out, None, None, None, None


# ---------------------------------------------------------------------------- a2/a3 logprob
def _logits_view(logits: torch.Tensor):
    """[nb, nt, V] (or [T, V]) with unit vocab stride -> (nb, nt, V, sb, st, dtype code)."""
    if logits.dtype == torch.bfloat16:
        dt = BF16
    elif logits.dtype == torch.float32:
        dt = F32
    else:
        raise TypeError(f"logits must be bf16 or f32, got {logits.dtype}")
    if logits.dim() == 2:
        logits = logits.unsqueeze(0)
    if logits.dim() != 3:
        raise ValueError(f"logits must be [nb, nt, V] or [T, V], got {tuple(logits.shape)}")
    if logits.stride(2) != 1:
        raise ValueError("logits must be contiguous along the vocab dimension")
    nb, nt, V = logits.shape
    return logits, nb, nt, V, logits.stride(0), logits.stride(1), dt


def _labels_view(labels: torch.Tensor, nb: int, nt: int):
    if labels.dtype != torch.int64:
        labels = labels.to(torch.int64)
    if labels.dim() == 1:
        labels = labels.unsqueeze(0)
    if tuple(labels.shape) != (nb, nt):
        raise ValueError(f"labels shape {tuple(labels.shape)} != logits leading shape {(nb, nt)}")
    return labels, labels.stride(0), labels.stride(1)


class LogprobEntropyFunction(torch.autograd.Function):
    """logits [nb,nt,V] (bf16/f32, any row strides) -> (logp f32 [nb,nt], entropy f32 [nb,nt])."""

    @staticmethod
    def forward(ctx, logits, labels, temperature, compute_entropy):
        dev = _require_gpu(logits, labels)
        lg, nb, nt, V, sb, st, dt = _logits_view(logits.detach())
        lab, lsb, lst = _labels_view(labels, nb, nt)
        logp = torch.empty((nb, nt), dtype=torch.float32, device=dev)
        ent = torch.empty((nb, nt), dtype=torch.float32, device=dev)
        lse = torch.empty((nb, nt), dtype=torch.float32, device=dev)
        _ffi.call(
            "skyrl_logprob_fwd", _ptr(lg), dt, sb, st, nb, nt, V, _ptr(lab), lsb, lst, float(temperature),
            _ptr(logp), _ptr(ent), _ptr(lse), _stream(dev),
        )
        ctx.temperature = float(temperature)
        ctx.in_shape = logits.shape
        ctx.save_for_backward(logits, lab, lse, ent)
        if not compute_entropy:
            ctx.mark_non_differentiable(ent)
        if logits.dim() == 2:
            return logp.squeeze(0), ent.squeeze(0)
        return logp, ent

    @staticmethod
    def backward(ctx, g_logp, g_ent):
        logits, lab, lse, ent = ctx.saved_tensors
        lg, nb, nt, V, sb, st, dt = _logits_view(logits.detach())
        dev = lg.device
        glp = (torch.zeros((nb, nt), dtype=torch.float32, device=dev) if g_logp is None
               else g_logp.to(torch.float32).reshape(nb, nt).contiguous())
        gent = None if g_ent is None else g_ent.to(torch.float32).reshape(nb, nt).contiguous()
        dx = torch.empty((nb, nt, V), dtype=lg.dtype, device=dev)
        _ffi.call(
            "skyrl_logprob_bwd", _ptr(lg), dt, sb, st, nb, nt, V, _ptr(lab), lab.stride(0), lab.stride(1),
            ctx.temperature, _ptr(lse), _ptr(ent), _ptr(glp), _ptr(gent), _ptr(dx), _stream(dev),
        )
        return dx.reshape(ctx.in_shape), None, None, None


def logprobs_and_entropy(logits, labels, temperature: float = 1.0, compute_entropy: bool = True):
    return LogprobEntropyFunction.apply(logits, labels, temperature, compute_entropy)


# ---------------------------------------------------------------------------- fused training pass
class PolicyTrainFunction(torch.autograd.Function):
    """logits -> (loss, metrics, logp, entropy) with dlogits produced in the same pass.

    Equivalent to logprobs_and_entropy + ppo_loss (+ their backward) for regular/dual_clip
    PPO; gradients flow to `logits` only (logp/entropy are returned for logging).
    """

    @staticmethod
    def forward(ctx, logits, labels, old_log_probs, advantages, loss_mask, ref_log_probs, params, temperature):
        dev = _require_gpu(logits, labels, old_log_probs, advantages, loss_mask, ref_log_probs)
        lg, nb, nt, V, sb, st, dt = _logits_view(logits.detach())
        if dt != BF16:
            raise TypeError("the fused training pass takes bf16 logits")
        lab, lsb, lst = _labels_view(labels, nb, nt)
        old = _f32c(old_log_probs.detach(), "old_log_probs")
        adv = _f32c(advantages.detach(), "advantages")
        mask = None if loss_mask is None else loss_mask.detach().to(torch.float32).contiguous()
        ref = None if ref_log_probs is None else _f32c(ref_log_probs.detach(), "ref_log_probs")
        for name, t in (("old_log_probs", old), ("advantages", adv), ("loss_mask", mask), ("ref_log_probs", ref)):
            if t is not None and tuple(t.shape) != (nb, nt):
                raise ValueError(f"{name} shape {tuple(t.shape)} != {(nb, nt)}")
        loss = torch.empty((), dtype=torch.float32, device=dev)
        metrics = torch.empty(_ffi.M_COUNT, dtype=torch.float32, device=dev)
        logp = torch.empty((nb, nt), dtype=torch.float32, device=dev)
        ent = torch.empty((nb, nt), dtype=torch.float32, device=dev)
        if V % 8 == 0 and lg.data_ptr() % 16 == 0 and sb % 8 == 0 and st % 8 == 0:
            flat = torch.empty(nb * nt * V, dtype=torch.bfloat16, device=dev)
            dx = flat.view(nb, nt, V)
        else:
            # rows not 16-B aligned (GPT-2's odd V): dlogits rows mirror the logits rows' strides
            # and position within 16 B, which the register-resident kernel needs
            off = (lg.data_ptr() // 2) % 8
            flat = torch.empty(off + (nb - 1) * sb + (nt - 1) * st + V, dtype=torch.bfloat16, device=dev)
            dx = flat.as_strided((nb, nt, V), (sb, st, 1), storage_offset=off)
        ws = WORKSPACES.get(dev, "policy_train", _ffi.query("skyrl_policy_train_workspace_bytes", nb, nt))
        _ffi.call(
            "skyrl_policy_train_fwd", _ptr(lg), dt, sb, st, nb, nt, V, _ptr(lab), lsb, lst, float(temperature),
            _ptr(old), _ptr(adv), _ptr(mask), _ptr(ref), ctypes.byref(params), _ptr(loss), _ptr(metrics),
            _ptr(logp), _ptr(ent), _ptr(dx), dx.stride(0), dx.stride(1), _ptr(ws), _stream(dev),
        )
        ctx.in_shape = logits.shape
        ctx.save_for_backward(dx, flat)
        ctx.mark_non_differentiable(metrics, logp, ent)
        return loss, metrics, logp, ent

    @staticmethod
    def backward(ctx, g_loss, g_metrics, g_logp, g_ent):
        dx, flat = ctx.saved_tensors
        g = g_loss.detach().to(torch.float32).reshape(1).contiguous()
        _ffi.call("skyrl_scale_bf16_by_device_scalar", _ptr(g), _ptr(flat), flat.numel(), _stream(dx.device))
        return dx.reshape(ctx.in_shape), None, None, None, None, None, None, None


def policy_train(logits, labels, old_log_probs, advantages, loss_mask, params, ref_log_probs=None,
                 temperature: float = 1.0):
    """Fused policy pass; returns (loss 0-d, metrics [8], logp [n,R], entropy [n,R])."""
    return PolicyTrainFunction.apply(logits, labels, old_log_probs, advantages, loss_mask, ref_log_probs, params,
                                     temperature)


class PolicyTrainRaggedFunction(torch.autograd.Function):
    """Packed logits [ntok, V] (the live response tokens of a sample-packed micro-batch) ->
    (loss, metrics, logp [n,R], entropy [n,R]) with dlogits [ntok, V] from the same pass
    (skyrl_policy_train_ragged_fwd); `token_pos` maps each token to its [n, R] position."""

    @staticmethod
    def forward(ctx, logits, labels, token_pos, old_log_probs, advantages, loss_mask, ref_log_probs, params,
                temperature):
        dev = _require_gpu(logits, labels, token_pos, old_log_probs, advantages, loss_mask, ref_log_probs)
        lg = logits.detach()
        if lg.dtype != torch.bfloat16 or lg.dim() != 2 or lg.stride(1) != 1:
            raise TypeError("ragged policy pass: logits must be bf16 [ntok, V] with unit vocab stride")
        ntok, V = lg.shape
        nb, nt = old_log_probs.shape
        lab = labels.detach().to(device=dev, dtype=torch.int64).contiguous().view(-1)
        pos = token_pos.detach().to(device=dev, dtype=torch.int32).contiguous().view(-1)
        if lab.numel() != ntok or pos.numel() != ntok:
            raise ValueError(f"labels / token_pos need {ntok} entries, got {lab.numel()} / {pos.numel()}")
        old = _f32c(old_log_probs.detach(), "old_log_probs")
        adv = _f32c(advantages.detach(), "advantages")
        mask = loss_mask.detach().to(torch.float32).contiguous()
        ref = None if ref_log_probs is None else _f32c(ref_log_probs.detach(), "ref_log_probs")
        for name, t in (("advantages", adv), ("loss_mask", mask), ("ref_log_probs", ref)):
            if t is not None and tuple(t.shape) != (nb, nt):
                raise ValueError(f"{name} shape {tuple(t.shape)} != {(nb, nt)}")
        loss = torch.empty((), dtype=torch.float32, device=dev)
        metrics = torch.empty(_ffi.M_COUNT, dtype=torch.float32, device=dev)
        logp = torch.zeros((nb, nt), dtype=torch.float32, device=dev)
        ent = torch.zeros((nb, nt), dtype=torch.float32, device=dev)
        dx = torch.empty((ntok, V), dtype=torch.bfloat16, device=dev)
        ws = WORKSPACES.get(dev, "policy_train", _ffi.query("skyrl_policy_train_workspace_bytes", nb, nt))
        _ffi.call("skyrl_policy_train_ragged_fwd", _ptr(lg), BF16, lg.stride(0), ntok, V, _ptr(lab), _ptr(pos), nb, nt,
                  float(temperature), _ptr(old), _ptr(adv), _ptr(mask), _ptr(ref), ctypes.byref(params), _ptr(loss),
                  _ptr(metrics), _ptr(logp), _ptr(ent), _ptr(dx), dx.stride(0), _ptr(ws), _stream(dev))
        ctx.save_for_backward(dx)
        ctx.mark_non_differentiable(metrics, logp, ent)
        return loss, metrics, logp, ent

    @staticmethod
    def backward(ctx, g_loss, g_metrics, g_logp, g_ent):
        (dx,) = ctx.saved_tensors
        g = g_loss.detach().to(torch.float32).reshape(1).contiguous()
        _ffi.call("skyrl_scale_bf16_by_device_scalar", _ptr(g), _ptr(dx), dx.numel(), _stream(dx.device))
        return dx, None, None, None, None, None, None, None, None


def policy_train_ragged(logits, labels, token_pos, old_log_probs, advantages, loss_mask, params,
                        ref_log_probs=None, temperature: float = 1.0):
    """Fused policy pass over packed tokens (see PolicyTrainRaggedFunction); returns
    (loss 0-d, metrics [8], logp [n,R], entropy [n,R]); positions no token maps to read 0."""
    return PolicyTrainRaggedFunction.apply(logits, labels, token_pos, old_log_probs, advantages, loss_mask,
                                           ref_log_probs, params, temperature)


_STEP_LAYOUT: Dict[Tuple, Tuple[int, int, int]] = {}


class PolicyTrainStep:
    """One mini-batch's fused policy passes in the step form (ABI 8, policy_train.hip):

      step = PolicyTrainStep(old, adv, loss_mask, params, micro_rows, ref_log_probs=ref)  # plan: 1 launch
      for k, (i, j) in enumerate(micro-batches):
          loss_k = step.micro(k, z_k, labels_k, token_pos_k)   # the fused pass of micro-batch k
          loss_k.backward()                                    # dlogits were written by the pass
      losses, metrics = step.fold()                            # every micro-batch's loss: 1 launch

    The reference's micro-batch loop (workers/worker.py:731-900) reads loss and metrics only
    after the mini-batch's backward passes (optim_step :900-925), so the per-micro-batch fold
    waits until then; the per-call form (policy_train / policy_train_ragged) pays two
    single-workgroup launches (scales, epilogue) per micro-batch instead. Per micro-batch the
    loss and metrics are the per-call form's bits. `micro` returns a 0-d view of `self.loss[k]`,
    valid after `fold()` (stream-ordered; nothing between reads it). Per-token arrays are the
    mini-batch's [n_total, R]; `self.logp` / `self.entropy` collect the passes' outputs
    (positions no packed token maps to stay 0). One mini-batch in flight per device and stream
    (the workspace is shared)."""

    def __init__(self, old_log_probs, advantages, loss_mask, params, micro_rows: int, ref_log_probs=None,
                 temperature: float = 1.0, grpo=None):
        """grpo (optional): dict(scores=[n_total] per-row reward sums, response_mask=[n_total, R],
        group_size=G, epsilon=1e-6, norm_by_std=True, loss_mask_row_sum=None (pack's row sums: no
        loss-mask read in the plan)): the plan launch also computes the
        mini-batch's GRPO advantages (contiguous groups of G rows) INTO `advantages`
        (skyrl_policy_train_plan_grpo), so GRPO costs no launch of its own."""
        dev = _require_gpu(old_log_probs, advantages, loss_mask, ref_log_probs)
        self.dev = dev
        self.old = _f32c(old_log_probs.detach(), "old_log_probs")
        n_total, R = self.old.shape
        self.adv = _f32c(advantages.detach(), "advantages")
        if grpo is not None and self.adv.data_ptr() != advantages.data_ptr():
            raise ValueError("grpo: advantages must be a contiguous f32 tensor (written in place)")
        self.mask = loss_mask.detach().to(torch.float32).contiguous()
        self.ref = None if ref_log_probs is None else _f32c(ref_log_probs.detach(), "ref_log_probs")
        for name, t in (("advantages", self.adv), ("loss_mask", self.mask), ("ref_log_probs", self.ref)):
            if t is not None and tuple(t.shape) != (n_total, R):
                raise ValueError(f"{name} shape {tuple(t.shape)} != {(n_total, R)}")
        if micro_rows <= 0:
            raise ValueError("micro_rows must be positive")
        self.params, self.temperature = params, float(temperature)
        self.n_total, self.R, self.mb = int(n_total), int(R), int(micro_rows)
        self.n_micro = -(-self.n_total // self.mb)
        nbytes = _ffi.query("skyrl_policy_train_step_workspace_bytes", self.n_total, self.R, self.mb)
        self.ws = WORKSPACES.get(dev, "policy_train_step", nbytes)
        key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
        layout = (self.n_total, self.R, self.mb)
        if _STEP_LAYOUT.get(key) != layout:  # regions moved: no stale exchange granules in the new places
            self.ws.zero_()
            _STEP_LAYOUT[key] = layout
        self.loss = torch.empty(self.n_micro, dtype=torch.float32, device=dev)
        self.metrics = torch.empty((self.n_micro, _ffi.M_COUNT), dtype=torch.float32, device=dev)
        self.logp = torch.zeros((self.n_total, self.R), dtype=torch.float32, device=dev)
        self.entropy = torch.zeros((self.n_total, self.R), dtype=torch.float32, device=dev)
        if grpo is None:
            _ffi.call("skyrl_policy_train_plan", _ptr(self.mask), self.n_total, self.R, self.mb, ctypes.byref(params),
                      _ptr(self.ws), _stream(dev))
        else:
            scores = _f32c(grpo["scores"].detach(), "scores").view(-1)
            rmask = grpo["response_mask"].detach().contiguous()
            if scores.numel() != self.n_total or tuple(rmask.shape) != (self.n_total, self.R):
                raise ValueError("grpo: scores [n_total] and response_mask [n_total, R] expected")
            if rmask.dtype not in _MASK_DTYPES:
                raise TypeError(f"grpo: response_mask dtype {rmask.dtype} unsupported")
            rsum = grpo.get("loss_mask_row_sum")  # pack's: the plan then reads no loss mask
            if rsum is not None:
                rsum = _f32c(rsum.detach(), "loss_mask_row_sum").view(-1)
                if rsum.numel() != self.n_total:
                    raise ValueError("grpo: loss_mask_row_sum [n_total] expected")
            _ffi.call("skyrl_policy_train_plan_grpo", _ptr(self.mask), self.n_total, self.R, self.mb,
                      ctypes.byref(params), _ptr(scores), _ptr(rmask), _MASK_DTYPES[rmask.dtype],
                      int(grpo["group_size"]), float(grpo.get("epsilon", 1e-6)), int(bool(grpo.get("norm_by_std", True))),
                      _ptr(self.adv), _ptr(rsum), _ptr(self.ws), _stream(dev))

    def rows(self, k: int) -> Tuple[int, int]:
        return k * self.mb, min(self.n_total, (k + 1) * self.mb)

    def micro(self, k: int, logits, labels, token_pos=None):
        """Micro-batch k's fused pass. Dense: logits [rows, R, V] (unit vocab stride, rows of
        one [rows*R, V] matrix) and labels [rows, R]; packed: logits [ntok, V], labels [ntok]
        and token_pos [ntok] (positions within the micro-batch's [rows, R]). Returns the
        micro-batch's loss (0-d, differentiable w.r.t. logits; its value is written by fold())."""
        return _PolicyTrainMicroFunction.apply(logits, labels, token_pos, self, int(k))

    def fold(self) -> Tuple[torch.Tensor, torch.Tensor]:
        _ffi.call("skyrl_policy_train_fold", _ptr(self.mask), self.n_total, self.R, self.mb,
                  ctypes.byref(self.params), _ptr(self.loss), _ptr(self.metrics), _ptr(self.ws), _stream(self.dev))
        return self.loss, self.metrics


class _PolicyTrainMicroFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, token_pos, step, k):
        dev = _require_gpu(logits, labels, token_pos)
        if not 0 <= k < step.n_micro:
            raise IndexError(f"micro-batch {k} of {step.n_micro}")
        r0, r1 = step.rows(k)
        lg = logits.detach()
        if lg.dtype != torch.bfloat16 or lg.stride(-1) != 1:
            raise TypeError("policy pass: logits must be bf16 with unit vocab stride")
        V = lg.shape[-1]
        if token_pos is None:  # dense [rows, R, V]: rows of one [rows*R, V] matrix
            if lg.dim() != 3 or tuple(lg.shape[:2]) != (r1 - r0, step.R) or lg.stride(0) != step.R * lg.stride(1):
                raise ValueError(f"dense logits must be [{r1 - r0}, {step.R}, V] rows of one matrix")
            ntok, ld = (r1 - r0) * step.R, lg.stride(1)
            lab = labels.detach().to(device=dev, dtype=torch.int64)
            if tuple(lab.shape) != (r1 - r0, step.R):
                raise ValueError("labels must be [rows, R]")
            lsb, lst, pos = lab.stride(0), lab.stride(1), None
        else:
            if lg.dim() != 2:
                raise ValueError("packed logits must be [ntok, V]")
            ntok, ld = lg.shape[0], lg.stride(0)
            lab = labels.detach().to(device=dev, dtype=torch.int64).contiguous().view(-1)
            pos = token_pos.detach().to(device=dev, dtype=torch.int32).contiguous().view(-1)
            if lab.numel() != ntok or pos.numel() != ntok:
                raise ValueError(f"labels / token_pos need {ntok} entries, got {lab.numel()} / {pos.numel()}")
            lsb, lst = 0, 1
        dx = torch.empty(lg.shape, dtype=torch.bfloat16, device=dev)
        ld_grad = dx.stride(-2)
        _ffi.call("skyrl_policy_train_micro_fwd", _ptr(lg), BF16, ld, ntok, V, _ptr(lab), lsb, lst, _ptr(pos), k,
                  step.n_total, step.R, step.mb, step.temperature, _ptr(step.old), _ptr(step.adv), _ptr(step.mask),
                  _ptr(step.ref), ctypes.byref(step.params), _ptr(step.logp), _ptr(step.entropy), _ptr(dx), ld_grad,
                  _ptr(step.ws), _stream(dev))
        ctx.save_for_backward(dx)
        return step.loss[k]

    @staticmethod
    def backward(ctx, g_loss):
        (dx,) = ctx.saved_tensors
        g = g_loss.detach().to(torch.float32).reshape(1).contiguous()
        _ffi.call("skyrl_scale_bf16_by_device_scalar", _ptr(g), _ptr(dx), dx.numel(), _stream(dx.device))
        return dx, None, None, None, None


# ---------------------------------------------------------------------------- a1 sampler
def sample(
    logits: torch.Tensor,
    *,
    temperature: float = 1.0,
    top_k: int = -1,
    top_p: float = 1.0,
    min_p: float = 0.0,
    seed: int = 0,
    seq_ids: Optional[torch.Tensor] = None,
    step: int = 0,
    want_logprobs: bool = True,
    tokens_out: Optional[torch.Tensor] = None,
    logp_out: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """One decode step over logits [nseq, V] -> (tokens int32 [nseq], logprob f32 [nseq])."""
    dev = _require_gpu(logits, seq_ids)
    if logits.dim() != 2 or logits.stride(1) != 1:
        raise ValueError("logits must be [nseq, V] with unit vocab stride")
    dt = BF16 if logits.dtype == torch.bfloat16 else (F32 if logits.dtype == torch.float32 else None)
    if dt is None:
        raise TypeError(f"logits must be bf16 or f32, got {logits.dtype}")
    nseq, V = logits.shape
    ids = None if seq_ids is None else seq_ids.to(device=dev, dtype=torch.int64).contiguous()
    tokens = tokens_out if tokens_out is not None else torch.empty(nseq, dtype=torch.int32, device=dev)
    if tokens.dtype != torch.int32 or tokens.numel() != nseq or not tokens.is_contiguous():
        raise ValueError("tokens_out must be a contiguous int32 tensor of nseq elements")
    logp = logp_out if logp_out is not None else (
        torch.empty(nseq, dtype=torch.float32, device=dev) if want_logprobs else None)
    if logp is not None and (logp.dtype != torch.float32 or logp.numel() != nseq or not logp.is_contiguous()):
        raise ValueError("logp_out must be a contiguous float32 tensor of nseq elements")
    ws = WORKSPACES.get(dev, "sample", _ffi.query("skyrl_sample_workspace_bytes", nseq, V))
    _ffi.call(
        "skyrl_sample", _ptr(logits), dt, logits.stride(0), nseq, V, float(temperature), int(top_k), float(top_p),
        float(min_p),
        ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), _ptr(ids), int(step), _ptr(tokens), _ptr(logp), _ptr(ws),
        _stream(dev),
    )
    return tokens, logp


# ------------------------------------------------- §8(f)1 decode: lm_head GEMM + fused sampler
def _lmhead_operands(hidden: torch.Tensor, weight: torch.Tensor):
    dev = _require_gpu(hidden, weight)
    if hidden.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
        raise TypeError("lm_head operands must be bf16")
    if hidden.dim() != 2 or weight.dim() != 2 or hidden.shape[1] != weight.shape[1]:
        raise ValueError(f"hidden [M,K] and weight [V,K] expected, got {tuple(hidden.shape)} and {tuple(weight.shape)}")
    if hidden.stride(1) != 1 or weight.stride(1) != 1:
        raise ValueError("lm_head operands need a unit K stride")
    return dev


def lmhead_gemm(hidden: torch.Tensor, weight: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 logits [M,V] = hidden [M,K] @ weight[V,K]^T on the MFMA kernel of the fused sampler."""
    dev = _lmhead_operands(hidden, weight)
    M, K = hidden.shape
    V = weight.shape[0]
    z = out if out is not None else torch.empty((M, V), dtype=torch.bfloat16, device=dev)
    _ffi.call("skyrl_lmhead_gemm", _ptr(hidden), hidden.stride(0), _ptr(weight), weight.stride(0), M, V, K, _ptr(z),
              z.stride(0), _stream(dev))
    return z


def lmhead_sample(
    hidden: torch.Tensor,
    weight: torch.Tensor,
    *,
    temperature: float = 1.0,
    seed: int = 0,
    seq_ids: Optional[torch.Tensor] = None,
    step: int = 0,
    want_logprobs: bool = True,
    tokens_out: Optional[torch.Tensor] = None,
    logp_out: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """sample(hidden @ weight^T, temperature, seed, seq_ids, step) without materializing the logits:
    the same tokens as ops.sample on ops.lmhead_gemm's logits (no top_k / top_p / min_p)."""
    dev = _lmhead_operands(hidden, weight)
    M, K = hidden.shape
    V = weight.shape[0]
    ids = None if seq_ids is None else seq_ids.to(device=dev, dtype=torch.int64).contiguous()
    tokens = tokens_out if tokens_out is not None else torch.empty(M, dtype=torch.int32, device=dev)
    logp = logp_out if logp_out is not None else (
        torch.empty(M, dtype=torch.float32, device=dev) if want_logprobs else None)
    ws = WORKSPACES.get(dev, "lmhead_sample", _ffi.query("skyrl_lmhead_sample_workspace_bytes", M, V))
    _ffi.call("skyrl_lmhead_sample", _ptr(hidden), hidden.stride(0), _ptr(weight), weight.stride(0), M, V, K,
              float(temperature), ctypes.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), _ptr(ids), int(step),
              _ptr(tokens), _ptr(logp), _ptr(ws), _stream(dev))
    return tokens, logp


def lmhead_logprob_fwd(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor, temperature: float = 1.0,
                       compute_entropy: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """No-grad log_softmax(hidden @ weight^T / T)[labels] (+ entropy) for hidden [T, K], labels [T]
    (int64, any stride), through the MFMA GEMM's online-softmax epilogue: no [T, V] logits."""
    dev = _lmhead_operands(hidden, weight)
    T, K = hidden.shape
    V = weight.shape[0]
    lab = labels.to(device=dev, dtype=torch.int64)
    if lab.dim() != 1 or lab.numel() != T:
        raise ValueError("labels must be [T]")
    logp = torch.empty(T, dtype=torch.float32, device=dev)
    ent = torch.empty(T, dtype=torch.float32, device=dev) if compute_entropy else None
    ws = WORKSPACES.get(dev, "lmhead_logprob", _ffi.query("skyrl_lmhead_logprob_workspace_bytes", T, V))
    _ffi.call("skyrl_lmhead_logprob_fwd", _ptr(hidden), hidden.stride(0), _ptr(weight), weight.stride(0), T, V, K,
              _ptr(lab), lab.stride(0), float(temperature), _ptr(logp), _ptr(ent), None, _ptr(ws), _stream(dev))
    return logp, ent


# ---------------------------------------------------------------------------- a9 pack
def pack_experience(
    prompt_tokens: torch.Tensor, prompt_off: torch.Tensor,
    response_tokens: torch.Tensor, response_off: torch.Tensor,
    reward_vals: torch.Tensor, reward_off: torch.Tensor,
    loss_mask_vals: torch.Tensor, loss_mask_off: torch.Tensor,
    logprob_vals: Optional[torch.Tensor], logprob_off: Optional[torch.Tensor],
    *, N: int, P: int, R: int, pad: int = 0, pad_token_id: int = 0, return_row_sums: bool = False,
):
    """Device CSR inputs -> (sequences, attention_mask, response_mask, rewards, loss_mask, rollout_logprobs)
    [+ loss_mask_row_sum, reward_row_sum f32 [N+pad] when ``return_row_sums``: the loss's
    reduction scales and the GRPO scores, see grpo_advantage(scores=) / ppo_loss]."""
    dev = _require_gpu(prompt_tokens, response_tokens, reward_vals, loss_mask_vals)

    def i64(t):
        return t.to(device=dev, dtype=torch.int64).contiguous()

    def f32(t):
        return t.to(device=dev, dtype=torch.float32).contiguous()

    keep = [i64(prompt_tokens), i64(prompt_off), i64(response_tokens), i64(response_off), f32(reward_vals),
            i64(reward_off), f32(loss_mask_vals), i64(loss_mask_off)]
    has_lp = logprob_vals is not None
    if has_lp:
        keep += [f32(logprob_vals), i64(logprob_off)]
    ins = _ffi.PackInputs(*[t.data_ptr() for t in keep], *([None, None] if not has_lp else []))
    Np = N + pad
    S = P + R
    seq = torch.empty((Np, S), dtype=torch.int64, device=dev)
    att = torch.empty((Np, S), dtype=torch.int64, device=dev)
    rmask = torch.empty((Np, R), dtype=torch.int64, device=dev)
    rew = torch.empty((Np, R), dtype=torch.float32, device=dev)
    lmask = torch.empty((Np, R), dtype=torch.float32, device=dev)
    rlp = torch.empty((Np, R), dtype=torch.float32, device=dev) if has_lp else None
    rows = torch.empty(Np, dtype=torch.float32, device=dev) if return_row_sums else None
    wrows = torch.empty(Np, dtype=torch.float32, device=dev) if return_row_sums else None
    _ffi.call(
        "skyrl_pack_experience", ctypes.byref(ins), N, pad, P, R, int(pad_token_id), _ptr(seq), _ptr(att),
        _ptr(rmask), _ptr(rew), _ptr(lmask), _ptr(rlp), _ptr(rows), _ptr(wrows), _stream(dev),
    )
    if return_row_sums:
        return seq, att, rmask, rew, lmask, rlp, rows, wrows
    return seq, att, rmask, rew, lmask, rlp


# ---------------------------------------------------------------------------- a12 helpers
def scale_and_sumsq(flat_grad: torch.Tensor, scale: float, sumsq: torch.Tensor) -> None:
    dev = _require_gpu(flat_grad, sumsq)
    if flat_grad.dtype != torch.float32 or not flat_grad.is_contiguous():
        raise TypeError("flat_grad must be a contiguous float32 bucket")
    _ffi.call("skyrl_scale_and_sumsq", _ptr(flat_grad), flat_grad.numel(), float(scale), _ptr(sumsq), _stream(dev))
