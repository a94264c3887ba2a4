"""Algorithm plugin surface of skyrl_train.utils.ppo_utils, driven by the HIP hot path.

Same public names, signatures, registry semantics and error messages as
skyrl_train/utils/ppo_utils.py (reference snapshot 2026-02-27), so reference plugins
(`@register_advantage_estimator`, `@register_policy_loss`) and call sites work unchanged:

  hot path (HIP, skyrl_amd.ops):  compute_grpo_outcome_advantage   (ppo_utils.py:1132)
                                  compute_gae_advantage_return     (:1101)
                                  compute_approx_kl                (:88)
                                  ppo_policy_loss regular/dual_clip (:548)
                                  ppo_critic_loss                  (:175)
  secondary registry entries:     skyrl_amd.secondary (torch restatements, same names)

Registries are process-local (the reference syncs them through a named Ray actor when
Ray is initialised, :197-302; this build has no Ray: one process per GPU, plugins are
registered at import time in every rank).
"""

from __future__ import annotations

import enum
from functools import wraps
from typing import Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from . import ops
from .config import AlgorithmConfig
from .torch_utils import masked_mean, safe_exp_delta

try:  # Python >= 3.11
    from enum import StrEnum
except ImportError:  # Python 3.10: same behaviour as the stdlib class for our use
    class StrEnum(str, enum.Enum):
        def __str__(self) -> str:
            return str(self.value)


# ----------------------------------------------------------------------------- KL controllers
class AdaptiveKLController:
    """ppo_utils.py:45-61 (Ziegler et al. 2019 proportional controller)."""

    def __init__(self, init_kl_coef, target, horizon):
        self.value = init_kl_coef
        self.target = target
        self.horizon = horizon

    def update(self, current, n_steps):
        err = float(np.clip(current / self.target - 1, -0.2, 0.2))
        self.value *= 1 + err * n_steps / self.horizon


class FixedKLController:
    def __init__(self, kl_coef):
        self.value = kl_coef

    def update(self, current, n_steps):
        pass


def get_kl_controller(algorithm_cfg):
    kind = algorithm_cfg.kl_ctrl.type
    if kind == "fixed":
        return FixedKLController(kl_coef=algorithm_cfg.kl_loss_coef)
    if kind == "adaptive":
        if algorithm_cfg.kl_ctrl.horizon <= 0:
            raise ValueError(f"horizon must be larger than 0. Got {algorithm_cfg.kl_ctrl.horizon}")
        return AdaptiveKLController(algorithm_cfg.kl_loss_coef, algorithm_cfg.kl_ctrl.kl_target,
                                    algorithm_cfg.kl_ctrl.horizon)
    raise ValueError(f"Invalid KL controller type: {kind}")


# ----------------------------------------------------------------------------- registries
class BaseFunctionRegistry:
    """Name -> callable registry (ppo_utils.py:221-392 semantics, process-local)."""

    _function_type = "Function"

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        cls._functions: Dict[str, Callable] = {}

    @staticmethod
    def _key(name) -> str:
        return name.value if isinstance(name, enum.Enum) else name

    @classmethod
    def register(cls, name, func: Callable):
        key = cls._key(name)
        if key in cls._functions:
            raise ValueError(f"{cls._function_type} '{key}' already registered")
        cls._functions[key] = func

    @classmethod
    def get(cls, name) -> Callable:
        key = cls._key(name)
        if key not in cls._functions:
            raise ValueError(
                f"Unknown {cls._function_type.lower()} '{key}'. Available: {list(cls._functions.keys())}"
            )
        return cls._functions[key]

    @classmethod
    def list_available(cls) -> List[str]:
        return list(cls._functions.keys())

    @classmethod
    def unregister(cls, name):
        key = cls._key(name)
        if key not in cls._functions:
            raise ValueError(f"{cls._function_type} '{key}' not registered")
        del cls._functions[key]

    @classmethod
    def reset(cls):
        cls._functions.clear()

    @classmethod
    def sync_with_actor(cls):
        raise Exception("Ray is not initialized, cannot sync with actor")


class AdvantageEstimator(StrEnum):
    GAE = "gae"
    GRPO = "grpo"
    RLOO = "rloo"
    REINFORCE_PP = "reinforce++"


class PolicyLossType(StrEnum):
    REGULAR = "regular"
    DUAL_CLIP = "dual_clip"
    GSPO = "gspo"
    CISPO = "cispo"
    CLIP_COV = "clip_cov"
    KL_COV = "kl_cov"
    SAPO = "sapo"
    CROSS_ENTROPY = "cross_entropy"
    IMPORTANCE_SAMPLING = "importance_sampling"


class AdvantageEstimatorRegistry(BaseFunctionRegistry):
    _function_type = "advantage estimator"

    @classmethod
    def repopulate_registry(cls):
        have = set(cls.list_available())
        for name, fn in _DEFAULT_ESTIMATORS().items():
            if name not in have:
                cls.register(name, fn)


class PolicyLossRegistry(BaseFunctionRegistry):
    _function_type = "policy loss"

    @classmethod
    def repopulate_registry(cls):
        have = set(cls.list_available())
        for name, fn in _DEFAULT_LOSSES().items():
            if name not in have:
                cls.register(name, fn)


def register_advantage_estimator(name):
    def deco(func):
        @wraps(func)
        def wrapper(*args, **kwargs):
            return func(*args, **kwargs)

        AdvantageEstimatorRegistry.register(name, wrapper)
        return wrapper

    return deco


def register_policy_loss(name):
    def deco(func):
        @wraps(func)
        def wrapper(*args, **kwargs):
            return func(*args, **kwargs)

        PolicyLossRegistry.register(name, wrapper)
        return wrapper

    return deco


def sync_registries():
    raise ValueError("Ray is not initialized, cannot sync registries")


def repopulate_all_registries():
    PolicyLossRegistry.repopulate_registry()
    AdvantageEstimatorRegistry.repopulate_registry()


# ----------------------------------------------------------------------------- a6 KL
@torch.no_grad()
def compute_approx_kl(log_probs, log_probs_base, loss_mask=None, kl_estimator_type: str = "k3"):
    """HIP elementwise estimator (ppo_utils.py:88-124); no gradient, as in the reference."""
    return ops.approx_kl(log_probs, log_probs_base, loss_mask, kl_estimator_type)


# ----------------------------------------------------------------------------- whitening helpers
def masked_var(values, mask, unbiased=True):
    mean = masked_mean(values, mask)
    var = masked_mean((values - mean) ** 2, mask)
    if unbiased:
        msum = mask.sum()
        if msum == 0:
            raise ValueError("At least one element in the mask has to be 1.")
        if msum == 1:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
        var = var * (msum / (msum - 1))
    return var


def masked_whiten(values, mask, shift_mean=True):
    mean, var = masked_mean(values, mask), masked_var(values, mask)
    out = (values - mean) * torch.rsqrt(var + 1e-8)
    if not shift_mean:
        out += mean
    return out


@torch.no_grad()
def normalize_advantages_dict(data, group=None):
    """ppo_utils.py:127-145 (advantage_batch_normalize) on the HIP kernels (ops.normalize_advantages):
    the unmasked mean, the masked squared deviations; a new advantages tensor (returns keep the
    old one, as in the reference). `group`: the data-parallel group whose ranks hold the rows of
    one global batch (the sums are all-reduced once)."""
    data["advantages"] = ops.normalize_advantages(data["advantages"], data["response_mask"], group=group)
    return data


# ----------------------------------------------------------------------------- a8 critic
def ppo_critic_loss(values, old_values, returns, config, loss_mask=None) -> Tuple[torch.Tensor, Optional[float]]:
    """HIP clipped value loss (ppo_utils.py:175-193); returns (loss, clipfrac or None)."""
    vc = config.value_clip
    loss, clipfrac = ops.CriticLossFunction.apply(values, old_values, returns, loss_mask, vc)
    return loss, (clipfrac.item() if vc is not None else None)


# ----------------------------------------------------------------------------- a7 PG loss
def _off_policy_enabled(config) -> bool:
    opc = getattr(config, "off_policy_correction", None)
    return opc is not None and (opc.tis_ratio_type is not None or opc.sequence_mask_metric is not None)


def ppo_params_from_config(config, *, use_kl_loss=False, use_entropy_loss=False, has_entropy=False):
    return ops.make_ppo_params(
        eps_clip_low=config.eps_clip_low, eps_clip_high=config.eps_clip_high, clip_ratio_c=config.clip_ratio_c,
        policy_loss_type=config.policy_loss_type, loss_reduction=config.loss_reduction,
        max_seq_len=config.max_seq_len, use_kl_loss=use_kl_loss, kl_estimator_type=config.kl_estimator_type,
        kl_loss_coef=config.kl_loss_coef, use_entropy_loss=use_entropy_loss,
        entropy_loss_coef=config.entropy_loss_coef, has_entropy=has_entropy,
    )


def ppo_policy_loss(log_probs, old_log_probs, advantages, config, loss_mask=None, rollout_logprobs=None):
    """regular / dual_clip PPO loss on the HIP path (ppo_utils.py:548-586).

    With off-policy correction enabled (off_policy_correction_utils.py:262-296) the TIS ratio
    w > 0 (detached) folds into the advantages -- -min(r A w, clip(r) A w) = w * -min(r A, clip(r) A),
    and dual_clip's branch on sign(A) is unchanged -- and the corrected mask drives the
    reduction, so the same HIP kernels run; clip_ratio keeps the uncorrected mask, as in the
    reference (it is computed before the correction).
    """
    assert config.policy_loss_type in ["regular", "dual_clip"], "loss_type must be either 'regular' or 'dual_clip'"
    params = ppo_params_from_config(config)
    if rollout_logprobs is not None and _off_policy_enabled(config):
        from .secondary import off_policy_terms

        tis, extra, pg_mask = off_policy_terms(old_log_probs, rollout_logprobs, loss_mask,
                                               config.off_policy_correction)
        adv = advantages * tis if tis is not None else advantages
        loss, _ = ops.ppo_loss(log_probs, old_log_probs, adv, pg_mask, params)
        with torch.no_grad():
            ratio = safe_exp_delta(log_probs.detach() - old_log_probs, clip=20.0, out_dtype=log_probs.dtype)
            clipped = ratio.clamp(1 - config.eps_clip_low, 1 + config.eps_clip_high)
            clip = masked_mean((-(clipped * advantages) > -(ratio * advantages)).float(), loss_mask).mean().item()
        return loss, {"clip_ratio": clip, **extra}
    loss, metrics = ops.ppo_loss(log_probs, old_log_probs, advantages, loss_mask, params)
    return loss, {"clip_ratio": metrics[4].item()}


def reduce_loss(loss, loss_mask, loss_reduction, max_seq_len=None):
    """ppo_utils.py:984-1009 (torch; used by the secondary losses)."""
    if loss_reduction == "token_mean":
        return masked_mean(loss, loss_mask)
    if loss_reduction == "sequence_mean":
        return masked_mean(loss, loss_mask, dim=-1).mean()
    if loss_reduction == "seq_mean_token_sum_norm":
        assert max_seq_len is not None, "max_seq_len must be provided for seq_mean_token_sum_norm loss reduction"
        tot = (loss * loss_mask).sum(-1) if loss_mask is not None else loss.sum(-1)
        return (tot / max_seq_len).mean()
    raise ValueError(f"Invalid loss reduction type: {loss_reduction}")


# ----------------------------------------------------------------------------- a4 / a5 estimators
def compute_grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon: float = 1e-6,
                                   grpo_norm_by_std: bool = True, scores=None, **kwargs):
    """HIP GRPO advantage (ppo_utils.py:1132-1182). Returns (advantages, returns) aliased.
    ``scores`` (f32 [N], the pack kernel's per-row reward sums, in the kernel's own summation
    order) skips the reward reads."""
    off, rows, ng = ops.groups_from_index(index)
    R = token_level_rewards.shape[-1]
    if R % 4 == 0 and ops.contiguous_group_size(off, rows, ng):
        off = rows = None  # contiguous equal groups: the index-free kernel
    adv = ops.grpo_advantage(token_level_rewards, response_mask, off, rows, ng, epsilon, grpo_norm_by_std,
                             scores=scores)
    return adv, adv


def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma: float, lambd: float, **kwargs):
    """HIP GAE + masked whitening (ppo_utils.py:1101-1129)."""
    return ops.gae_advantage_return(token_level_rewards, values, response_mask, gamma, lambd)


def compute_advantages_and_returns(token_level_rewards, response_mask, index, adv_estimator, config, values=None,
                                   grpo_norm_by_std: bool = True, gamma=1.0, lambd=1.0, **kwargs):
    fn = AdvantageEstimatorRegistry.get(adv_estimator)
    return fn(token_level_rewards=token_level_rewards, response_mask=response_mask, index=index, values=values,
              grpo_norm_by_std=grpo_norm_by_std, gamma=gamma, lambd=lambd, config=config, **kwargs)


def _DEFAULT_ESTIMATORS():
    from . import secondary

    return {
        "grpo": compute_grpo_outcome_advantage,
        "gae": compute_gae_advantage_return,
        "rloo": secondary.compute_rloo_outcome_advantage,
        "reinforce++": secondary.compute_reinforce_plus_plus_outcome_advantage,
    }


def _DEFAULT_LOSSES():
    from . import secondary

    return {
        "regular": ppo_policy_loss,
        "dual_clip": ppo_policy_loss,
        "gspo": secondary.gspo_policy_loss,
        "clip_cov": secondary.compute_policy_loss_clip_cov,
        "kl_cov": secondary.compute_policy_loss_kl_cov,
        "sapo": secondary.sapo_policy_loss,
        "cross_entropy": secondary.cross_entropy_loss,
        "importance_sampling": secondary.importance_sampling_loss,
        "cispo": secondary.compute_policy_loss_cispo,
    }


repopulate_all_registries()
