"""Typed config for the hot path: the same keys and defaults as the reference.

Mirrors skyrl_train/config/config.py:219-335 (AlgorithmConfig and its nested configs,
SamplingParams) and config/ppo_base_config.yaml:92-189,316-324, so a reference
`trainer.algorithm.*` / `generator.sampling_params.*` dict builds the same object.
"""

from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


class _FromDict:
    @classmethod
    def from_dict(cls, d: Optional[Dict[str, Any]]):
        """Build recursively from a plain dict; unknown keys raise (reference: build_nested_dataclass)."""
        if d is None:
            return cls()
        if isinstance(d, cls):
            return d
        kwargs = {}
        names = {f.name: f for f in dataclasses.fields(cls)}
        for k, v in dict(d).items():
            if k not in names:
                raise ValueError(f"{cls.__name__}: unknown key {k!r}")
            sub = _NESTED.get((cls.__name__, k))
            kwargs[k] = sub.from_dict(v) if (sub is not None and isinstance(v, dict)) else v
        return cls(**kwargs)


@dataclass
class KLCtrlConfig(_FromDict):
    type: str = "fixed"
    kl_target: float = 0.1
    horizon: int = 10000


@dataclass
class SAPOConfig(_FromDict):
    tau_pos: float = 1.0
    tau_neg: float = 1.05


@dataclass
class DynamicSamplingConfig(_FromDict):
    type: Optional[str] = None
    max_sample_batches: int = 30
    min_replace_ratio: float = 0.3


@dataclass
class ClipCovConfig(_FromDict):
    clip_ratio: float = 0.0002
    clip_cov_lb: float = 1.0
    clip_cov_ub: float = 5.0


@dataclass
class KLCovConfig(_FromDict):
    kl_cov_frac: float = 0.2
    ppo_kl_coef: float = 1.0


@dataclass
class CISPOConfig(_FromDict):
    cispo_eps_clip_low: float = 0.0
    cispo_eps_clip_high: float = 5.0


@dataclass
class OffPolicyCorrectionConfig(_FromDict):
    tis_ratio_type: Optional[str] = None
    token_tis_ratio_clip_high: float = 2.0
    sequence_tis_ratio_clip_high: float = 5.0
    sequence_mask_metric: Optional[str] = None
    geo_mask_high: float = 1.01
    geo_mask_low: float = 0.99
    product_mask_high: float = 2.0
    product_mask_low: float = 0.5
    outlier_token_is_threshold_low: Optional[float] = None
    outlier_token_is_threshold_high: Optional[float] = None


@dataclass
class AlgorithmConfig(_FromDict):
    advantage_estimator: str = "grpo"
    kl_ctrl: KLCtrlConfig = field(default_factory=KLCtrlConfig)
    kl_estimator_type: str = "k3"
    use_kl_in_reward: bool = False
    use_kl_loss: bool = True
    kl_loss_coef: float = 0.001
    use_entropy_loss: bool = False
    entropy_loss_coef: float = 0.01
    advantage_batch_normalize: bool = False
    value_head_prefix: str = "value_head"
    policy_loss_type: str = "regular"
    loss_reduction: str = "token_mean"
    grpo_norm_by_std: bool = True
    zero_variance_filter: bool = False
    lambd: float = 1.0
    gamma: float = 1.0
    eps_clip_low: float = 0.2
    eps_clip_high: float = 0.2
    clip_ratio_c: float = 3.0
    tis_imp_ratio_cap: float = -1.0
    use_tis: bool = False
    off_policy_correction: OffPolicyCorrectionConfig = field(default_factory=OffPolicyCorrectionConfig)
    sapo: SAPOConfig = field(default_factory=SAPOConfig)
    value_clip: Optional[float] = 0.2
    dynamic_sampling: DynamicSamplingConfig = field(default_factory=DynamicSamplingConfig)
    clip_cov: ClipCovConfig = field(default_factory=ClipCovConfig)
    kl_cov: KLCovConfig = field(default_factory=KLCovConfig)
    cispo: CISPOConfig = field(default_factory=CISPOConfig)
    max_seq_len: Optional[int] = None


@dataclass
class SamplingParams(_FromDict):
    """generator.sampling_params (ppo_base_config.yaml:316-324)."""

    max_generate_length: int = 1024
    repetition_penalty: float = 1.0
    temperature: float = 1.0
    top_p: float = 1.0
    min_p: float = 0.0
    top_k: int = -1
    logprobs: Optional[int] = 0
    stop: Optional[List[str]] = None
    additional_kwargs: Optional[Dict[str, Any]] = None


_NESTED = {
    ("AlgorithmConfig", "kl_ctrl"): KLCtrlConfig,
    ("AlgorithmConfig", "off_policy_correction"): OffPolicyCorrectionConfig,
    ("AlgorithmConfig", "sapo"): SAPOConfig,
    ("AlgorithmConfig", "dynamic_sampling"): DynamicSamplingConfig,
    ("AlgorithmConfig", "clip_cov"): ClipCovConfig,
    ("AlgorithmConfig", "kl_cov"): KLCovConfig,
    ("AlgorithmConfig", "cispo"): CISPOConfig,
}
