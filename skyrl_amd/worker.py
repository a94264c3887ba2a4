"""Policy/critic worker micro-batch step on the HIP path (a2/a3/a6/a7/a8 + a13 + a12 hooks).

Mirror of PolicyWorkerBase._forward_backward_micro (skyrl-train/skyrl_train/workers/
worker.py:731-900), CriticWorkerBase._forward_backward_micro (:1062-1114) and optim_step
(:900-925). The transformer forward/backward stays PyTorch (north_star): the step takes the
model's logits ``[n, S, V]`` (bf16, requires grad) and returns the same status dict as the
reference, with the loss already back-propagated into the logits.

For regular / dual_clip PPO without off-policy correction (the reference defaults) the whole
loss -- logprob + entropy over V, PPO clip, KL(ref) term, entropy term, reduction, and the
logits gradient -- is ONE fused kernel per micro-batch (skyrl_policy_train_fwd): the logits
are read from HBM once and the gradient written once, and the metrics come back in one
8-float device vector (one host read per micro-batch, as the reference's .item() calls).
Every other registered loss runs as logprob kernel -> registry loss -> KL/entropy terms,
exactly the reference's composition.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from . import ops
from .comm import all_reduce_metrics
from .ppo_utils import PolicyLossRegistry, _off_policy_enabled, compute_approx_kl, ppo_params_from_config
from .torch_utils import masked_mean


class PolicyMicroStep:
    """Loss + backward of one policy micro-batch given the model's logits."""

    def __init__(self, algorithm_cfg, temperature: float = 1.0, group=None, lr_fn=None):
        self.cfg = algorithm_cfg
        self.temperature = float(temperature)
        self.group = group
        self.lr_fn = lr_fn or (lambda: 0.0)
        self.micro_batches_accumulated = 0

    def _fused_ok(self, loss_name: str) -> bool:
        return loss_name in ("regular", "dual_clip") and not _off_policy_enabled(self.cfg)

    def __call__(self, logits: torch.Tensor, experience, loss_fn: Optional[str] = None,
                 backward: bool = True) -> Dict[str, Any]:
        cfg = self.cfg
        R = int(experience.num_actions)
        x = logits[:, -R - 1:-1]                 # response positions (model_wrapper.py:370), a view
        labels = experience.sequences[:, -R:]    # roll(sequences, -1)[:, -R-1:-1]
        mask = experience.loss_mask
        name = loss_fn if loss_fn is not None else cfg.policy_loss_type
        if self._fused_ok(name):
            params = ppo_params_from_config(cfg, use_kl_loss=cfg.use_kl_loss, use_entropy_loss=cfg.use_entropy_loss,
                                            has_entropy=True)
            if name != cfg.policy_loss_type:
                params.dual_clip = int(name == "dual_clip")
            loss, metrics, _, _ = ops.policy_train(x, labels, experience.action_log_probs, experience.advantages,
                                                   mask, params, experience.base_action_log_probs if
                                                   cfg.use_kl_loss else None, self.temperature)
            if backward:
                loss.backward()
            m = metrics.tolist()
            ops.check_loss_metrics(torch.tensor(m))  # the split rows' exchange never timed out
            status = {"final_loss": m[ops._ffi.M_FINAL_LOSS], "policy_loss": m[ops._ffi.M_POLICY_LOSS],
                      "policy_entropy": m[ops._ffi.M_ENTROPY], "response_length": R, "policy_lr": self.lr_fn(),
                      "loss_metrics/clip_ratio": m[ops._ffi.M_CLIP_RATIO]}
            if cfg.use_kl_loss:
                status["policy_kl"] = m[ops._ffi.M_KL]
        else:
            lp, ent = ops.logprobs_and_entropy(x, labels, self.temperature, compute_entropy=True)
            policy_loss, loss_metrics = PolicyLossRegistry.get(name)(
                lp, experience.action_log_probs, experience.advantages, config=cfg, loss_mask=mask,
                rollout_logprobs=experience.rollout_logprobs)
            if name == "cross_entropy":
                if backward:
                    policy_loss.backward()
                return all_reduce_metrics({"loss": policy_loss.item(), "response_length": R,
                                           "lr": self.lr_fn()}, self.group)
            with torch.set_grad_enabled(cfg.use_entropy_loss):
                entropy = masked_mean(ent if cfg.use_entropy_loss else ent.detach(), mask)
            ent_term = entropy * cfg.entropy_loss_coef if cfg.use_entropy_loss else torch.zeros((), device=lp.device)
            if cfg.use_kl_loss:
                kl = compute_approx_kl(lp, experience.base_action_log_probs, loss_mask=mask,
                                       kl_estimator_type=cfg.kl_estimator_type)
                kl_loss = masked_mean(kl, mask, dim=-1).mean()
            else:
                kl_loss = torch.zeros((), device=lp.device)
            loss = policy_loss + kl_loss * cfg.kl_loss_coef - ent_term
            if backward:
                loss.backward()
            status = {"final_loss": loss.item(), "policy_loss": policy_loss.item(),
                      "policy_entropy": entropy.item(), "response_length": R, "policy_lr": self.lr_fn()}
            for k, v in loss_metrics.items():
                status["loss_metrics/" + k] = v
            if cfg.use_kl_loss:
                status["policy_kl"] = kl_loss.item()
        self.micro_batches_accumulated += 1
        return all_reduce_metrics(status, self.group)


class CriticMicroStep:
    """CriticWorkerBase._forward_backward_micro (worker.py:1062-1114) given the value head output."""

    def __init__(self, algorithm_cfg, group=None, lr_fn=None):
        self.cfg = algorithm_cfg
        self.group = group
        self.lr_fn = lr_fn or (lambda: 0.0)

    def __call__(self, values: torch.Tensor, experience, backward: bool = True) -> Dict[str, Any]:
        from .ppo_utils import ppo_critic_loss

        loss, clipfrac = ppo_critic_loss(values, experience.values, experience.returns, self.cfg,
                                         loss_mask=experience.loss_mask)
        if backward:
            loss.backward()
        status = {"critic_loss": loss.item(), "values_mean": masked_mean(values.detach(), experience.loss_mask).item(),
                  "values_clipfrac": clipfrac, "critic_lr": self.lr_fn()}
        return all_reduce_metrics({k: v for k, v in status.items() if v is not None}, self.group)
