"""Ray-free GRPO/PPO driver: one training step = rollout on the MI355X engine -> experience pack
-> ref/old logprobs -> advantages -> clipped policy-gradient update -> weight sync back into
the engine.

Follows the step of RayPPOTrainer.train (skyrl_train/trainer.py:236-352): generate
(`generate`, :427-470), postprocess_generator_output + convert_to_training_input (:592-757),
fwd_logprobs_values_reward (:1037-1066), compute_advantages_and_returns (:759-862),
train_critic_and_policy -> _execute_training_step (:1067-1120) with the mini-/micro-batch
structure of PolicyWorkerBase (workers/worker.py:664-925), then the weight sync
(broadcast_to_inference_engines, fsdp_worker.py:201-228). Ray actors, FSDP sharding and
the dispatch layer collapse into this process: the learner is a HF transformers model under
torch.autocast(bf16) (the north star keeps the transformer in PyTorch), and everything on the
§8 path runs through the HIP kernels — the engine's sampler and decode loop, the pack kernel,
GRPO, the lm_head-fused logprob/entropy and the fused PPO/KL loss.
"""

from __future__ import annotations

import asyncio
import math
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch

from . import comm, ppo_utils, trainer_utils
from .config import AlgorithmConfig
from .lmhead import lmhead_logprobs_and_entropy
from .packing import enable_sample_packing, packed_hidden_states


@dataclass
class TrainerConfig:
    n_samples_per_prompt: int = 8
    policy_mini_batch_size: int = 256          # prompts per optimizer step (ppo_base_config.yaml)
    micro_train_batch_size_per_gpu: int = 1    # sequences per forward/backward
    micro_forward_batch_size_per_gpu: int = 1  # sequences per no-grad forward
    update_epochs_per_batch: int = 1
    lr: float = 1e-6
    critic_lr: float = 5e-6                     # trainer.critic.optimizer_config.lr
    betas: Sequence[float] = (0.9, 0.999)
    weight_decay: float = 0.01
    max_grad_norm: float = 1.0
    temperature: float = 1.0
    use_sample_packing: bool = True             # trainer.use_sample_packing (config.py:457): padding-free learner
    # "hip": comm.ShardedModuleOptimizer (flat fp32 master, reduce-scatter from the backward hooks,
    # one HIP clip + AdamW pass that also writes the engine's bf16 weights); "torch": torch.optim.AdamW
    # + clip_grad_norm_ + bucketed all-reduce (the A/B reference)
    optimizer: str = "hip"
    # policy micro-batches through ONE fused memory pass over the lm_head logits (logprob +
    # entropy + PPO/KL loss + dlogits, ops.policy_train_ragged) between the lm_head GEMM and its
    # backward GEMMs, instead of the chunked lm_head logprob + loss + chunk recompute (falls back
    # for V % 8 != 0 or V > 155,648, and for loss types other than regular / dual_clip)
    fused_policy_pass: bool = True
    sampling_params: Dict[str, Any] = field(default_factory=lambda: {"max_tokens": 1024, "min_tokens": 1})
    algorithm: AlgorithmConfig = field(default_factory=AlgorithmConfig)


def _positions(attention_mask: torch.Tensor) -> torch.Tensor:
    """model_wrapper.py:272-273: left-padded position ids."""
    pos = attention_mask.long().cumsum(-1) - 1
    return pos.masked_fill_(attention_mask == 0, 1)


class CriticModel(torch.nn.Module):
    """get_llm_for_sequence_regression's critic (model_wrapper.py:402-500): the HF base model plus
    `value_head = Linear(H, 1, bias=False)`; values of the last R action positions, i.e. the
    hidden states at [-R-1:-1] like the action log-probs."""

    def __init__(self, hf_config, value_head_prefix: str = "value_head"):
        super().__init__()
        from transformers import AutoModel

        self.model = AutoModel.from_config(hf_config)
        self.value_head_prefix = value_head_prefix
        setattr(self, value_head_prefix, torch.nn.Linear(hf_config.hidden_size, 1, bias=False))

    def forward(self, seq: torch.Tensor, att: torch.Tensor, R: int, packed: bool = False) -> torch.Tensor:
        if packed:  # padding-free (skyrl_amd.packing); the model must be switched by enable_sample_packing
            h = packed_hidden_states(self.model, seq, att, R)
            return getattr(self, self.value_head_prefix)(h).squeeze(-1)
        h = self.model(input_ids=seq, attention_mask=att, position_ids=_positions(att)).last_hidden_state
        return getattr(self, self.value_head_prefix)(h).squeeze(-1)[:, :-1][:, -R:]


class GRPOTrainer:
    """policy: HF CausalLM (fp32 master weights) on the GPU; ref: frozen HF CausalLM (or None when
    the KL loss is off); client: an InferenceEngineClient (or one engine) whose weights mirror the
    policy; reward_fn(prompt_ids, response_ids, extra) -> float. With `critic` (a CriticModel) the
    step is PPO with a value function: values in the no-grad pass, advantages by the configured
    estimator (GAE on the HIP kernel for advantage_estimator="gae"), critic update before the
    policy update."""

    def __init__(self, cfg: TrainerConfig, policy, client, reward_fn: Optional[Callable[..., float]], pad_token_id: int,
                 ref=None, generator=None, env_class: Optional[str] = None, dp_group=None, critic=None):
        self.critic = critic
        self.critic_optimizer = torch.optim.AdamW(critic.parameters(), lr=cfg.critic_lr, betas=tuple(cfg.betas),
                                                  weight_decay=cfg.weight_decay, eps=1e-8) if critic else None
        """With `generator` (a SkyRLGymGenerator over the same client) `step` takes chat prompts and
        env extras and runs the multi-turn agent loop: rewards and loss masks come from it.
        Under data parallelism (one process per GPU, `dp_group` initialised) every rank steps on
        its own prompts with its own colocated engine; gradients are mean-reduced in buckets
        whose all-reduces are launched from the last micro-batch's backward as each bucket
        completes (comm.BucketedGradAllReduce, overlapped with the rest of the backward), and
        metrics are all-reduced."""
        self.dp_group = dp_group
        self.generator = generator
        self.env_class = env_class
        self.cfg = cfg
        self.policy = policy
        self.ref = ref
        self.client = client
        self.reward_fn = reward_fn
        self.pad_token_id = pad_token_id
        alg = cfg.algorithm
        if alg.use_kl_loss and ref is None:
            raise ValueError("use_kl_loss needs a reference model")
        self.loss_params = ppo_utils.ppo_params_from_config(
            alg, use_kl_loss=alg.use_kl_loss, use_entropy_loss=alg.use_entropy_loss, has_entropy=True)
        if cfg.use_sample_packing:
            for m in (policy, ref, critic.model if critic is not None else None):
                if m is not None:
                    enable_sample_packing(m)
        world = torch.distributed.get_world_size(dp_group) if (
            torch.distributed.is_available() and torch.distributed.is_initialized()) else 1
        if cfg.optimizer not in ("hip", "torch"):
            raise ValueError(f"optimizer must be 'hip' or 'torch', got {cfg.optimizer!r}")
        self.optimizer = self.grad_sync = self.optim = None
        if cfg.optimizer == "hip":  # optim_step / FSDP2 (worker.py:902-924, fsdp_strategy.py:155-191)
            self.optim = comm.ShardedModuleOptimizer(
                policy, comm.AdamWConfig(lr=cfg.lr, betas=tuple(cfg.betas), eps=1e-8, weight_decay=cfg.weight_decay,
                                         max_grad_norm=cfg.max_grad_norm), group=dp_group)
        else:
            self.optimizer = torch.optim.AdamW(policy.parameters(), lr=cfg.lr, betas=tuple(cfg.betas),
                                               weight_decay=cfg.weight_decay, eps=1e-8)
            self.grad_sync = comm.BucketedGradAllReduce(policy.parameters(), dp_group) if world > 1 else None
        self.critic_grad_sync = (comm.BucketedGradAllReduce(critic.parameters(), dp_group)
                                 if world > 1 and critic is not None else None)
        self.global_step = 0
        self.timings: Dict[str, float] = {}  # seconds per phase of the last step (device-synchronised)
        self._t = 0.0

    def _mark(self, phase: str) -> None:
        torch.cuda.synchronize()
        now = time.perf_counter()
        self.timings[phase] = now - self._t
        self._t = now

    # ---------------------------------------------------------------- rollout
    async def _generate(self, prompts: List[List[int]]) -> Dict[str, Any]:
        G = self.cfg.n_samples_per_prompt
        ids = [p for p in prompts for _ in range(G)]
        sp = dict(self.cfg.sampling_params)
        sp.setdefault("logprobs", 0)
        sp.setdefault("temperature", self.cfg.temperature)
        out = await self.client.generate({"prompt_token_ids": ids, "sampling_params": sp})
        return {"prompt_token_ids": ids, "response_ids": out["response_ids"], "stop_reasons": out["stop_reasons"],
                "rollout_logprobs": out["response_logprobs"],
                "loss_masks": [[1] * len(r) for r in out["response_ids"]]}

    # ---------------------------------------------------------------- model passes
    def _wait_weights(self, model) -> None:
        """The policy's parameters are views of the HIP optimizer's master, which the previous
        optimizer step re-assembles on the comm stream (world > 1, left in flight): a pass that
        reads them -- base_model and the lm_head weight, not through the module's own forward --
        makes the current stream wait for that all-gather first (no host sync)."""
        if self.optim is not None and model is self.policy:
            self.optim.wait_weights()

    def _logprobs(self, model, seq, att, R, grad: bool):
        """action log-probs (and entropy) of the last R positions: HFModelWrapper.forward
        (model_wrapper.py:261-375) with the lm_head-fused HIP logprob/entropy."""
        self._wait_weights(model)
        with torch.autocast("cuda", dtype=torch.bfloat16), torch.set_grad_enabled(grad):
            base = model.base_model  # model.model (Qwen2/Llama), model.transformer (GPT-2)
            if self.cfg.use_sample_packing:
                h = packed_hidden_states(base, seq, att, R).to(torch.bfloat16)
            else:
                hidden = base(input_ids=seq, attention_mask=att, position_ids=_positions(att)).last_hidden_state
                h = hidden[:, -R - 1:-1].to(torch.bfloat16)
            w = model.get_output_embeddings().weight.to(torch.bfloat16)
            labels = seq[:, -R:]
            live = att[:, -R:].bool()  # positions whose label is a real response token
            if bool(live.all()):
                return lmhead_logprobs_and_entropy(h, w, labels, temperature=self.cfg.temperature,
                                                   compute_entropy=grad)
            # the lm_head GEMMs only over live rows (padding is about half of [n, R] at U[1, R]
            # responses); padded positions read 0, as the reference's pad_input leaves them
            lp_v, ent_v = lmhead_logprobs_and_entropy(h[live], w, labels[live], temperature=self.cfg.temperature,
                                                      compute_entropy=grad)
            zeros = torch.zeros(live.shape, dtype=torch.float32, device=h.device)
            return (zeros.masked_scatter(live, lp_v),
                    zeros.masked_scatter(live, ent_v) if ent_v is not None else None)

    @torch.no_grad()
    def _fwd_logprobs(self, model, data) -> torch.Tensor:
        model.eval()  # forward passes run without dropout (worker.py:982); training in train mode (:750)
        seq, att = data["sequences"], data["attention_mask"]
        R = data["response_mask"].shape[1]
        mb = self.cfg.micro_forward_batch_size_per_gpu
        # one autocast region over all micro-batches: each fp32 weight is cast to bf16 once per
        # pass (autocast's cast cache lives until the outermost region exits), not once per
        # micro-batch
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return torch.cat([self._logprobs(model, seq[i:i + mb], att[i:i + mb], R, grad=False)[0]
                              for i in range(0, len(seq), mb)])

    @torch.no_grad()
    def _fwd_values(self, data) -> torch.Tensor:
        self.critic.eval()  # worker.py:1172-1179
        seq, att = data["sequences"], data["attention_mask"]
        R = data["response_mask"].shape[1]
        mb = self.cfg.micro_forward_batch_size_per_gpu
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return torch.cat([self.critic(seq[i:i + mb], att[i:i + mb], R, self.cfg.use_sample_packing).float()
                              for i in range(0, len(seq), mb)])

    # ---------------------------------------------------------------- step
    def step(self, prompts: List[List[int]], extras: Optional[List[Any]] = None) -> Dict[str, float]:
        cfg, alg = self.cfg, self.cfg.algorithm
        G = cfg.n_samples_per_prompt
        self.timings = {}
        torch.cuda.synchronize()
        self._t = time.perf_counter()
        ext = extras or [None] * len(prompts)
        if self.generator is not None:  # multi-turn agent loop: per-token rewards + observation masks
            from .generators import TrajectoryID
            from .generators.skyrl_gym_generator import get_vllm_sampling_params

            gen = asyncio.run(self.generator.generate({
                "sampling_params": get_vllm_sampling_params(self.generator.cfg.sampling_params),
                "prompts": [p for p in prompts for _ in range(G)],
                "env_classes": [self.env_class] * (G * len(prompts)),
                "env_extras": [dict(e or {}) for e in ext for _ in range(G)],
                "trajectory_ids": [TrajectoryID(f"{self.global_step}_{i}", j) for i in range(len(prompts))
                                   for j in range(G)]}))
        else:
            gen = asyncio.run(self._generate(prompts))
        self._mark("generate")
        if self.generator is None:
            gen["rewards"] = [float(self.reward_fn(p, r, ext[i // G]))
                              for i, (p, r) in enumerate(zip(gen["prompt_token_ids"], gen["response_ids"]))]
        metrics = self.train_on(gen)
        self._sync_weights()
        self._mark("weight_sync")
        return metrics

    def train_on(self, gen: Dict[str, Any]) -> Dict[str, float]:
        """Everything after generation for one batch of groups (G consecutive trajectories per
        prompt, rewards filled in): pack, old/ref logprobs (+ values), advantages, critic and
        policy updates. Advances global_step; the caller syncs the engine's weights."""
        cfg, alg = self.cfg, self.cfg.algorithm
        G = cfg.n_samples_per_prompt
        step_wise = gen.get("is_last_step") is not None
        if step_wise:  # one sample per turn: a step's group is its trajectory's prompt
            uids = [t.instance_id for t in gen["trajectory_ids"]]
        else:
            uids = [str(i // G) for i in range(len(gen["response_ids"]))]
        gen, metrics = trainer_utils.postprocess_generator_output(gen, uids, G, step_wise=step_wise)
        data = trainer_utils.convert_to_training_input(gen, uids, self.pad_token_id, dp_size=1,
                                                       device=next(self.policy.parameters()).device,
                                                       step_wise=step_wise)
        self._mark("reward_and_pack")
        # fwd_logprobs_values_reward: old (policy) and ref log-probs, no grad
        data["action_log_probs"] = self._fwd_logprobs(self.policy, data)
        if self.ref is not None:
            data["base_action_log_probs"] = self._fwd_logprobs(self.ref, data)
        if self.critic is not None:
            data["values"] = self._fwd_values(data)
        self._mark("fwd_logprobs")
        # GRPO inside the policy step's plan launch (skyrl_policy_train_plan_grpo) when the built-in
        # estimator would run on contiguous groups with pack's reward row sums: the same advantages
        # (bit for bit), no launch of their own; the estimator's metrics follow the update
        plan_grpo = self._plan_grpo_ok(data, step_wise)
        if plan_grpo:
            data["advantages"] = torch.empty_like(data["rewards"])
            data["returns"] = data["advantages"]  # compute_grpo_outcome_advantage returns (adv, adv)
        else:
            data = trainer_utils.compute_advantages_and_returns(data, alg)
            if alg.advantage_batch_normalize:  # trainer.py:275-276 / fully_async_trainer.py:514-515
                data = ppo_utils.normalize_advantages_dict(data, group=self._dp_group_if_dist())
        self._mark("advantages")
        metrics.update(data.metadata.get("metrics", {}))
        m = data["loss_mask"]
        rl = data["rollout_logprobs"]
        if rl is not None:  # rollout (engine) vs learner log-probs of the same tokens
            metrics["logprobs_diff_mean"] = float(((rl - data["action_log_probs"]).abs() * m).sum() / m.sum().clamp(min=1))
        if self.critic is not None:  # train_critic_and_policy: the critic steps first (trainer.py:1085-1120)
            metrics.update(self._train_critic(data))
        metrics.update(self._train_policy(data, plan_grpo=plan_grpo))
        if plan_grpo:
            trainer_utils.advantage_metrics(data)
            metrics.update(data.metadata["metrics"])
        self._mark("train")
        self.global_step += 1
        return metrics

    def _train_critic(self, data) -> Dict[str, float]:
        """CriticWorkerBase._forward_backward_micro (worker.py:1062-1114) + optim_step: HIP clipped
        value loss against the GAE returns, loss / n_micro, clip, AdamW."""
        self.critic.train()  # worker.py:1074
        cfg = self.cfg
        n = len(data["sequences"])
        mini = cfg.policy_mini_batch_size * cfg.n_samples_per_prompt
        mb = cfg.micro_train_batch_size_per_gpu
        R = data["response_mask"].shape[1]
        acc: Dict[str, List[float]] = {}
        for s0, s1 in trainer_utils.mini_batch_slices(n, mini):
            n_micro = math.ceil((s1 - s0) / mb)
            for i in range(s0, s1, mb):
                j = min(i + mb, s1)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    v = self.critic(data["sequences"][i:j], data["attention_mask"][i:j], R,
                                    self.cfg.use_sample_packing).float()
                loss, clipfrac = ppo_utils.ppo_critic_loss(v, data["values"][i:j], data["returns"][i:j],
                                                           cfg.algorithm, loss_mask=data["loss_mask"][i:j])
                if self.critic_grad_sync is not None and j == s1:
                    self.critic_grad_sync.arm()
                (loss / n_micro).backward()
                acc.setdefault("critic_loss", []).append(float(loss.detach()))
                if clipfrac is not None:
                    acc.setdefault("values_clipfrac", []).append(clipfrac)
            if self.critic_grad_sync is not None:
                self.critic_grad_sync.wait()
            gn = torch.nn.utils.clip_grad_norm_(self.critic.parameters(), cfg.max_grad_norm)
            self.critic_optimizer.step()
            if self.critic_grad_sync is not None:
                self.critic_grad_sync.zero_grad()
            else:
                self.critic_optimizer.zero_grad(set_to_none=True)
            acc.setdefault("critic_grad_norm", []).append(float(gn))
        return comm.all_reduce_metrics(trainer_utils.reduce_metrics(acc), group=self.dp_group,
                                       device=next(self.critic.parameters()).device)

    def _dp_group_if_dist(self):
        """The data-parallel group when torch.distributed is up (the ranks' rows form one batch)."""
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            return self.dp_group if self.dp_group is not None else torch.distributed.group.WORLD
        return None

    def _plan_grpo_ok(self, data, step_wise: bool) -> bool:
        """GRPO can run inside the policy step's plan launch: the built-in GRPO estimator (not a
        plugin registered under its name), no critic, no advantage_batch_normalize (whose batch
        statistics need every advantage before the first micro-batch), the fused policy pass,
        pack's reward row sums (absent once a reward KL penalty changed the rewards), contiguous
        groups of G rows that the mini-batches do not cut (no DP pad rows), and every row inside a
        trained mini-batch (the reference estimates the dropped tail rows too)."""
        alg, G = self.cfg.algorithm, self.cfg.n_samples_per_prompt
        n = len(data["rewards"])
        return (not step_wise and self.critic is None and alg.advantage_estimator == "grpo"
                and not alg.advantage_batch_normalize
                and ppo_utils.AdvantageEstimatorRegistry.get("grpo") is ppo_utils.compute_grpo_outcome_advantage
                and data.get("reward_row_sum") is not None and data.metadata.get("pad_size", 0) == 0
                and 1 <= G <= 64 and n % (self.cfg.policy_mini_batch_size * G) == 0 and self._fused_pass_ok())

    def _train_policy(self, data, plan_grpo: bool = False) -> Dict[str, float]:
        """_execute_training_step: mini-batches of policy_mini_batch_size prompts (no shuffle,
        trainer.py:1067-1081), micro-batches inside, loss scaled by 1/n_micro, grad clip, AdamW.
        With the fused pass every mini-batch is one ops.PolicyTrainStep: one plan launch (the
        loss scales of all its micro-batches), the micro-batches' fused passes, one fold launch
        (every micro-batch's loss and metrics), read once and checked before the optimizer
        step, so a failed exchange never reaches the weights."""
        from . import ops

        self.policy.train()  # worker.py:750
        cfg = self.cfg
        n = len(data["sequences"])
        mini = cfg.policy_mini_batch_size * cfg.n_samples_per_prompt
        mb = cfg.micro_train_batch_size_per_gpu
        R = data["response_mask"].shape[1]
        fused = self._fused_pass_ok()
        acc: Dict[str, List[float]] = {}
        for epoch in range(cfg.update_epochs_per_batch):
            for s0, s1 in trainer_utils.mini_batch_slices(n, mini):
                n_micro = math.ceil((s1 - s0) / mb)
                step = None
                if fused:
                    grpo = None
                    if plan_grpo and epoch == 0:  # this mini-batch's advantages, in the plan launch
                        grpo = dict(scores=data["reward_row_sum"][s0:s1], response_mask=data["response_mask"][s0:s1],
                                    group_size=cfg.n_samples_per_prompt, epsilon=1e-6,
                                    norm_by_std=cfg.algorithm.grpo_norm_by_std,
                                    loss_mask_row_sum=(data["loss_mask_row_sum"][s0:s1]
                                                       if data.get("loss_mask_row_sum") is not None else None))
                    step = ops.PolicyTrainStep(
                        data["action_log_probs"][s0:s1], data["advantages"][s0:s1], data["loss_mask"][s0:s1],
                        self.loss_params, mb,
                        ref_log_probs=data["base_action_log_probs"][s0:s1] if self.ref is not None else None,
                        temperature=cfg.temperature, grpo=grpo)
                mets = []
                for k, i in enumerate(range(s0, s1, mb)):
                    j = min(i + mb, s1)
                    if step is not None:
                        loss = self._fused_policy_pass(step, k, data, i, j, R)
                    else:
                        ref = data["base_action_log_probs"][i:j] if self.ref is not None else None
                        lp, ent = self._logprobs(self.policy, data["sequences"][i:j], data["attention_mask"][i:j],
                                                 R, grad=True)
                        loss, met = self._loss(lp, data, i, j, ref, ent)
                        mets.append(met)
                    if self.optim is not None:
                        if j == s1:
                            self.optim.arm()  # the last micro-batch: buckets reduce-scatter during its backward
                        if loss is not None:
                            loss.backward()  # 1/n_micro is applied by the optimizer step (worker.py:909-914)
                    else:
                        if self.grad_sync is not None and j == s1:
                            self.grad_sync.arm()  # the last micro-batch: buckets all-reduce during its backward
                        if loss is not None:
                            (loss / n_micro).backward()
                allm = (step.fold()[1] if step is not None else torch.stack(mets)).cpu()  # one host read
                ops.check_loss_metrics(allm)  # before the optimizer step: nothing NaN reaches the weights
                if self.optim is not None:
                    grad_norm = self.optim.step(n_micro)
                else:
                    if self.grad_sync is not None:
                        self.grad_sync.wait()
                    grad_norm = torch.nn.utils.clip_grad_norm_(self.policy.parameters(), cfg.max_grad_norm)
                    self.optimizer.step()
                    if self.grad_sync is not None:
                        self.grad_sync.zero_grad()
                    else:
                        self.optimizer.zero_grad(set_to_none=True)
                grad_norm = float(grad_norm)
                mt = allm.mean(0).tolist()
                for k, v in (("final_loss", mt[0]), ("policy_loss", mt[1]), ("policy_entropy", mt[2]),
                             ("policy_kl", mt[3]), ("ppo_clip_ratio", mt[4]), ("grad_norm", grad_norm)):
                    acc.setdefault(k, []).append(v)
        return comm.all_reduce_metrics(trainer_utils.reduce_metrics(acc), group=self.dp_group,
                                       device=next(self.policy.parameters()).device)

    def _fused_pass_ok(self) -> bool:
        """The fused pass takes regular / dual_clip PPO at the vocabularies the split kernel is
        built for (asked of the library: the same plan the launch makes)."""
        from . import _ffi

        if not self.cfg.fused_policy_pass or self.cfg.algorithm.policy_loss_type not in ("regular", "dual_clip"):
            return False
        V = self.policy.get_output_embeddings().weight.shape[0]
        return bool(_ffi.query("skyrl_policy_train_supports", V, int(V % 8 == 0), float(self.cfg.temperature)))

    def _fused_policy_pass(self, step, k, data, i, j, R):
        """Micro-batch k's policy forward + loss with the lm_head logits feeding one fused pass:
        hidden states of the live response tokens (packed), z = h W^T (bf16, the reference's
        lm_head under autocast, model_wrapper.py:308-363), then the step's fused pass computes
        logprob, entropy, the PPO/KL/entropy loss terms (worker.py:801-876) and dL/dz in one read
        of z; autograd's lm_head backward takes dL/dz into the dh / dW GEMMs. Same loss, metrics
        and gradients as _logprobs + _loss (tests/test_gpu_trainer_e2e.py). A micro-batch with no
        response token (not reachable from valid generator output: every response has a token, the
        generator output check rejects empty reward lists as the reference's does) would contribute
        a zero loss through the same forward (the fold counts it as 0), so its backward still
        reaches every parameter and the per-bucket reduce-scatters fire from the backward hooks in
        the same order on every rank."""
        seq, att = data["sequences"][i:j], data["attention_mask"][i:j]
        live = att[:, -R:].bool()
        pos = torch.nonzero(live.reshape(-1)).reshape(-1).to(torch.int32)
        model = self.policy
        self._wait_weights(model)
        if pos.numel() == 0:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                hidden = model.base_model(input_ids=seq, attention_mask=att,
                                          position_ids=_positions(att)).last_hidden_state
                w = model.get_output_embeddings().weight
            # one element of each, native dtype (no fp32 copy of the [V, H] weight, no overflow to
            # inf * 0): the slice's backward still reaches every parameter with a dense zero
            # gradient, so every grad hook fires
            return (hidden[..., :1].sum() + w.view(-1)[:1].sum()).float() * 0.0
        with torch.autocast("cuda", dtype=torch.bfloat16):
            base = model.base_model
            if self.cfg.use_sample_packing:
                h = packed_hidden_states(base, seq, att, R).to(torch.bfloat16)
            else:
                hidden = base(input_ids=seq, attention_mask=att, position_ids=_positions(att)).last_hidden_state
                h = hidden[:, -R - 1:-1].to(torch.bfloat16)
            w = model.get_output_embeddings().weight.to(torch.bfloat16)
            z = torch.matmul(h[live], w.t())  # [live tokens, V] bf16
        return step.micro(k, z, seq[:, -R:][live], pos)

    def _loss(self, lp, data, i, j, ref, ent):
        """The micro-batch's policy loss (worker.py:801-876) on the fused HIP loss over the
        advantages compute_advantages_and_returns wrote (GRPO runs once per step), with the pack
        kernel's loss-mask row sums and the fold deferred to the backward launch (loss and
        metrics are read after backward, as the reference does)."""
        from . import ops

        rows = data.get("loss_mask_row_sum")
        rows = rows[i:j] if rows is not None else None
        return ops.ppo_loss(lp, data["action_log_probs"][i:j], data["advantages"][i:j], data["loss_mask"][i:j],
                            self.loss_params, ref_log_probs=ref, entropy=ent, loss_mask_row_sum=rows,
                            defer_fold=True)

    @torch.no_grad()
    def weight_update_request(self) -> Dict[str, Any]:
        """broadcast_to_inference_engines: the bf16 weights of every parameter under its HF name.
        With the HIP optimizer these are views of the bf16 copy its update pass (world 1) or its
        bf16 all-gather (world > 1) wrote: no per-parameter cast."""
        if self.optim is not None:
            named = self.optim.named_bf16()
            return {"names": [n for n, _ in named], "tensors": [t for _, t in named]}
        names, tensors = [], []
        for name, p in self.policy.named_parameters():
            names.append(name)
            tensors.append(p.detach().to(torch.bfloat16))
        return {"names": names, "tensors": tensors}

    def _sync_weights(self):
        asyncio.run(self.client.update_named_weights(self.weight_update_request()))
