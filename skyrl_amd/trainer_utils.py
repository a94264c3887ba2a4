"""Trainer-side host surface around the hot path: a4/a6 trainer wrappers, a9 experience
conversion, a10 data order and batching.

Each function mirrors the reference function named in its docstring (same arguments,
outputs, metric keys and error behaviour). The arithmetic runs in the HIP kernels
(skyrl_amd.ops); the Python here is list flattening, index math and metric plumbing.

References (skyrl-train/skyrl_train/):
  postprocess_generator_output       trainer.py:680-757
  get_metrics_from_generator_output  generators/utils.py:170-218
  zero_variance_filter               utils/trainer_utils.py:568-590
  validate_generator_output          utils/trainer_utils.py:593-640
  convert_prompts_responses_...      dataset/preprocess.py:28-132
  convert_to_training_input          trainer.py:592-666
  pad_batch                          trainer.py:872-907
  compute_advantages_and_returns     trainer.py:759-862
  apply_reward_kl_penalty            trainer.py:981-1035
  _remove_tail_data                  trainer.py:353-375
  build_dataloader (order)           utils/trainer_utils.py:661-699 (torch DataLoader, seeded
                                     generator, shuffle=True, drop_last=True)
  mini-batch / DP slicing            trainer.py:1040-1081, distributed/dispatch.py:122-205
  reduce_metrics / BatchIterator     workers/worker_utils.py:8-90
"""

from __future__ import annotations

import copy
import itertools
import math
from collections import defaultdict
from dataclasses import dataclass
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from .training_batch import TrainingInputBatch


# ------------------------------------------------------------------------------ rewards / metrics
def get_metrics_from_generator_output(generator_output: Dict[str, Any], uids: List[str]) -> Dict[str, float]:
    """generators/utils.py:170-218: avg_score, pass_at_n, mean_positive_reward."""
    rewards = generator_output["rewards"]
    if not len(rewards):
        raise ValueError(f"`rewards` must be a non-empty list, got {rewards}")
    per_uid = defaultdict(list)
    if isinstance(rewards[0], list):
        mean_raw = float(np.mean([sum(r) for r in rewards]))
        mean_pos = float(np.mean([sum(max(x, 0) for x in r) for r in rewards]))
        for i, r in enumerate(rewards):
            if len(r) == 0:
                raise ValueError("Token-level rewards must be a non-empty list.")
            per_uid[uids[i]].append(r[-1])
    else:
        mean_raw = float(np.mean(rewards))
        mean_pos = float(np.mean(np.maximum(rewards, 0.0)))
        for i, r in enumerate(rewards):
            per_uid[uids[i]].append(r)
    pass_at_n = sum(1 for v in per_uid.values() if any(r > 0 for r in v)) / len(per_uid)
    return {"avg_score": mean_raw, "pass_at_n": pass_at_n, "mean_positive_reward": mean_pos}


def zero_variance_filter(rewards: List[float], uids: List[str]) -> List[int]:
    """utils/trainer_utils.py:568-590: indices whose uid group has non-zero reward std (or is a singleton)."""
    groups = defaultdict(list)
    for uid, r in zip(uids, rewards):
        groups[uid].append(r)
    kept = {u for u, v in groups.items() if np.std(v) > 0 or len(v) == 1}
    return [i for i, u in enumerate(uids) if u in kept]


def validate_generator_output(num_prompts: int, generator_output: Dict[str, Any]) -> None:
    """utils/trainer_utils.py:593-640."""
    if len(generator_output["response_ids"]) <= 0:
        raise RuntimeError("No outputs generated")
    n = len(generator_output["response_ids"])
    assert num_prompts == n, f"Mismatch between prompts ({num_prompts}) and responses ({n})"
    assert n == len(generator_output["prompt_token_ids"]), (
        f"Mismatch between responses ({n}) and prompt_token_ids ({len(generator_output['prompt_token_ids'])})")
    for key in ("response_ids", "loss_masks", "rewards", "rollout_logprobs"):
        v = generator_output.get(key)
        if isinstance(v, list):
            assert len(v) == n, f"Generator output {key} length must be equal to response_ids length, got {len(v)} and {n}"
    for i, (resp, lm, rew) in enumerate(zip(generator_output["response_ids"], generator_output["loss_masks"],
                                            generator_output["rewards"])):
        assert len(resp) == len(lm), (
            f"Response ids and loss masks must have the same length, for sample {i} got {len(resp)} and {len(lm)}")
        if isinstance(rew, list):
            assert len(rew) == len(resp), (
                f"Token rewards and response ids must have the same length, for sample {i} got {len(rew)} and {len(resp)}")


def _last_steps(generator_output: Dict[str, Any], uids: List[str]):
    """The last-step samples of step-wise output, for metrics (trainer.py:700-713)."""
    last = generator_output["is_last_step"]
    out = {k: [v[i] for i in range(len(v)) if last[i]] for k, v in generator_output.items() if isinstance(v, list)}
    return out, [u for u, ls in zip(uids, last) if ls]


def postprocess_generator_output(generator_output: Dict[str, Any], uids: List[str], n_samples_per_prompt: int,
                                 zero_variance_filter_enabled: bool = False, step_wise: bool = False
                                 ) -> Tuple[Dict[str, Any], Dict[str, float]]:
    """trainer.py:680-757: response-level rewards go on the last response token; returns
    (generator_output with per-token rewards, reward metrics). Step-wise output is measured on
    each trajectory's last step only."""
    if step_wise:
        m = get_metrics_from_generator_output(*_last_steps(generator_output, uids))
    else:
        m = get_metrics_from_generator_output(generator_output, uids)
    rewards = generator_output["rewards"]
    responses = generator_output["response_ids"]
    if rewards and isinstance(rewards[0], list):
        per_token = rewards
    else:
        if zero_variance_filter_enabled:
            keep = set(zero_variance_filter(rewards, uids))
            generator_output["loss_masks"] = [lm if i in keep else [0] * len(lm)
                                              for i, lm in enumerate(generator_output["loss_masks"])]
        per_token = []
        for r, resp in zip(rewards, responses):
            t = [0.0] * len(resp)
            t[-1] = float(r)
            per_token.append(t)
    generator_output["rewards"] = per_token
    metrics = {
        f"reward/avg_pass_at_{n_samples_per_prompt}": m["pass_at_n"],
        "reward/avg_raw_reward": m["avg_score"],
        "reward/mean_positive_reward": m["mean_positive_reward"],
    }
    return generator_output, metrics


# ------------------------------------------------------------------------------ a9 pack
def flatten_ragged(lists: Sequence[Sequence], dtype) -> Tuple[np.ndarray, np.ndarray]:
    """Ragged Python lists -> (values, int64 offsets[len+1]) CSR, one pass, no per-row arrays."""
    lens = np.fromiter((len(x) for x in lists), dtype=np.int64, count=len(lists))
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    vals = np.fromiter(itertools.chain.from_iterable(lists), dtype=dtype, count=int(off[-1]))
    return vals, off


def _pad_id(tokenizer_or_pad_id) -> int:
    if isinstance(tokenizer_or_pad_id, (int, np.integer)):
        return int(tokenizer_or_pad_id)
    return int(tokenizer_or_pad_id.pad_token_id)


def convert_prompts_responses_to_batch_tensors(tokenizer, prompts: List[List[int]], responses: List[List[int]],
                                               rewards: List[List[float]], loss_masks: List[List[int]],
                                               logprobs: Optional[List[List[float]]] = None, *, device=None,
                                               pad_rows: int = 0, return_row_sums: bool = False):
    """dataset/preprocess.py:28-132 on the HIP pack kernel. ``tokenizer`` may be the pad id.

    Returns (sequences int64[N,P+R], attention_mask int64, response_mask int64[N,R],
    rewards f32[N,R], loss_mask f32[N,R], rollout_logprobs f32[N,R] | None) on ``device``,
    with ``pad_rows`` extra rows appended as pad_batch does (fused into the same kernel);
    with ``return_row_sums`` also the per-row loss-mask and reward sums (f32 [N]: the fused
    loss's reduction scales and the GRPO scores) from the same kernel.
    """
    from . import ops

    if not (len(prompts) == len(responses) == len(rewards) == len(loss_masks)) or len(prompts) == 0:
        raise AssertionError("prompts, responses, rewards and loss_masks must be non-empty and equally long")
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    N = len(prompts)
    pv, po = flatten_ragged(prompts, np.int64)
    rv, ro = flatten_ragged(responses, np.int64)
    wv, wo = flatten_ragged([list(r) if not isinstance(r, torch.Tensor) else r.tolist() for r in rewards],
                            np.float32)
    mv, mo = flatten_ragged(loss_masks, np.float32)
    P = int(np.max(np.diff(po)))
    R = int(np.max(np.diff(ro)))
    has_lp = bool(logprobs)
    lv, lo = flatten_ragged(logprobs, np.float32) if has_lp else (None, None)

    def dev(a):
        return None if a is None else torch.from_numpy(a).pin_memory().to(device, non_blocking=True)

    return ops.pack_experience(dev(pv), dev(po), dev(rv), dev(ro), dev(wv), dev(wo), dev(mv), dev(mo), dev(lv),
                               dev(lo), N=N, P=P, R=R, pad=pad_rows, pad_token_id=_pad_id(tokenizer),
                               return_row_sums=return_row_sums)


def pad_size_for(batch_size: int, dp_size: int) -> int:
    return math.ceil(batch_size / dp_size) * dp_size - batch_size


def pad_batch(training_input: TrainingInputBatch, dp_size: int) -> TrainingInputBatch:
    """trainer.py:872-907: pad to a multiple of dp_size by cloning the first rows; loss_mask 0 and
    is_last_step 1 for pads; uids get "pad{i}"."""
    pad = pad_size_for(training_input.batch_size, dp_size)
    training_input.metadata["pad_size"] = pad
    if pad == 0:
        return training_input
    new = {}
    for key, t in training_input.items():
        if t is None:
            continue
        extra = tuple(t.shape[1:])
        if key == "is_last_step":
            p = torch.ones(pad, *extra, dtype=t.dtype, device=t.device)
        elif key in ("loss_mask", "loss_mask_row_sum"):  # the row sums follow the pads' zero loss mask
            p = torch.zeros(pad, *extra, dtype=t.dtype, device=t.device)
        else:
            p = t[:pad].clone()
        new[key] = torch.cat([t, p], dim=0)
    out = TrainingInputBatch(new)
    out.metadata = {"uids": training_input.metadata["uids"] + [f"pad{i}" for i in range(pad)]}
    if "trajectory_ids" in training_input.metadata:
        out.metadata["trajectory_ids"] = training_input.metadata["trajectory_ids"] + [f"pad{i}" for i in range(pad)]
    for k, v in training_input.metadata.items():
        if k not in ("uids", "trajectory_ids"):
            out.metadata[k] = copy.deepcopy(v)
    return out


def convert_to_training_input(generator_output: Dict[str, Any], uids: List[str], tokenizer, dp_size: int = 1,
                              device=None, off_policy_correction_enabled: bool = False,
                              step_wise: bool = False) -> TrainingInputBatch:
    """trainer.py:592-666 with pad_batch fused into the pack kernel. Step-wise output also
    carries is_last_step and the trajectory ids (metadata), and its average response length
    counts last steps only (trainer.py:645-660)."""
    resp = generator_output["response_ids"]
    N = len(resp)
    pad = pad_size_for(N, dp_size)
    logprobs = generator_output.get("rollout_logprobs", None)
    seq, att, rmask, rew, lmask, rlp, lm_rows, rw_rows = convert_prompts_responses_to_batch_tensors(
        tokenizer, generator_output["prompt_token_ids"], resp, generator_output["rewards"],
        generator_output["loss_masks"], logprobs, device=device, pad_rows=pad, return_row_sums=True)
    if off_policy_correction_enabled:
        assert rlp is not None, "expected non-null rollout logprobs tensor when off_policy_correction is enabled"
        assert rlp.shape == lmask.shape, "Logprobs should look like responses"
    fields = {"sequences": seq, "attention_mask": att, "response_mask": rmask, "rewards": rew, "loss_mask": lmask,
              "rollout_logprobs": rlp,
              # with the batch, from the pack kernel: the fused loss's reduction scales and the GRPO
              # scores (kept only while "rewards" is unchanged; apply_reward_kl_penalty drops it)
              "loss_mask_row_sum": lm_rows, "reward_row_sum": rw_rows}
    if generator_output.get("is_last_step", None) is not None:
        ils = torch.tensor(generator_output["is_last_step"], dtype=torch.bool)
        fields["is_last_step"] = torch.cat([ils, torch.ones(pad, dtype=torch.bool)]).to(seq.device)
    batch = TrainingInputBatch(fields)
    batch.metadata = {
        "uids": list(uids) + [f"pad{i}" for i in range(pad)],
        "response_length": rmask.shape[1],
        "avg_response_length": sum(len(r) for r in resp) / N,
        "pad_size": pad,
        # every loss mask no longer than its response: loss_mask is 0 outside response_mask
        "loss_mask_within_response": all(len(m) <= len(r) for m, r in zip(generator_output["loss_masks"], resp)),
    }
    if step_wise:
        assert generator_output.get("trajectory_ids") is not None, \
            "Expected `trajectory_ids` in generator output for step wise training"
        batch.metadata["trajectory_ids"] = [t.to_string() if hasattr(t, "to_string") else str(t)
                                            for t in generator_output["trajectory_ids"]] + \
            [f"pad{i}" for i in range(pad)]
        last = generator_output["is_last_step"]
        batch.metadata["avg_response_length"] = sum(len(r) for r, ls in zip(resp, last) if ls) / N
    return batch


# ------------------------------------------------------------------------------ a4 / a6 trainer wrappers
@torch.no_grad()
def compute_advantages_and_returns(data: TrainingInputBatch, algorithm_cfg) -> TrainingInputBatch:
    """trainer.py:759-862 (non step-wise): advantages/returns through the registry, plus the
    metrics avg_final_rewards / avg_response_length / avg_advantages / avg_advantages_abs.
    The metric reductions run on the device; one host read for all four."""
    from . import ppo_utils

    rewards = data["rewards"]
    kw = dict(adv_estimator=algorithm_cfg.advantage_estimator, config=algorithm_cfg, gamma=algorithm_cfg.gamma,
              lambd=algorithm_cfg.lambd, grpo_norm_by_std=algorithm_cfg.grpo_norm_by_std)
    values = data.get("values")
    step_wise = data.get("is_last_step") is not None and data.metadata.get("trajectory_ids") is not None
    if step_wise:
        # trainer.py:777-808: estimate on each trajectory's last step, then give every step of a
        # trajectory its last step's advantages/returns (steps of a trajectory are contiguous)
        last = data["is_last_step"].bool()
        idx = np.array(data.metadata["uids"])[last.cpu().numpy()]
        la, lr = ppo_utils.compute_advantages_and_returns(
            token_level_rewards=rewards[last], response_mask=data["response_mask"][last], index=list(idx),
            values=values[last] if values is not None else None, **kw)
        traj = torch.cat([torch.zeros(1, dtype=torch.int64, device=last.device), last[:-1].long()]).cumsum(0)
        assert int(traj[-1]) + 1 == len(la), (
            f"number of groups {int(traj[-1]) + 1} doesn't match the number of trajectories as given by "
            f"`is_last_step` {len(la)}. The `is_last_step` tensor is likely malformed")
        adv, ret = la[traj], lr[traj]
    else:
        if algorithm_cfg.advantage_estimator == "grpo" and data.get("reward_row_sum") is not None:
            kw["scores"] = data["reward_row_sum"]  # the pack kernel's row sums: no reward re-read
        adv, ret = ppo_utils.compute_advantages_and_returns(
            token_level_rewards=rewards, response_mask=data["response_mask"], index=data.metadata["uids"],
            values=values, **kw)
    data["returns"] = ret
    data["advantages"] = adv
    advantage_metrics(data, step_wise)
    return data


def advantage_metrics(data: TrainingInputBatch, step_wise: bool = False) -> None:
    """trainer.py:838-860's metrics of compute_advantages_and_returns: avg_final_rewards /
    avg_response_length / avg_advantages / avg_advantages_abs over the non-pad rows (device
    reductions, one host read)."""
    rewards, adv = data["rewards"], data["advantages"]
    pad = data.metadata.get("pad_size", 0)
    n = len(rewards) - pad
    m = data["response_mask"][:n].to(torch.float32)
    a = adv[:n]
    cnt = m.sum()
    rs = rewards.sum(-1)[:n]
    avg_reward = rs[data["is_last_step"][:n].bool()].mean() if step_wise else rs.mean()
    stats = torch.stack([avg_reward, (a * m).sum() / cnt, (a.abs() * m).sum() / cnt]).tolist()
    data.metadata.setdefault("metrics", {}).update({
        "avg_final_rewards": stats[0],
        "avg_response_length": data.metadata["avg_response_length"],
        "avg_advantages": stats[1],
        "avg_advantages_abs": stats[2],
    })


@torch.no_grad()
def apply_reward_kl_penalty(data: TrainingInputBatch, algorithm_cfg, reward_kl_controller=None) -> TrainingInputBatch:
    """trainer.py:981-1035 on the fused HIP kernel (kl, masked mean, abs-max, reward update in one pass)."""
    from . import ops

    coef = reward_kl_controller.value if reward_kl_controller is not None else algorithm_cfg.kl_loss_coef
    new_rewards, m = ops.reward_kl_penalty(data["rewards"], data["action_log_probs"], data["base_action_log_probs"],
                                           data["loss_mask"], algorithm_cfg.kl_estimator_type, max(0, coef))
    data["rewards"] = new_rewards
    if data.get("reward_row_sum") is not None:  # the pack's GRPO scores summed the old rewards
        del data["reward_row_sum"]
    avg_kl, avg_kl_max = m.tolist()
    if reward_kl_controller is not None:
        reward_kl_controller.update(current=avg_kl, n_steps=data["rewards"].shape[0])
    data.metadata.setdefault("metrics", {}).update({"avg_kl": avg_kl, "avg_kl_max": avg_kl_max,
                                                    "kl_loss_coef": coef})
    return data


# ------------------------------------------------------------------------------ a10 order / batching
def remove_tail_data(entries: List[Any], lcm_dp_size: int, n_samples_per_prompt: int) -> List[Any]:
    """trainer.py:353-375: keep the largest prompt count m with (m * n) % lcm_dp == 0."""
    stride = lcm_dp_size // math.gcd(lcm_dp_size, n_samples_per_prompt)
    if stride <= 1:
        return entries
    return entries[: (len(entries) // stride) * stride]


class PromptOrder:
    """Prompt-level batch order of build_dataloader (utils/trainer_utils.py:661-699) for training:
    torch.Generator().manual_seed(seed), shuffle=True, drop_last=True. Reproduces torch
    DataLoader's generator consumption: per epoch one int64 draw for the worker base seed,
    randperm(n) for the RandomSampler and the sampler's (empty) tail permutation. Pinned
    against torch.utils.data.DataLoader; the reference wraps torchdata's StatefulDataLoader
    (not in this image), whose sampler is assumed to consume the generator the same way."""

    def __init__(self, num_prompts: int, batch_size: int, seed: int = 42, drop_last: bool = True):
        self.n, self.bs, self.drop_last = num_prompts, batch_size, drop_last
        self.gen = torch.Generator()
        self.gen.manual_seed(seed)

    def __len__(self):
        return self.n // self.bs if self.drop_last else math.ceil(self.n / self.bs)

    def epoch(self) -> List[List[int]]:
        torch.empty((), dtype=torch.int64).random_(generator=self.gen)  # _BaseDataLoaderIter._base_seed
        perm = torch.randperm(self.n, generator=self.gen).tolist()
        # RandomSampler.__iter__ evaluates its trailing randperm(n)[:num_samples % n] when the
        # BatchSampler drains it at the end of every epoch: one more permutation's worth of draws
        torch.randperm(self.n, generator=self.gen)
        return [perm[i:i + self.bs] for i in range(0, len(self) * self.bs, self.bs)] if self.drop_last else \
            [perm[i:i + self.bs] for i in range(0, self.n, self.bs)]


def mini_batch_slices(batch_size: int, mini_batch_size: int) -> List[Tuple[int, int]]:
    """trainer.py:1067-1081: contiguous mini-batches, no shuffle, tail dropped."""
    return [(i * mini_batch_size, (i + 1) * mini_batch_size) for i in range(batch_size // mini_batch_size)]


def dp_slice(start: int, end: int, dp_size: int, dp_rank: int) -> Tuple[int, int]:
    """dispatch.py:163-205 (dispatch_from_staged): this DP rank's contiguous slice of a mini-batch."""
    n = end - start
    assert n % dp_size == 0, f"mini_batch_size must be divisible by dp_size, got {n} and {dp_size}"
    c = n // dp_size
    return start + dp_rank * c, start + (dp_rank + 1) * c


def reduce_metrics(metrics: Dict[str, List[float]]) -> Dict[str, float]:
    """worker_utils.py:8-22: mean, except *_max -> max and *_min -> min."""
    out = {}
    for k, v in metrics.items():
        assert len(v) > 0, f"No metrics for key {k}"
        assert all(isinstance(x, (int, float)) for x in v), f"Metrics for key {k} are not all numbers"
        out[k] = max(v) if k.endswith("_max") else min(v) if k.endswith("_min") else sum(v) / len(v)
    return out


@dataclass
class Experience:
    """dataset/replay_buffer.py:39-116 (the fields the micro-batch loop reads)."""

    sequences: torch.Tensor
    action_log_probs: Optional[torch.Tensor]
    base_action_log_probs: Optional[torch.Tensor]
    values: Optional[torch.Tensor]
    returns: Optional[torch.Tensor]
    advantages: Optional[torch.Tensor]
    attention_mask: Optional[torch.Tensor]
    loss_mask: Optional[torch.Tensor]
    action_mask: Optional[torch.Tensor]
    rollout_logprobs: Optional[torch.Tensor]
    num_actions: int
    info: Optional[dict]
    kl: Optional[torch.Tensor] = None
    metadata: Optional[Dict[str, Any]] = None


class BatchIterator:
    """worker_utils.py:38-90: micro-batches of a TrainingInputBatch as Experience objects."""

    def __init__(self, data: TrainingInputBatch, sample_batch_size: int, drop_last: bool = False):
        assert not drop_last, "drop_last is not supported yet"
        self.data = data
        self.sample_batch_size = sample_batch_size
        self.num_micro_batches = math.ceil(data.batch_size / sample_batch_size)
        self._chunks = data.chunk(sample_batch_size)
        self._iter = iter(self._chunks)

    def __len__(self):
        return self.num_micro_batches

    def __iter__(self):
        return self

    def __next__(self) -> Experience:
        try:
            return self.batch_to_experience(next(self._iter))
        except StopIteration:
            self._iter = iter(self._chunks)
            raise

    @staticmethod
    def batch_to_experience(batch: TrainingInputBatch) -> Experience:
        return Experience(
            sequences=batch["sequences"], action_log_probs=batch.get("action_log_probs"),
            base_action_log_probs=batch.get("base_action_log_probs"), values=batch.get("values"),
            returns=batch.get("returns"), advantages=batch.get("advantages"),
            attention_mask=batch.get("attention_mask"), loss_mask=batch.get("loss_mask"),
            action_mask=batch.get("response_mask"), num_actions=batch.metadata["response_length"],
            rollout_logprobs=batch.get("rollout_logprobs"), info={}, metadata=batch.metadata)
