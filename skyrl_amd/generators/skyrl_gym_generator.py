"""Multi-turn agent loop: token-in/token-out generation against text envs.

Same contract as SkyRLGymGenerator (skyrl_train/generators/skyrl_gym_generator.py:102-983):
`generate(GeneratorInput) -> GeneratorOutput` runs one agent loop per trajectory. Each turn is
one `generate` on the inference client (the MI355X engine) with the running token ids as the
prompt. The env answers with observations, which are tokenized and appended with loss mask 0
(rollout logprob 0.0), so the learner trains only on tokens the policy produced. Per-step
rewards land on the last generated token of their turn.

Modes (as the reference):
  * use_conversation_multi_turn=True: observations become user messages in the chat template;
    their ids are the template's suffix after a fixed base conversation (the "fixed base"
    tokenization, :140-158, :513-547), plus the generation prompt for the next turn;
  * use_conversation_multi_turn=False: the whole interaction is one assistant message; the
    observation text is encoded directly, a turn's trailing eos is dropped (:915-983), and an
    eos is appended at the end unless the trajectory was cut by length.
Not built: custom chat templates (re-tokenizing chat history), step-wise trajectories and the
batched (single engine call) mode — they raise.
"""

from __future__ import annotations

import asyncio
import copy
import uuid
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .. import envs as envs_mod
from ..config import SamplingParams


@dataclass
class TrajectoryID:
    instance_id: str
    repetition_id: int

    def to_string(self) -> str:
        return f"{self.instance_id}_{self.repetition_id}"


@dataclass
class GeneratorConfig:
    """The generator.* keys the agent loop reads (config/config.py:347-391)."""

    max_turns: int = 1
    max_input_length: int = 512
    batched: bool = False
    use_conversation_multi_turn: bool = True
    append_eos_token_after_stop_str_in_multi_turn: bool = True
    zero_reward_on_non_stop: bool = False
    apply_overlong_filtering: bool = False
    step_wise_trajectories: bool = False
    chat_template_kwargs: Dict[str, Any] = field(default_factory=dict)
    sampling_params: SamplingParams = field(default_factory=SamplingParams)


@dataclass
class _Turn:
    text: str
    ids: List[int]
    logprobs: Optional[List[float]]
    new_obs: List[Dict[str, str]]
    obs_ids: List[int]
    reward: float
    added_eos: bool

    def loss_mask(self) -> List[int]:  # TurnOutput.get_turn_loss_mask (:73-87)
        gen = [1] * len(self.ids)
        if self.added_eos:
            gen[-1] = 0
        return gen + [0] * len(self.obs_ids)

    def rollout_logprobs(self) -> Optional[List[float]]:
        if not self.logprobs:
            return None
        return self.logprobs + [0.0] * len(self.obs_ids)


def chat_ids(tokenizer, messages, add_generation_prompt: bool, **kw) -> List[int]:
    """apply_chat_template(tokenize=True) as a plain id list (transformers >= 5 returns a
    BatchEncoding by default, 4.x a list)."""
    out = tokenizer.apply_chat_template(messages, add_generation_prompt=add_generation_prompt, tokenize=True, **kw)
    if hasattr(out, "keys") and "input_ids" in out:
        out = out["input_ids"]
    return list(out)


def get_generation_prompt_ids(tokenizer, **kw) -> List[int]:
    """Ids the chat template adds for add_generation_prompt=True (utils.py:147-167)."""
    base = chat_ids(tokenizer, [{"role": "user", "content": ""}], False, **kw)
    gen = chat_ids(tokenizer, [{"role": "user", "content": ""}], True, **kw)
    return gen[len(base):]


def get_vllm_sampling_params(sp: SamplingParams) -> Dict[str, Any]:
    """generator.sampling_params -> the engine's request dict (inference_engines/utils.py:15-42)."""
    out = {"min_tokens": 1, "skip_special_tokens": True, "include_stop_str_in_output": True,
           "max_tokens": sp.max_generate_length, "temperature": sp.temperature, "top_p": sp.top_p,
           "top_k": sp.top_k, "min_p": sp.min_p, "logprobs": sp.logprobs,
           "stop": list(sp.stop) if sp.stop is not None else None}
    for k, v in (sp.additional_kwargs or {}).items():
        out.setdefault(k, v)
    return out


def get_rollout_metrics(responses, rewards, env_metrics=None, env_classes=None) -> Dict[str, float]:
    """utils.py:293-348."""
    n = np.array([len(r) for r in responses])
    flat = np.array([float(np.sum(r)) if isinstance(r, list) else float(r) for r in rewards])
    nz, z = flat > 0.0, flat == 0.0
    out = {
        "generate/min_num_tokens": np.min(n).item(),
        "generate/max_num_tokens": np.max(n).item(),
        "generate/avg_num_tokens": np.mean(n).item(),
        "generate/std_num_tokens": np.std(n).item(),
        "generate/avg_tokens_non_zero_rewards": (np.mean(n[nz]) if nz.sum() > 0 else np.zeros(1)).item(),
        "generate/avg_tokens_zero_rewards": (np.mean(n[z]) if z.sum() > 0 else np.zeros(1)).item(),
    }
    if env_metrics is not None and env_classes is not None:
        per_env = defaultdict(list)
        for cls, m in zip(env_classes, env_metrics):
            per_env[cls].append(m)
        for cls, ms in per_env.items():
            vals: Dict[str, List[float]] = {}
            for m in ms:
                for k, v in m.items():
                    if isinstance(v, (bool, int, float)):
                        vals.setdefault(k, []).append(float(v))
            for k, v in vals.items():
                out[f"environment/{cls}/{k}"] = sum(v) / len(v)
    return out


def apply_overlong_filtering(loss_masks, response_ids, eos_token_id):
    """DAPO overlong filtering: a response that does not end in eos trains on nothing (utils.py:274-290)."""
    return [[0] * len(m) if not r or r[-1] != eos_token_id else m for m, r in zip(loss_masks, response_ids)]


class SkyRLGymGenerator:
    def __init__(self, generator_cfg: GeneratorConfig, env_cfg: Optional[Dict[str, Any]], inference_engine_client,
                 tokenizer):
        cfg = generator_cfg
        if cfg.batched or cfg.step_wise_trajectories:
            raise NotImplementedError("batched and step-wise trajectories are not built (agent loop only)")
        self.cfg = cfg
        self.env_cfg = env_cfg or {}
        self.client = inference_engine_client
        self.tokenizer = tokenizer
        self.max_turns = cfg.max_turns
        self.multi_turn = cfg.use_conversation_multi_turn
        kw = cfg.chat_template_kwargs
        self.generation_prompt_ids = get_generation_prompt_ids(tokenizer, **kw) if self.multi_turn else None
        self.base_conversation = [{"role": "system", "content": "You are a helpful assistant."},
                                  {"role": "user", "content": "I am a user."}]
        base = chat_ids(tokenizer, self.base_conversation, False, **kw)
        eos = tokenizer.eos_token_id
        if eos in base:  # cut after the last eos so the observation suffix carries what follows it
            base = base[:len(base) - base[::-1].index(eos)]
        self.base_conversation_token_ids = base

    # ---------------------------------------------------------------- one trajectory
    def _obs_ids(self, new_obs, done: bool) -> List[int]:
        if self.multi_turn:
            if new_obs:
                full = chat_ids(self.tokenizer, [*self.base_conversation, *new_obs], not done,
                                **self.cfg.chat_template_kwargs)
                return full[len(self.base_conversation_token_ids):]
            return [] if done else list(self.generation_prompt_ids)
        ids: List[int] = []
        for m in new_obs:
            ids.extend(self.tokenizer.encode(m["content"], add_special_tokens=False))
        return ids

    async def agent_loop(self, prompt, env_class: str, env_extras: Dict[str, Any], max_tokens: int,
                         max_input_length: int, sampling_params: Optional[Dict[str, Any]] = None,
                         trajectory_id: Optional[TrajectoryID] = None):
        tok = self.tokenizer
        eos = tok.eos_token_id
        env_extras = dict(env_extras or {})
        env_extras["max_turns"] = self.max_turns
        env = envs_mod.make(env_class, env_config=self.env_cfg.get(env_class), extras=env_extras)
        session_id = trajectory_id.to_string() if trajectory_id is not None else uuid.uuid4().hex
        chat, _ = env.init(copy.deepcopy(prompt))
        input_ids = chat_ids(tok, chat, True, **self.cfg.chat_template_kwargs)
        p0 = len(input_ids)
        cur_sp = sampling_params if sampling_params is not None else vars(self.cfg.sampling_params)
        stop_strs = cur_sp.get("stop", None)
        loss_mask: List[int] = []
        logprobs: Optional[List[float]] = [] if self.cfg.sampling_params.logprobs is not None else None
        end_idx: Optional[int] = None
        per_step: List[Tuple[float, Optional[int]]] = []
        done = False
        stop_reason = "stop"
        while not done:
            if len(input_ids) > max_input_length:
                stop_reason = "length"
                break
            out = await self.client.generate({"prompt_token_ids": [input_ids], "session_ids": [session_id],
                                              "sampling_params": sampling_params})
            text = out["responses"][0]
            ids = list(out["response_ids"][0])
            stop_reason = out["stop_reasons"][0]
            lps = out.get("response_logprobs", None)
            lps = list(lps[0]) if lps is not None else None
            added_eos = False
            if stop_strs is not None and self.cfg.append_eos_token_after_stop_str_in_multi_turn and self.multi_turn:
                if text.endswith(tuple(stop_strs)) and ids[-1] != eos:
                    ids.append(eos)
                    if lps is not None:
                        lps.append(0.0)
                    added_eos = True
            step = env.step(text)
            new_obs = step["observations"]
            done = step["done"]
            if step.get("postprocessed_action", None) is not None:
                text = step["postprocessed_action"]
                ids = tok.encode(text, add_special_tokens=False)
            turn = _Turn(text, ids, lps, new_obs, self._obs_ids(new_obs, done), step["reward"], added_eos)
            if text.endswith(tok.eos_token):  # chat history bookkeeping (_update_chat_history)
                text = text[:-len(tok.eos_token)]
            chat = chat + [{"role": "assistant", "content": text}] + list(new_obs)
            if self.multi_turn:
                end_idx = len(input_ids) + len(turn.ids) - 1
                input_ids += turn.ids + turn.obs_ids
                loss_mask += turn.loss_mask()
                t_lp = turn.rollout_logprobs()
                if logprobs is not None and t_lp is not None:
                    logprobs += t_lp
            else:
                gen = turn.ids[:-1] if turn.ids and turn.ids[-1] == eos else list(turn.ids)
                end_idx = len(input_ids) + len(gen) - 1
                input_ids += gen + turn.obs_ids
                loss_mask += [1] * len(gen) + [0] * len(turn.obs_ids)
                if logprobs is not None and turn.logprobs is not None:
                    logprobs += turn.logprobs[:len(gen)] + [0.0] * len(turn.obs_ids)
            per_step.append((turn.reward, end_idx))
        env_metrics = env.get_metrics()
        env.close()
        prompt_ids = input_ids[:p0]
        n_resp = (end_idx - p0 + 1) if end_idx is not None else 0
        assert not any(loss_mask[n_resp:]), "loss_mask after the response end must be 0"
        response_ids = input_ids[p0:p0 + n_resp]
        loss_mask = loss_mask[:n_resp]
        rollout_lp = logprobs[:n_resp] if logprobs is not None else None
        per_step = [(r, i - p0) for r, i in per_step]
        appended_eos = False
        if not self.multi_turn and stop_reason != "length" and response_ids and response_ids[-1] != eos:
            response_ids.append(eos)
            loss_mask.append(1)
            if rollout_lp is not None:
                rollout_lp.append(0.0)
            appended_eos = True
        rewards = [0.0] * len(response_ids)
        for i, (r, idx) in enumerate(per_step):
            if idx >= len(response_ids):
                break
            if appended_eos and i == len(per_step) - 1:
                rewards[-1] = r
            else:
                rewards[idx] += r
        return {"response_ids": response_ids, "reward": rewards, "stop_reason": stop_reason, "loss_mask": loss_mask,
                "prompt_ids": prompt_ids, "rollout_logprobs": rollout_lp, "env_metrics": env_metrics}

    # ---------------------------------------------------------------- batch
    async def generate(self, input_batch: Dict[str, Any]) -> Dict[str, Any]:
        prompts = input_batch["prompts"]
        env_classes = input_batch["env_classes"]
        extras = input_batch.get("env_extras") or [{} for _ in prompts]
        tids = input_batch.get("trajectory_ids", None)
        sp = input_batch.get("sampling_params", None)
        outs = await asyncio.gather(*[
            self.agent_loop(prompts[i], env_classes[i], extras[i], self.cfg.sampling_params.max_generate_length,
                            self.cfg.max_input_length, sampling_params=sp,
                            trajectory_id=tids[i] if tids is not None else None) for i in range(len(prompts))])
        responses = [o["response_ids"] for o in outs]
        rewards = [o["reward"] for o in outs]
        stop_reasons = [o["stop_reason"] for o in outs]
        loss_masks = [o["loss_mask"] for o in outs]
        get_lp = (sp.get("logprobs", None) is not None) if sp is not None else (
            self.cfg.sampling_params.logprobs is not None)
        metrics = get_rollout_metrics(responses, rewards, [o["env_metrics"] for o in outs], env_classes)
        if self.cfg.zero_reward_on_non_stop:
            rewards = [r if s == "stop" else ([0.0] * len(r) if isinstance(r, list) else 0.0)
                       for r, s in zip(rewards, stop_reasons)]
        if self.cfg.apply_overlong_filtering:
            loss_masks = apply_overlong_filtering(loss_masks, responses, self.tokenizer.eos_token_id)
        return {"prompt_token_ids": [o["prompt_ids"] for o in outs], "response_ids": responses, "rewards": rewards,
                "loss_masks": loss_masks, "stop_reasons": stop_reasons, "rollout_metrics": metrics,
                "rollout_logprobs": [o["rollout_logprobs"] for o in outs] if get_lp else None,
                "trajectory_ids": None, "is_last_step": None}
