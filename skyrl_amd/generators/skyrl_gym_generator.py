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
    eos is appended at the end unless the trajectory was cut by length;
  * custom chat template (generator.chat_template) with multi-turn: the chat history is
    re-tokenized every turn, and the final loss mask is the template's assistant-token mask
    (:220-249, :291-301, :412-425, :813-847);
  * step_wise_trajectories: one training sample per turn (prompt = the re-applied chat so far,
    response = the turn's ids + observation ids), flattened with trajectory ids and is_last_step
    (:270-379, :454-459, :712-733);
  * batched: one text-in engine call for single-turn rollouts (generate_batched, :579-663).
"""

from __future__ import annotations

import asyncio
import copy
import os
import uuid
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .. import envs as envs_mod
from ..config import SamplingParams

# generator.chat_template by name (generators/utils.py:62-99): templates with {% generation %}
# tags, so the assistant-token mask of the re-tokenized history is the loss mask
CUSTOM_CHAT_TEMPLATES = {
    "qwen3_with_thinking": (
        "{% for message in messages %}"
        "{% if (message['role'] != 'assistant') %}"
        "{{'<|im_start|>' + message['role'] + '\n' + message['content'] + '<|im_end|>' + '\n'}}"
        "{% elif (message['role'] == 'assistant')%}"
        "{{'<|im_start|>' + message['role'] + '\n'}}"
        "{% generation %}"
        "{{message['content'] + '<|im_end|>'}}"
        "{% endgeneration %}"
        "{{'\n'}}"
        "{% endif %}"
        "{% endfor %}"
    ),
    # drops the <think> part of every assistant message but the last one
    "qwen3_without_thinking": (
        "{% for message in messages %}"
        "{% if (message['role'] != 'assistant') %}"
        "{{'<|im_start|>' + message['role'] + '\n' + message['content'] + '<|im_end|>' + '\n'}}"
        "{% elif (message['role'] == 'assistant')%}"
        "{{'<|im_start|>' + message['role'] + '\n'}}"
        "{% generation %}"
        "{% set full_content = message['content'] %}"
        "{% set mycontent = message['content'] %}"
        "{% set is_last_message = loop.last and messages[-1]['role'] == 'assistant' %}"
        "{% if '</think>' in full_content and not is_last_message %}"
        "{% set mycontent = full_content.split('</think>')[-1].lstrip('\n') %}"
        "{% endif %}"
        "{{mycontent + '<|im_end|>'}}"
        "{% endgeneration %}"
        "{{'\n'}}"
        "{% endif %}"
        "{% endfor %}"
    ),
}


@dataclass
class ChatTemplateConfig:
    """generator.chat_template (config.py:336-338): source "name" (CUSTOM_CHAT_TEMPLATES) or
    "file" (a template file path); no name_or_path = the tokenizer's own template."""

    source: str = "name"
    name_or_path: Optional[str] = None


def get_custom_chat_template(cfg=None) -> Optional[str]:
    """generators/utils.py:102-144."""
    if cfg is None:
        return None
    if isinstance(cfg, dict):
        cfg = ChatTemplateConfig(**cfg)
    if not cfg.source:
        raise ValueError("'source' is required in chat_template_config")
    if not cfg.name_or_path:
        return None
    if cfg.source == "name":
        if cfg.name_or_path not in CUSTOM_CHAT_TEMPLATES:
            raise ValueError(f"Template name '{cfg.name_or_path}' not found. "
                             f"Available templates: {list(CUSTOM_CHAT_TEMPLATES.keys())}")
        return CUSTOM_CHAT_TEMPLATES[cfg.name_or_path]
    if cfg.source == "file":
        path = cfg.name_or_path
        if os.path.normpath(path).startswith("..") or "\x00" in path:
            raise ValueError(f"Invalid template file path '{path}'")
        try:
            with open(os.path.abspath(os.path.expanduser(path)), "r", encoding="utf-8") as f:
                return f.read()
        except OSError as e:
            raise ValueError(f"Template file '{path}' not found") from e
    raise ValueError(f"Invalid source '{cfg.source}'. Must be 'name' or 'file'")


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
    chat_template: ChatTemplateConfig = field(default_factory=ChatTemplateConfig)
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


def _chat_ids(tokenizer, messages, add_generation_prompt: bool, chat_template=None, **kw) -> List[int]:
    if chat_template is not None:
        kw = dict(kw, chat_template=chat_template)
    return chat_ids(tokenizer, messages, add_generation_prompt, **kw)


class SkyRLGymGenerator:
    def __init__(self, generator_cfg: GeneratorConfig, env_cfg: Optional[Dict[str, Any]], inference_engine_client,
                 tokenizer):
        cfg = generator_cfg
        self.cfg = cfg
        self.env_cfg = env_cfg or {}
        self.client = inference_engine_client
        self.tokenizer = tokenizer
        self.max_turns = cfg.max_turns
        self.batched = cfg.batched
        self.multi_turn = cfg.use_conversation_multi_turn
        self.custom_chat_template = get_custom_chat_template(cfg.chat_template)
        kw = cfg.chat_template_kwargs
        self.generation_prompt_ids = get_generation_prompt_ids(tokenizer, **kw) if self.multi_turn else None
        self._validate_cfg()
        self.base_conversation = [{"role": "system", "content": "You are a helpful assistant."},
                                  {"role": "user", "content": "I am a user."}]
        base = chat_ids(tokenizer, self.base_conversation, False, **kw)
        eos = tokenizer.eos_token_id
        if eos in base:  # cut after the last eos so the observation suffix carries what follows it
            base = base[:len(base) - base[::-1].index(eos)]
        self.base_conversation_token_ids = base

    def _validate_cfg(self):  # :160-176
        cfg = self.cfg
        if len(cfg.chat_template_kwargs) and cfg.batched:
            raise ValueError("`chat_template_kwargs` is not compatible with `batched=True` since the chat templating "
                             "is handled by the inference engine")
        if cfg.step_wise_trajectories:
            if self.batched:
                raise ValueError("`step_wise_trajectories` doesn't support `batched=True`")
            if self.custom_chat_template is not None:
                raise ValueError(f"`step_wise_trajectories` doesn't support custom chat template, got {cfg.chat_template}")
            if not self.multi_turn:
                raise ValueError("`step_wise_trajectories` doesn't support `use_conversation_multi_turn=False`")

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
        """One trajectory. Returns the TrajectoryOutput fields as a dict, or for step-wise
        trajectories {"step_outputs": [per-turn dicts]}."""
        tok = self.tokenizer
        eos = tok.eos_token_id
        kw = self.cfg.chat_template_kwargs
        retok = self.multi_turn and self.custom_chat_template is not None
        tmpl = self.custom_chat_template if retok else None
        step_wise = self.cfg.step_wise_trajectories
        env_extras = dict(env_extras or {})
        env_extras["max_turns"] = self.max_turns
        env = envs_mod.make(env_class, env_config=self.env_cfg.get(env_class), extras=env_extras)
        session_id = trajectory_id.to_string() if trajectory_id is not None else uuid.uuid4().hex
        chat, _ = env.init(copy.deepcopy(prompt))
        chat0 = len(chat)
        input_ids = _chat_ids(tok, chat, not retok, tmpl, **kw)
        p0 = len(input_ids)
        cur_sp = sampling_params if sampling_params is not None else vars(self.cfg.sampling_params)
        stop_strs = cur_sp.get("stop", None)
        loss_mask: Optional[List[int]] = []
        logprobs: Optional[List[float]] = [] if self.cfg.sampling_params.logprobs is not None else None
        end_idx: Optional[int] = None
        per_step: List[Tuple[float, Optional[int]]] = []
        steps: List[Dict[str, Any]] = []
        new_obs: List[Dict[str, str]] = []
        done = False
        stop_reason = "stop"
        while not done:
            if len(input_ids) > max_input_length:
                stop_reason = "length"
                break
            if step_wise or retok:  # re-apply the whole chat template (so the length check is right)
                input_ids = _chat_ids(tok, chat, True, tmpl, **kw)
                loss_mask = []
                logprobs = None
            out = await self.client.generate({"prompt_token_ids": [input_ids], "session_ids": [session_id],
                                              "sampling_params": sampling_params})
            text = out["responses"][0]
            ids = list(out["response_ids"][0])
            stop_reason = out["stop_reasons"][0]
            lps = out.get("response_logprobs", None)
            if lps is not None:
                lps = list(lps[0])
                if self.custom_chat_template is not None:
                    raise ValueError("Response Logprobs bookkeeping is not supported with custom chat template")
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
            if step_wise:
                steps.append({"response_ids": turn.ids + turn.obs_ids, "reward": turn.reward,
                              "loss_mask": turn.loss_mask(), "prompt_ids": list(input_ids),
                              "rollout_logprobs": turn.rollout_logprobs(), "stop_reason": stop_reason,
                              "env_metrics": env.get_metrics() if done else {}})
            if text.endswith(tok.eos_token):  # chat history bookkeeping (_update_chat_history)
                text = text[:-len(tok.eos_token)]
            chat = chat + [{"role": "assistant", "content": text}] + list(new_obs)
            if retok:  # loss mask, response end and logprobs come from the re-tokenized history
                loss_mask, end_idx, logprobs = None, None, None
            elif self.multi_turn and step_wise:  # no cumulative ids: the turn is its own sample
                end_idx, loss_mask, logprobs = len(turn.ids) - 1, None, None
            elif self.multi_turn:
                end_idx = len(input_ids) + len(turn.ids) - 1
                input_ids = input_ids + turn.ids + turn.obs_ids
                loss_mask += turn.loss_mask()
                t_lp = turn.rollout_logprobs()
                if logprobs is not None and t_lp is not None:
                    logprobs += t_lp
            else:
                gen = turn.ids[:-1] if turn.ids and turn.ids[-1] == eos else list(turn.ids)
                end_idx = len(input_ids) + len(gen) - 1
                input_ids = input_ids + gen + turn.obs_ids
                loss_mask += [1] * len(gen) + [0] * len(turn.obs_ids)
                if logprobs is not None and turn.logprobs is not None:
                    logprobs += turn.logprobs[:len(gen)] + [0.0] * len(turn.obs_ids)
            per_step.append((turn.reward, end_idx))
        env_metrics = env.get_metrics()
        env.close()
        if step_wise:  # per-token reward on each turn's last generated token (:454-459)
            for so, (r, idx) in zip(steps, per_step):
                pt = [0.0] * len(so["response_ids"])
                pt[idx] = float(r)
                so["reward"] = pt
            return {"step_outputs": steps}
        prompt_ids = input_ids[:p0]
        rollout_lp = None
        if retok:  # the template's assistant-token mask over the turns (final observation excluded)
            enc = tok.apply_chat_template(chat[chat0:len(chat) - len(new_obs)], chat_template=tmpl,
                                          add_generation_prompt=False, return_dict=True,
                                          return_assistant_tokens_mask=True, tokenize=True, **kw)
            loss_mask = list(enc["assistant_masks"])
            response_ids = list(enc["input_ids"])
        else:
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
        if self.custom_chat_template:
            rewards = per_step[-1][0]  # one response-level reward: the last step's
        else:
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

    # ---------------------------------------------------------------- single-turn, one engine call
    async def generate_batched(self, prompts, env_classes, env_extras, max_tokens: int,
                               sampling_params: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        """Text-in-token-out single-turn rollouts in one engine call (:579-663)."""
        envs, init_prompts = [], []
        for cls, extra, prompt in zip(env_classes, env_extras, prompts):
            extra = dict(extra or {})
            extra["max_turns"] = self.max_turns
            env = envs_mod.make(cls, env_config=self.env_cfg.get(cls), extras=extra)
            init_prompt, _ = env.init(prompt)
            init_prompts.append(init_prompt)
            envs.append(env)
        out = await self.client.generate({"prompts": init_prompts, "sampling_params": sampling_params})
        outputs, responses, stop_reasons = out["responses"], out["response_ids"], out["stop_reasons"]
        logprobs = out.get("response_logprobs", None)
        truncated, rewards, loss_masks, env_metrics = [], [], [], []
        truncated_lp: Optional[List[List[float]]] = [] if logprobs is not None else None
        for i, (text, resp, env) in enumerate(zip(outputs, responses, envs)):
            rewards.append(env.step(text)["reward"])
            resp = list(resp)[:max_tokens]
            loss_masks.append([1] * len(resp))
            truncated.append(resp)
            if logprobs is not None:
                truncated_lp.append(list(logprobs[i])[:len(resp)])
            env_metrics.append(env.get_metrics())
            env.close()
        prompt_token_ids = [chat_ids(self.tokenizer, p, True) for p in init_prompts]
        metrics = get_rollout_metrics(responses, rewards, env_metrics, env_classes)
        if self.cfg.apply_overlong_filtering:
            loss_masks = apply_overlong_filtering(loss_masks, responses, self.tokenizer.eos_token_id)
        return {"prompt_token_ids": prompt_token_ids, "response_ids": truncated, "rewards": rewards,
                "loss_masks": loss_masks, "stop_reasons": stop_reasons, "rollout_metrics": metrics,
                "rollout_logprobs": truncated_lp}

    # ---------------------------------------------------------------- batch
    async def generate(self, input_batch: Dict[str, Any]) -> Dict[str, Any]:
        prompts = input_batch["prompts"]
        env_classes = input_batch["env_classes"]
        extras = input_batch.get("env_extras") or [{} for _ in prompts]
        tids = input_batch.get("trajectory_ids", None)
        step_wise = self.cfg.step_wise_trajectories
        if step_wise:
            assert tids is not None, "`trajectory_ids` is a required field for step wise training"
        sp = input_batch.get("sampling_params", None)
        max_tokens = self.cfg.sampling_params.max_generate_length
        if self.batched:
            return await self.generate_batched(prompts, env_classes, extras, max_tokens, sp)
        outs = await asyncio.gather(*[
            self.agent_loop(prompts[i], env_classes[i], extras[i], max_tokens, self.cfg.max_input_length,
                            sampling_params=sp, trajectory_id=tids[i] if tids is not None else None)
            for i in range(len(prompts))])
        is_last_step = out_tids = None
        if step_wise:  # flatten turns into samples (:712-733)
            flat, is_last_step, out_tids, classes = [], [], [], []
            for i, o in enumerate(outs):
                for j, so in enumerate(o["step_outputs"]):
                    flat.append(so)
                    is_last_step.append(j == len(o["step_outputs"]) - 1)
                    out_tids.append(tids[i])
                    classes.append(env_classes[i])
            outs, env_classes = flat, classes
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
                "trajectory_ids": out_tids, "is_last_step": is_last_step}
