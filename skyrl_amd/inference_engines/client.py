"""InferenceEngineClient: fans a batch out over the rollout engines and implements the
in-flight weight-update protocol (pause -> abort -> update -> resume, with token-in/token-out
retry of aborted requests).

Mirrors skyrl_train/inference_engines/inference_engine_client.py:37-330,590-630 and
route_prompts_to_engines (inference_engines/utils.py:84-150) without the HTTP endpoint.
"""

from __future__ import annotations

import asyncio
import hashlib
import random
import threading
from typing import Any, Dict, List, Optional, Union

from .base import InferenceEngineInput, InferenceEngineInterface, InferenceEngineOutput

ABORT_GENERATION_GRACE_PERIOD_SECONDS = 5


def hash_with_sha256(x: Union[int, str]) -> int:
    return int.from_bytes(hashlib.sha256(str(x).encode()).digest(), "big")


def route_prompts_to_engines(num_prompts: int, num_inference_engines: int,
                             session_ids: Optional[List[Union[int, str]]]) -> Dict[int, List[int]]:
    """utils.py:88-150: single prompt without session -> random engine; batch without
    sessions -> even contiguous split; with sessions -> sha256(session) % engines."""
    assert num_prompts > 0, "Number of prompts must be greater than 0"
    assert num_inference_engines > 0, "Number of inference engines must be greater than 0"
    if session_ids is not None:
        assert isinstance(session_ids, list) and all(isinstance(s, (int, str)) for s in session_ids), \
            "Session ID must be a list of integers or strings"
        assert len(session_ids) == num_prompts, "Session ID must have the same length as the number of prompts"
    if session_ids is None and num_prompts == 1:
        return {random.randint(0, num_inference_engines - 1): [0]}
    out: Dict[int, List[int]] = {}
    if session_ids is None:
        per = (num_prompts + num_inference_engines - 1) // num_inference_engines
        for r in range(num_inference_engines):
            ids = list(range(r * per, min((r + 1) * per, num_prompts)))
            if ids:
                out[r] = ids
        return out
    for i, sid in enumerate(session_ids):
        out.setdefault(hash_with_sha256(str(sid)) % num_inference_engines, []).append(i)
    return out


class InferenceEngineClient(InferenceEngineInterface):
    def __init__(self, engines: List[InferenceEngineInterface], tokenizer=None,
                 abort_grace_seconds: float = ABORT_GENERATION_GRACE_PERIOD_SECONDS):
        self.engines = engines
        self.tokenizer = tokenizer
        self.generation_paused_event = threading.Event()
        self.abort_grace_seconds = abort_grace_seconds

    async def _run_on_all_engines(self, method_name: str, *args, **kwargs):
        assert len(self.engines) > 0, "No engines to call method on"
        return await asyncio.gather(*[getattr(e, method_name)(*args, **kwargs) for e in self.engines])

    async def generate(self, input_batch: InferenceEngineInput) -> InferenceEngineOutput:
        prompts = input_batch.get("prompts")
        ids = input_batch.get("prompt_token_ids")
        session_ids = input_batch.get("session_ids")
        sp = input_batch.get("sampling_params")
        if (prompts is None) == (ids is None):
            raise ValueError("Either `prompts` or `prompt_token_ids` must be provided, but not both.")
        if ids is None:
            if self.tokenizer is None:
                raise ValueError("`prompts` need a tokenizer with a chat template")
            ids = self.tokenizer.apply_chat_template(prompts, add_generation_prompt=True, add_special_tokens=False,
                                                     return_dict=True, tokenize=True)["input_ids"]
        routing = route_prompts_to_engines(len(ids), len(self.engines), session_ids)
        if len(ids) == 1:
            ((eidx, _),) = routing.items()
            return await self._generate_single_with_retry(eidx, ids[0], sp)
        if self.generation_paused_event.is_set():
            raise RuntimeError("pause_generation is unsupported for batched InferenceEngineClient.generate().")
        order, tasks = [], []
        for eidx, idx in routing.items():
            tasks.append(asyncio.create_task(self.engines[eidx].generate(
                {"prompt_token_ids": [ids[i] for i in idx], "sampling_params": sp})))
            order.append(idx)
        results = await asyncio.gather(*tasks)
        n = len(ids)
        responses, reasons = [""] * n, [""] * n
        rids: List[List[int]] = [[] for _ in range(n)]
        lps: List[Optional[List[float]]] = [None] * n
        any_lp = False
        for idx, res in zip(order, results):
            for j, i in enumerate(idx):
                responses[i] = res["responses"][j]
                reasons[i] = res["stop_reasons"][j]
                rids[i] = res["response_ids"][j]
                if res.get("response_logprobs"):
                    any_lp = True
                    lps[i] = res["response_logprobs"][j]
        return InferenceEngineOutput(responses=responses, stop_reasons=reasons, response_ids=rids,
                                     response_logprobs=lps if any_lp else None)

    async def _generate_single_with_retry(self, engine_idx: int, original_prompt_ids: List[int],
                                          sampling_params: Optional[Dict[str, Any]]) -> InferenceEngineOutput:
        """inference_engine_client.py:223-330: resend (prompt + accumulated tokens) while the
        engine answers "abort", shrinking max_tokens by what was already generated."""
        sampling_params = dict(sampling_params or {})
        max_key = "max_tokens" if "max_tokens" in sampling_params else (
            "max_completion_tokens" if "max_completion_tokens" in sampling_params else None)
        original_max = sampling_params.get(max_key) if max_key else None
        acc_ids: List[int] = []
        acc_lps: List[float] = []
        stop_reason, text, turns = "abort", None, 0
        while stop_reason == "abort":
            await self._wait_for_generation_to_resume()
            cur = dict(sampling_params)
            if original_max is not None:
                new_max = original_max - len(acc_ids)
                assert new_max >= 0, f"Expect new_max_tokens to be non-negative, but got {new_max}"
                cur[max_key] = new_max
            out = await self.engines[engine_idx].generate(
                {"prompt_token_ids": [list(original_prompt_ids) + acc_ids], "sampling_params": cur})
            new_ids = out["response_ids"][0]
            text = out["responses"][0]
            stop_reason = out["stop_reasons"][0]
            new_lps = (out.get("response_logprobs") or [None])[0]
            if stop_reason == "abort" and len(new_ids) == 0:
                continue
            acc_ids.extend(new_ids)
            if new_lps is not None:
                acc_lps.extend(new_lps)
            turns += 1
        if turns != 1 and self.tokenizer is not None:
            text = self.tokenizer.decode(acc_ids, skip_special_tokens=True)
        return InferenceEngineOutput(responses=[text or ""], stop_reasons=[stop_reason], response_ids=[acc_ids],
                                     response_logprobs=[acc_lps] if acc_lps else None)

    def _select_engine_idx(self, session_id=None) -> int:
        if session_id is None:
            return random.randint(0, len(self.engines) - 1)
        return hash_with_sha256(str(session_id)) % len(self.engines)

    async def sample(self, prompt_token_ids: List[int], num_samples: int, sampling_params: Dict[str, Any],
                     session_id=None) -> InferenceEngineOutput:
        await self._wait_for_generation_to_resume()
        return await self.engines[self._select_engine_idx(session_id)].sample(
            prompt_token_ids=prompt_token_ids, num_samples=num_samples, sampling_params=sampling_params)

    # ---------------------------------------------------------------- pause / resume
    async def _wait_for_generation_to_resume(self) -> None:
        while self.generation_paused_event.is_set():
            await asyncio.sleep(0.05)

    async def pause_generation(self) -> None:
        """inference_engine_client.py:597-618: block new requests, let in-flight ones reach the
        schedulers, then abort them (they come back as "abort" and are retried on resume)."""
        if self.generation_paused_event.is_set():
            raise RuntimeError("Generation is already paused, cannot pause again.")
        self.generation_paused_event.set()
        await asyncio.sleep(self.abort_grace_seconds)
        await self._run_on_all_engines("abort_generation")

    async def resume_generation(self) -> None:
        if not self.generation_paused_event.is_set():
            raise RuntimeError("Generation is not paused, cannot resume.")
        self.generation_paused_event.clear()

    async def abort_generation(self) -> None:
        raise NotImplementedError("InferenceEngineClient does not implement abort_generation(), but calls "
                                  "`abort_generation` on all engines in `pause_generation()`.")

    # ---------------------------------------------------------------- fan-out
    async def wake_up(self, *args: Any, **kwargs: Any):
        return await self._run_on_all_engines("wake_up", *args, **kwargs)

    async def sleep(self, *args: Any, **kwargs: Any):
        return await self._run_on_all_engines("sleep", *args, **kwargs)

    async def init_weight_update_communicator(self, init_info):
        return await self._run_on_all_engines("init_weight_update_communicator", init_info)

    async def update_named_weights(self, request):
        return await self._run_on_all_engines("update_named_weights", request)

    async def reset_prefix_cache(self):
        return await self._run_on_all_engines("reset_prefix_cache")

    async def teardown(self):
        return await self._run_on_all_engines("teardown")

    async def chat_completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("HTTP endpoints are out of scope")

    async def completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("HTTP endpoints are out of scope")

    def tp_size(self) -> int:
        return self.engines[0].tp_size()

    def pp_size(self) -> int:
        return self.engines[0].pp_size()

    def dp_size(self) -> int:
        return len(self.engines)
