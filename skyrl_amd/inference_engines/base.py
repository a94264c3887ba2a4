"""Inference-engine plugin surface: the reference's InferenceEngineInterface and its I/O types.

Mirrors skyrl_train/inference_engines/base.py:1-166 (same names, fields and default `sample`
behaviour), so a Generator written against the reference drives the MI355X engine unchanged.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, Hashable, List, Optional, TypedDict

MessageType = Dict[str, str]
ConversationType = List[MessageType]


class InferenceEngineInput(TypedDict, total=False):
    # Either prompts or prompt_token_ids must be provided, but not both (base.py:12-17).
    prompts: Optional[List[ConversationType]]
    prompt_token_ids: Optional[List[List[int]]]
    sampling_params: Optional[Dict[str, Any]]
    session_ids: Optional[List[Hashable]]


class InferenceEngineOutput(TypedDict):
    # base.py:20-31: token ids are the engine's outputs; text is their decoding.
    responses: List[str]
    response_ids: List[List[int]]
    stop_reasons: List[str]
    response_logprobs: Optional[List[List[float]]]


class InferenceEngineInterface(ABC):
    """base.py:34-166."""

    @abstractmethod
    async def generate(self, input_batch: InferenceEngineInput) -> InferenceEngineOutput:
        raise NotImplementedError

    async def sample(self, prompt_token_ids: List[int], num_samples: int,
                     sampling_params: Dict[str, Any]) -> InferenceEngineOutput:
        """num_samples independent completions of one prompt (base.py:42-87)."""
        ids, texts, reasons, lps = [], [], [], []
        for _ in range(num_samples):
            out = await self.generate({"prompts": None, "prompt_token_ids": [prompt_token_ids],
                                       "sampling_params": sampling_params, "session_ids": None})
            ids.append(out["response_ids"][0])
            texts.append(out["responses"][0])
            reasons.append(out["stop_reasons"][0])
            if out.get("response_logprobs") is not None:
                lps.append(out["response_logprobs"][0])
        return {"response_ids": ids, "responses": texts, "stop_reasons": reasons,
                "response_logprobs": lps if lps else None}

    @abstractmethod
    async def chat_completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError

    @abstractmethod
    async def completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError

    @abstractmethod
    async def wake_up(self, *args: Any, **kwargs: Any):
        raise NotImplementedError

    @abstractmethod
    async def sleep(self, *args: Any, **kwargs: Any):
        raise NotImplementedError

    @abstractmethod
    async def init_weight_update_communicator(self, init_info):
        raise NotImplementedError

    @abstractmethod
    async def update_named_weights(self, request):
        raise NotImplementedError

    @abstractmethod
    async def teardown(self):
        raise NotImplementedError

    @abstractmethod
    async def reset_prefix_cache(self):
        raise NotImplementedError

    @abstractmethod
    def tp_size(self) -> int:
        raise NotImplementedError

    @abstractmethod
    def pp_size(self) -> int:
        raise NotImplementedError

    @abstractmethod
    def dp_size(self) -> int:
        raise NotImplementedError

    @abstractmethod
    async def abort_generation(self) -> None:
        """Abort all running and waiting requests: they return the tokens generated so far with
        stop_reason "abort" (a waiting request returns zero tokens) (base.py:159-166)."""
        raise NotImplementedError
