"""Rollout token sampler: the per-decode-step launcher of skyrl_sample.

Replaces the vLLM sampler behind VLLMInferenceEngine.generate
(skyrl_train/inference_engines/vllm/vllm_engine.py:196-218) for the build's own decode
loop. `SamplingParams` keys and defaults follow config/ppo_base_config.yaml:316-324
(temperature 1.0, top_k -1, min_p 0.0, top_p 1.0, logprobs 0); the per-engine seed
convention is `seed + engine_index` (ray_wrapped_inference_engine.py:241).

A decode loop calls the sampler once per generated token for every live sequence, so the
host cost per call matters: TokenSampler binds the ctypes argument list once and each
`step()` is a single foreign call (a few microseconds), leaving the GPU as the bound.
"""

from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _ffi, ops
from .config import SamplingParams


class TokenSampler:
    """Samples one token per sequence per decode step into preallocated [max_steps, nseq] buffers."""

    def __init__(self, nseq: int, vocab: int, max_steps: int, device, params: Optional[SamplingParams] = None,
                 seed: int = 0, seq_ids: Optional[torch.Tensor] = None, dtype=torch.bfloat16):
        p = params or SamplingParams()
        self.nseq, self.vocab, self.max_steps = nseq, vocab, max_steps
        self.device = torch.device(device)
        self.params = p
        self.seed = int(seed)
        self.dtype_code = _ffi.BF16 if dtype == torch.bfloat16 else _ffi.F32
        self.tokens = torch.empty((max_steps, nseq), dtype=torch.int32, device=self.device)
        self.logprobs = torch.empty((max_steps, nseq), dtype=torch.float32, device=self.device)
        self.seq_ids = (torch.arange(nseq, dtype=torch.int64, device=self.device) if seq_ids is None
                        else seq_ids.to(self.device, torch.int64).contiguous())
        self.workspace = torch.zeros(_ffi.query("skyrl_sample_workspace_bytes", nseq, vocab), dtype=torch.uint8,
                                     device=self.device)
        self._fn = _ffi.load().skyrl_sample
        self._fn_ex = _ffi.load().skyrl_sample_ex  # under an active _ffi.variant(...)
        self._ids_ptr, self._ws_ptr = self.seq_ids.data_ptr(), self.workspace.data_ptr()
        self._tok_ptr, self._lp_ptr = self.tokens.data_ptr(), self.logprobs.data_ptr()
        self._err = _ffi.load().skyrl_last_error

    def step_ptr(self, logits_ptr: int, row_stride: int, t: int, stream_handle: int, nseq: Optional[int] = None):
        """Lowest-overhead form for decode loops: raw device address of row 0 of step t's
        [nseq, V] logits, row stride in elements, and the hipStream_t handle. `nseq` (default all):
        the live sequences of this step, the first nseq of the sampler's (a continuous batch whose
        finished sequences have left; their slots keep their earlier outputs)."""
        p = self.params
        n = self.nseq if nseq is None else int(nseq)
        if not 0 <= n <= self.nseq:
            raise ValueError(f"nseq {n} outside [0, {self.nseq}]")
        args = (logits_ptr, self.dtype_code, row_stride, n, self.vocab, float(p.temperature),
                int(p.top_k if p.top_k is not None else -1), _top_p(p), float(p.min_p or 0.0),
                ctypes.c_uint64(self.seed & 0xFFFFFFFFFFFFFFFF), self._ids_ptr, int(t),
                self._tok_ptr + 4 * self.nseq * t, self._lp_ptr + 4 * self.nseq * t, self._ws_ptr, stream_handle)
        v = _ffi.current_variant()
        rc = self._fn(*args) if v is None else self._fn_ex(*args, ctypes.byref(v))
        if rc != 0:
            raise _ffi.SkyrlHipError(f"skyrl_sample failed: {self._err().decode()}")

    def step(self, logits: torch.Tensor, t: int, stream: Optional[torch.cuda.Stream] = None):
        """Sample decode step t from logits [nseq, V] (unit vocab stride, any row stride)."""
        if logits.shape != (self.nseq, self.vocab) or logits.stride(1) != 1:
            raise ValueError(f"logits must be [{self.nseq}, {self.vocab}] with unit vocab stride")
        s = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        p = self.params
        args = (logits.data_ptr(), self.dtype_code, logits.stride(0), self.nseq, self.vocab, float(p.temperature),
                int(p.top_k if p.top_k is not None else -1), _top_p(p), float(p.min_p or 0.0),
                ctypes.c_uint64(self.seed & 0xFFFFFFFFFFFFFFFF), self.seq_ids.data_ptr(), int(t),
                self.tokens[t].data_ptr(), self.logprobs[t].data_ptr(), self.workspace.data_ptr(), s)
        v = _ffi.current_variant()
        rc = self._fn(*args) if v is None else self._fn_ex(*args, ctypes.byref(v))
        if rc != 0:
            raise _ffi.SkyrlHipError(f"skyrl_sample failed: {self._err().decode()}")
        return self.tokens[t], self.logprobs[t]


def _top_p(p: SamplingParams) -> float:
    return 1.0 if p.top_p is None else float(p.top_p)


def sample(logits: torch.Tensor, params: Optional[SamplingParams] = None, seed: int = 0,
           seq_ids: Optional[torch.Tensor] = None, step: int = 0):
    """One-shot sampling of [nseq, V] logits with reference SamplingParams semantics."""
    p = params or SamplingParams()
    return ops.sample(logits, temperature=p.temperature, top_k=p.top_k if p.top_k is not None else -1,
                      top_p=_top_p(p), min_p=p.min_p or 0.0, seed=seed, seq_ids=seq_ids, step=step)
