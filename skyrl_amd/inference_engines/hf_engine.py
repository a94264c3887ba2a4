"""Rollout engine for any HF causal LM: the HF forward with its own KV cache, HIP sampler.

The reference's fallback path for models vLLM does not serve is HFModelWrapper.generate
(skyrl-train/skyrl_train/model_wrapper.py:185-218: `model.generate(do_sample=True,
temperature, top_k, top_p, min_p, min_new_tokens, eos/pad ids)`). This engine keeps that
structure -- one left-padded batch, the HF model's own forward and past_key_values per decode
step -- and replaces HF's sampling with the HIP sampler (skyrl_sample, a1), so the
architectures the paged engine (PagedDecoder: Qwen2/Llama) does not cover, e.g. GPT-2
(BASELINE config 1), roll out through the same sampler, sampling keys, stop rules and
InferenceEngineInterface surface as AMDInferenceEngine:

  * request keys: (seed-derived or running id) << 20 | response position, sampler step 0;
  * stop: eos (unless ignore_eos), stop_token_ids, max_tokens; stop ids suppressed below
    min_tokens; finish reasons "stop" / "length";
  * rollout logprobs: the sampled token's logprob on the unscaled logits (vLLM semantics).
"""

from __future__ import annotations

import asyncio
from typing import Any, Dict, List, Optional

import torch

from .base import InferenceEngineInput, InferenceEngineInterface, InferenceEngineOutput
from .engine import RequestParams

_POS_BITS = 20


class HFGenerateEngine(InferenceEngineInterface):
    """One engine on one GPU over a HF ``AutoModelForCausalLM`` (bf16 rollout copy)."""

    def __init__(self, model, eos_token_id: Optional[int] = None, pad_token_id: int = 0, seed: int = 0,
                 max_num_seqs: int = 256, tokenizer=None):
        self.model = model.eval().requires_grad_(False)
        self.device = next(model.parameters()).device
        self.eos_token_id = eos_token_id if eos_token_id is not None else getattr(model.config, "eos_token_id", None)
        self.pad_token_id = int(pad_token_id)
        self.seed = int(seed)
        self.max_num_seqs = int(max_num_seqs)
        self.tokenizer = tokenizer
        self._next_rid = 0
        self._ws = None
        self._receiver = None
        self._lock = asyncio.Lock()

    # ---------------------------------------------------------------- generation
    def _keys(self, n: int, params: RequestParams) -> List[int]:
        keys = []
        for _ in range(n):
            rid = self._next_rid
            self._next_rid += 1
            keys.append((int(params.seed) & ((1 << 42) - 1)) | (1 << 42) if params.seed is not None else rid)
        return keys

    @torch.no_grad()
    def _generate_batch(self, prompts: List[List[int]], params: RequestParams, keys: List[int]):
        from .. import _ffi
        from ..ops import _ptr, _stream

        dev = self.device
        n = len(prompts)
        L = max(len(p) for p in prompts)
        ids = torch.full((n, L), self.pad_token_id, dtype=torch.int64)
        att = torch.zeros((n, L), dtype=torch.int64)
        for i, p in enumerate(prompts):  # left padding, as HF generate expects
            ids[i, L - len(p):] = torch.tensor(p, dtype=torch.int64)
            att[i, L - len(p):] = 1
        ids, att = ids.to(dev), att.to(dev)
        pos = (att.cumsum(-1) - 1).clamp(min=0)
        out = self.model(input_ids=ids, attention_mask=att, position_ids=pos, use_cache=True)
        past = out.past_key_values
        logits = out.logits[:, -1]
        V = logits.shape[-1]
        ws_bytes = int(_ffi.query("skyrl_sample_workspace_bytes", n, V))
        if self._ws is None or self._ws.numel() < ws_bytes:
            self._ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=dev)
        key_base = torch.tensor(keys, dtype=torch.int64) << _POS_BITS
        tok_d = torch.empty(n, dtype=torch.int32, device=dev)
        lp_d = torch.empty(n, dtype=torch.float32, device=dev)
        stop_ids = set(params.stop_token_ids)
        if self.eos_token_id is not None and not params.ignore_eos:
            stop_ids.add(int(self.eos_token_id))
        out_tok: List[List[int]] = [[] for _ in range(n)]
        out_lp: List[List[float]] = [[] for _ in range(n)]
        reasons: List[Optional[str]] = [None] * n
        last_pos = pos[:, -1:]
        for t in range(params.max_tokens):
            lg = logits.to(torch.bfloat16).contiguous()
            if t < params.min_tokens and stop_ids:
                lg[:, sorted(stop_ids)] = float("-inf")
            keys_d = (key_base | t).to(dev)
            _ffi.call("skyrl_sample", _ptr(lg), _ffi.BF16, lg.stride(0), n, V, float(params.temperature),
                      int(params.top_k), float(params.top_p), float(params.min_p), self.seed & 0xFFFFFFFFFFFFFFFF,
                      _ptr(keys_d), 0, _ptr(tok_d), _ptr(lp_d), _ptr(self._ws), _stream(dev))
            toks, lps = tok_d.tolist(), lp_d.tolist()
            for i in range(n):
                if reasons[i] is not None:
                    continue
                out_tok[i].append(toks[i])
                out_lp[i].append(lps[i])
                k = len(out_tok[i])
                if k >= params.min_tokens and toks[i] in stop_ids:
                    reasons[i] = "stop"
                elif k >= params.max_tokens:
                    reasons[i] = "length"
            if all(r is not None for r in reasons):
                break
            nxt = tok_d.to(torch.int64).unsqueeze(1)
            att = torch.cat([att, torch.ones((n, 1), dtype=att.dtype, device=dev)], 1)
            last_pos = last_pos + 1
            out = self.model(input_ids=nxt, attention_mask=att, position_ids=last_pos, past_key_values=past,
                             use_cache=True)
            past = out.past_key_values
            logits = out.logits[:, -1]
        return out_tok, out_lp, reasons

    def _text(self, toks: List[int]) -> str:
        if self.tokenizer is None:
            return ""
        return self.tokenizer.decode(toks, skip_special_tokens=True)

    async def generate(self, input_batch: InferenceEngineInput) -> InferenceEngineOutput:
        ids = input_batch.get("prompt_token_ids")
        if input_batch.get("prompts") is not None or ids is None:
            raise ValueError("HFGenerateEngine only accepts `prompt_token_ids`, not `prompts`")
        params = RequestParams.from_dict(input_batch.get("sampling_params"))
        if params.stop:
            raise ValueError("stop strings are served by AMDInferenceEngine (it detokenizes incrementally)")
        toks, lps, reasons = [], [], []
        async with self._lock:
            for s in range(0, len(ids), self.max_num_seqs):
                chunk = [list(p) for p in ids[s:s + self.max_num_seqs]]
                t, lp, r = self._generate_batch(chunk, params, self._keys(len(chunk), params))
                toks += t
                lps += lp
                reasons += r
        return InferenceEngineOutput(responses=[self._text(t) for t in toks], response_ids=toks, stop_reasons=reasons,
                                     response_logprobs=lps if params.logprobs is not None else None)

    async def abort_generation(self) -> None:
        return None  # batches run to completion inside one generate call

    async def chat_completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("OpenAI HTTP endpoints are out of scope")

    async def completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("OpenAI HTTP endpoints are out of scope")

    async def wake_up(self, *args: Any, **kwargs: Any):
        return None

    async def sleep(self, *args: Any, **kwargs: Any):
        return None

    # ---------------------------------------------------------------- weights
    async def init_weight_update_communicator(self, init_info):
        if hasattr(init_info, "receive_weights"):
            self._receiver = init_info
        else:
            from ..comm import BroadcastWeightReceiver

            info = dict(init_info or {})
            dtype = next(self.model.parameters()).dtype
            self._receiver = BroadcastWeightReceiver(dtype, group=info.get("group"), src=info.get("src", 0),
                                                     device=self.device)

    async def update_named_weights(self, request):
        """Copies each named tensor into the model's parameter of the same HF name."""
        tensors = request.get("tensors") if isinstance(request, dict) else getattr(request, "tensors", None)
        names = request["names"] if isinstance(request, dict) else request.names
        pairs = zip(names, tensors) if tensors is not None else self._receiver.receive_weights(request)
        params = dict(self.model.named_parameters())
        n = 0
        with torch.no_grad():
            for name, t in pairs:
                if name not in params:
                    raise KeyError(f"unknown parameter {name!r}")
                params[name].copy_(t.to(params[name].dtype))
                n += 1
        return n

    async def reset_prefix_cache(self):
        return None

    async def teardown(self):
        return None

    def tp_size(self) -> int:
        return 1

    def pp_size(self) -> int:
        return 1

    def dp_size(self) -> int:
        return 1
