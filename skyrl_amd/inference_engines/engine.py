"""MI355X rollout engine: continuous batching over a paged KV cache, behind the reference's
InferenceEngineInterface.

Replaces vLLM inside the reference's VLLMInferenceEngine / AsyncVLLMInferenceEngine
(skyrl_train/inference_engines/vllm/vllm_engine.py): same request/response types
(base.py), vLLM SamplingParams keys (as built by get_vllm_sampling_params,
inference_engines/utils.py:15-42), finish reasons "stop" / "length" / "abort", and the
abort semantics pause_generation relies on (inference_engine_client.py:597-628: an aborted
request returns the tokens generated so far with stop_reason "abort").

Layers:
  * EngineCore — scheduler: waiting/running queues, block allocation with recompute
    preemption, stop conditions. Pure host logic over a runner interface (CPU-testable).
  * ModelRunner — builds the device inputs of one scheduled batch, runs PagedDecoder
    (prefill or decode) and the HIP sampler (skyrl_sample), returns tokens/logprobs.
  * AMDInferenceEngine — the async InferenceEngineInterface: generate/sample, abort,
    sleep/wake_up, weight updates (WeightUpdateRequest + receiver, or named tensors).

Sampling keys: the sampler draws its noise from (seed, key, step); the engine passes
key = (request key << 20) | response position and step 0, so a request's tokens depend
only on its own seed/position and logits — not on which other requests share the batch.
"""

from __future__ import annotations

import asyncio
import collections
import dataclasses
import heapq
import itertools
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .base import InferenceEngineInput, InferenceEngineInterface, InferenceEngineOutput

BLOCK_SIZE = 16
_POS_BITS = 20

WAITING, RUNNING, FINISHED = 0, 1, 2


@dataclass
class RequestParams:
    """Per-request vLLM SamplingParams subset the engine honours (vllm_engine.py:118-124)."""

    max_tokens: int = 16
    min_tokens: int = 0
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    min_p: float = 0.0
    logprobs: Optional[int] = None
    stop_token_ids: Tuple[int, ...] = ()
    stop: Tuple[str, ...] = ()  # stop strings (need the engine's tokenizer), kept in the output text
    ignore_eos: bool = False
    seed: Optional[int] = None
    n: int = 1
    # vLLM penalties (additional_kwargs / the Hydra sampling_params keys): repetition divides positive
    # (multiplies negative) logits of tokens in prompt + output; presence / frequency subtract
    # presence * [count > 0] + frequency * count for output tokens. Returned logprobs stay raw
    # (vLLM's default logprobs_mode): log_softmax of the unpenalized logits.
    repetition_penalty: float = 1.0
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0

    _ACCEPTED_NOOP = ("skip_special_tokens", "include_stop_str_in_output", "spaces_between_special_tokens",
                      "detokenize", "max_completion_tokens")

    @classmethod
    def from_dict(cls, d: Optional[Dict[str, Any]]) -> "RequestParams":
        d = dict(d or {})
        p = cls()
        if "max_completion_tokens" in d and "max_tokens" not in d:
            d["max_tokens"] = d["max_completion_tokens"]
        for k, v in d.items():
            if k in ("max_tokens", "min_tokens", "top_k", "seed", "logprobs", "n"):
                if v is not None:
                    setattr(p, k, int(v))
                elif k in ("logprobs", "seed"):
                    setattr(p, k, None)
            elif k in ("temperature", "top_p", "min_p", "repetition_penalty", "presence_penalty",
                       "frequency_penalty"):
                setattr(p, k, float(v) if v is not None else getattr(cls, k))
            elif k == "stop_token_ids":
                p.stop_token_ids = tuple(int(x) for x in (v or ()))
            elif k == "ignore_eos":
                p.ignore_eos = bool(v)
            elif k == "stop":
                p.stop = tuple([v] if isinstance(v, str) else (v or ()))
            elif k in cls._ACCEPTED_NOOP:
                continue
            else:
                raise ValueError(f"unsupported sampling parameter {k!r}")
        if p.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if p.n is None or p.n < 1:
            raise ValueError("n must be >= 1")
        if p.repetition_penalty <= 0:
            raise ValueError("repetition_penalty must be > 0")
        for k in ("presence_penalty", "frequency_penalty"):
            if not -2.0 <= getattr(p, k) <= 2.0:
                raise ValueError(f"{k} must be in [-2, 2]")
        if p.temperature < 0:
            raise ValueError("temperature must be >= 0")
        return p

    def sampler_key(self) -> Tuple[float, int, float, float]:
        return (self.temperature, self.top_k, self.top_p, self.min_p)

    def has_penalty(self) -> bool:
        return self.repetition_penalty != 1.0 or self.presence_penalty != 0.0 or self.frequency_penalty != 0.0


@dataclass
class Request:
    rid: int
    prompt: List[int]
    params: RequestParams
    key: int
    out_tokens: List[int] = field(default_factory=list)
    out_logprobs: List[float] = field(default_factory=list)
    blocks: List[int] = field(default_factory=list)
    state: int = WAITING
    row: int = -1  # persistent batch row while running (the runner's per-row device state)
    num_cached: int = 0  # leading tokens whose K/V came from the prefix cache at admission
    block_hashes: List[int] = field(default_factory=list)
    finish_reason: Optional[str] = None
    on_finish: Optional[Callable[["Request"], None]] = None

    @property
    def num_tokens(self) -> int:
        return len(self.prompt) + len(self.out_tokens)


class BlockAllocator:
    """Reference-counted KV-cache blocks with an optional prefix cache.

    Plain blocks return to a LIFO free list when their last user releases them. With prefix
    caching, a full block of a prefill input is registered under the chain hash of its tokens
    (hash of the previous block's hash and its 16 ids); when released it stays resident and
    evictable (LRU) so a later request with the same prefix can share it read-only — vLLM's
    automatic prefix caching (enable_prefix_caching, ppo_base_config.yaml generator section),
    which GRPO's n_samples_per_prompt identical prompts hit."""

    def __init__(self, num_blocks: int, enable_caching: bool = False):
        self.num_blocks = num_blocks
        self.enable_caching = enable_caching
        self._free: List[int] = list(range(num_blocks - 1, -1, -1))
        self._ref = [0] * num_blocks
        self._hash_of: Dict[int, int] = {}
        self._by_hash: Dict[int, int] = {}
        self._evictable: "collections.OrderedDict[int, None]" = collections.OrderedDict()
        self.hits = 0

    @property
    def num_free(self) -> int:
        return len(self._free) + len(self._evictable)

    def allocate(self, n: int) -> List[int]:
        if n > self.num_free:
            raise RuntimeError("out of KV-cache blocks")
        out = []
        for _ in range(n):
            if self._free:
                b = self._free.pop()
            else:  # evict the least recently released cached block
                b, _ = self._evictable.popitem(last=False)
                del self._by_hash[self._hash_of.pop(b)]
            self._ref[b] = 1
            out.append(b)
        return out

    def free(self, blocks: Iterable[int]) -> None:
        for b in reversed(list(blocks)):
            self._ref[b] -= 1
            if self._ref[b] == 0:
                if b in self._hash_of:
                    self._evictable[b] = None
                else:
                    self._free.append(b)

    # ---- prefix cache
    def lookup(self, h: int) -> Optional[int]:
        return self._by_hash.get(h)

    def acquire(self, b: int) -> None:
        """Take a reference on a cached block (found by lookup)."""
        if self._ref[b] == 0:
            del self._evictable[b]
        self._ref[b] += 1
        self.hits += 1

    def register(self, b: int, h: int) -> None:
        if self.enable_caching and h not in self._by_hash and b not in self._hash_of:
            self._by_hash[h] = b
            self._hash_of[b] = h

    def reset(self) -> None:
        """Forget every cached prefix (after a weight update the cached K/V are stale)."""
        for b in self._evictable:
            self._free.append(b)
        self._evictable.clear()
        self._hash_of.clear()
        self._by_hash.clear()


def block_hashes(tokens: Sequence[int], nblocks: int) -> List[int]:
    """Chain hashes of the first `nblocks` full 16-token blocks."""
    out, h = [], 0
    for i in range(nblocks):
        h = hash((h, tuple(tokens[i * BLOCK_SIZE:(i + 1) * BLOCK_SIZE])))
        out.append(h)
    return out


@dataclass
class ScheduledBatch:
    kind: str                       # "prefill" | "decode"
    requests: List[Request]
    # per request: (temperature, top_k, top_p, min_p), sampler key, mask-stop flag
    keys: np.ndarray                # int64 [n]: (key << 20) | response position
    suppress: List[Tuple[int, ...]]  # stop ids to mask (min_tokens not reached), per request


def _blocks_needed(num_tokens: int) -> int:
    return (num_tokens + BLOCK_SIZE - 1) // BLOCK_SIZE


class EngineCore:
    """Scheduler over a runner with `execute(batch) -> (tokens int64 [n], logprobs f32 [n])`."""

    def __init__(self, runner, num_blocks: int, max_num_seqs: int = 512, max_model_len: int = 4096,
                 max_prefill_tokens: int = 32768, eos_token_id: Optional[int] = None, seed: int = 0,
                 detokenize: Optional[Callable[[List[int]], str]] = None, enable_prefix_caching: bool = False):
        self.runner = runner
        self.detokenize = detokenize  # stop strings are matched on the decoded tail of the output
        self.allocator = BlockAllocator(num_blocks, enable_caching=enable_prefix_caching)
        self.max_num_seqs = max_num_seqs
        self.max_model_len = max_model_len
        self.max_prefill_tokens = max_prefill_tokens
        self.eos_token_id = eos_token_id
        self.seed = seed
        self.waiting: Deque[Request] = collections.deque()
        self.running: List[Request] = []
        self._rid = itertools.count()
        self._free_rows = list(range(max_num_seqs))  # lowest row first: keeps the batch compact
        self.num_preemptions = 0
        self.num_steps = 0
        self.stats: Dict[str, float] = collections.defaultdict(float)  # per-kind step counts and seconds

    # ---------------------------------------------------------------- requests
    def add_request(self, prompt: Sequence[int], params: RequestParams,
                    on_finish: Optional[Callable[[Request], None]] = None) -> Request:
        prompt = [int(t) for t in prompt]
        if len(prompt) == 0:
            raise ValueError("empty prompt")
        if len(prompt) + 1 > self.max_model_len:
            raise ValueError(f"prompt of {len(prompt)} tokens exceeds max_model_len={self.max_model_len}")
        if _blocks_needed(len(prompt) + 1) > self.allocator.num_blocks:
            raise ValueError("prompt does not fit in the KV cache")
        if params.stop and self.detokenize is None:
            raise ValueError("string stop sequences need the engine's tokenizer; pass stop_token_ids instead")
        rid = next(self._rid)
        key = (int(params.seed) & ((1 << 42) - 1)) | (1 << 42) if params.seed is not None else rid
        req = Request(rid=rid, prompt=prompt, params=params, key=key, on_finish=on_finish)
        self.waiting.append(req)
        return req

    def has_unfinished(self) -> bool:
        return bool(self.waiting or self.running)

    def abort_all(self) -> List[Request]:
        """Finish every waiting and running request with stop_reason "abort"."""
        done = []
        for r in list(self.running) + list(self.waiting):
            self._finish(r, "abort")
            done.append(r)
        self.running.clear()
        self.waiting.clear()
        return done

    def abort(self, rids: Iterable[int]) -> List[Request]:
        rids = set(rids)
        done = [r for r in list(self.running) + list(self.waiting) if r.rid in rids]
        for r in done:
            self._finish(r, "abort")
        self.running = [r for r in self.running if r.rid not in rids]
        self.waiting = collections.deque(r for r in self.waiting if r.rid not in rids)
        return done

    def _finish(self, r: Request, reason: str) -> None:
        if r.blocks:
            self.allocator.free(r.blocks)
            r.blocks = []
        self._release_row(r)
        r.state = FINISHED
        r.finish_reason = reason
        if r.on_finish is not None:
            r.on_finish(r)

    def _release_row(self, r: Request) -> None:
        if r.row >= 0:
            heapq.heappush(self._free_rows, r.row)
            r.row = -1

    # ---------------------------------------------------------------- scheduling
    def _schedule_prefill(self) -> List[Request]:
        """Admit waiting requests (FIFO) while rows, blocks and the padded-token budget last.
        With prefix caching a request takes the cached blocks of its longest cached prefix
        (never the block of its last token, which must be computed for its logits); a request
        whose next uncached block is being computed by an earlier request of this same batch
        waits one step, so the GRPO siblings of a prompt share its prefill."""
        alloc = self.allocator
        batch: List[Request] = []
        deferred: List[Request] = []
        pending = set()
        padded_max = 0
        while self.waiting and len(self.running) + len(batch) < self.max_num_seqs:
            r = self.waiting[0]
            toks = r.prompt + r.out_tokens
            n = len(toks)
            hashes = block_hashes(toks, (n - 1) // BLOCK_SIZE) if alloc.enable_caching else []
            cached = []
            for h in hashes:
                b = alloc.lookup(h)
                if b is None:
                    break
                cached.append(b)
            k = len(cached)
            if k < len(hashes) and hashes[k] in pending:
                deferred.append(self.waiting.popleft())
                continue
            lmax = max(padded_max, n - k * BLOCK_SIZE)
            if batch and lmax * (len(batch) + 1) > self.max_prefill_tokens:
                break
            need = _blocks_needed(n + 1) - k
            if need > alloc.num_free - sum(1 for b in cached if b in alloc._evictable):
                break
            self.waiting.popleft()
            for b in cached:
                alloc.acquire(b)
            r.blocks = cached + alloc.allocate(need)
            r.num_cached = k * BLOCK_SIZE
            r.block_hashes = hashes
            pending.update(hashes[k:])
            r.row = heapq.heappop(self._free_rows)
            r.state = RUNNING
            batch.append(r)
            padded_max = lmax
        self.waiting.extendleft(reversed(deferred))
        return batch

    def reset_prefix_cache(self) -> None:
        self.allocator.reset()

    def _ensure_decode_blocks(self) -> None:
        """Every running request needs the block holding position num_tokens-1; preempt the most
        recently admitted requests (recompute later) while blocks run out."""
        i = 0
        while i < len(self.running):
            r = self.running[i]
            need = _blocks_needed(r.num_tokens)
            if need <= len(r.blocks):
                i += 1
                continue
            if self.allocator.num_free > 0:
                r.blocks.extend(self.allocator.allocate(need - len(r.blocks)))
                i += 1
                continue
            victim = self.running.pop()
            self.allocator.free(victim.blocks)
            victim.blocks = []
            self._release_row(victim)
            victim.state = WAITING
            self.waiting.appendleft(victim)
            self.num_preemptions += 1
            if victim is r:
                continue  # r itself was preempted; index i now points past the end or at the next
        if not self.running and self.waiting and not self.allocator.num_free:
            raise RuntimeError("KV cache too small for a single request")

    def _keys_and_masks(self, reqs: List[Request]) -> Tuple[np.ndarray, List[Tuple[int, ...]]]:
        keys = np.fromiter(((r.key << _POS_BITS) | len(r.out_tokens) for r in reqs), dtype=np.int64,
                           count=len(reqs))
        sup = []
        for r in reqs:
            p = r.params
            if len(r.out_tokens) < p.min_tokens:
                ids = set(p.stop_token_ids)
                if self.eos_token_id is not None and not p.ignore_eos:
                    ids.add(self.eos_token_id)
                sup.append(tuple(sorted(ids)))
            else:
                sup.append(())
        return keys, sup

    def step(self) -> List[Request]:
        """Run one prefill or decode step; returns the requests that finished in it."""
        self.num_steps += 1
        batch = self._schedule_prefill()
        kind = "prefill"
        if not batch:
            self._ensure_decode_blocks()
            batch = list(self.running)
            kind = "decode"
            if not batch:
                return []
        t0 = time.perf_counter()
        keys, sup = self._keys_and_masks(batch)
        t1 = time.perf_counter()
        tokens, logprobs = self.runner.execute(ScheduledBatch(kind, batch, keys, sup))
        t2 = time.perf_counter()
        if kind == "prefill":
            self.running.extend(batch)
            for r in batch:  # the full blocks this prefill computed are now shareable
                for i in range(r.num_cached // BLOCK_SIZE, len(r.block_hashes)):
                    self.allocator.register(r.blocks[i], r.block_hashes[i])
        finished: List[Request] = []
        for r, t, lp in zip(batch, tokens.tolist(), logprobs.tolist()):
            r.out_tokens.append(t)
            r.out_logprobs.append(lp)
            reason = self._stop_reason(r, t)
            if reason is not None:
                finished.append(r)
                self._finish(r, reason)
        if finished:
            done = {id(r) for r in finished}
            self.running = [r for r in self.running if id(r) not in done]
        st = self.stats
        st[kind + "_steps"] += 1
        st[kind + "_exec_s"] += t2 - t1
        st[kind + "_host_s"] += (t1 - t0) + (time.perf_counter() - t2)
        return finished

    def _stop_reason(self, r: Request, tok: int) -> Optional[str]:
        p = r.params
        n = len(r.out_tokens)
        if n >= p.min_tokens:
            if tok in p.stop_token_ids:
                return "stop"
            if not p.ignore_eos and self.eos_token_id is not None and tok == self.eos_token_id:
                return "stop"
            if p.stop:  # a token covers >= 1 character: the last max-len tokens hold any new match
                tail = self.detokenize(r.out_tokens[-(max(len(s) for s in p.stop) + 1):])
                if any(s in tail for s in p.stop):
                    return "stop"
        if n >= p.max_tokens or r.num_tokens >= self.max_model_len:
            return "length"
        return None


class ModelRunner:
    """Device side of one scheduled batch: PagedDecoder forward + lm_head + HIP sampler.

    Decode runs over the persistent batch rows [0, nb) (nb = the smallest bucket >= 1 + the
    highest running row): per-row inputs (token, position, slot, context length, block-table
    row) are staged in pinned host buffers and copied with two H2D copies into static device
    buffers, and the forward + lm_head of bucket nb is a captured HIP graph replayed per step
    (one launch instead of ~10 per layer from Python). Idle rows feed token 0 at position 0
    with slot -1 (no cache write) and context 1. Prefill runs eagerly (ragged shapes)."""

    BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 192, 256, 384, 512, 768, 1024)

    def __init__(self, model, num_blocks: int, max_num_seqs: int, seed: int = 0, use_graphs: bool = True,
                 tunable_gemm: Optional[str] = None, fused_lmhead: str = "auto"):
        # tunable_gemm: a results-file path enables PyTorch TunableOp (runtime GEMM solution search)
        # around this runner's forwards only; the decode buckets' skinny GEMMs gain most (measured
        # 3.28 -> 2.32 ms per 28-layer decode step at 8 rows, `scripts/probe/tunable_probe.py`).
        self.tunable_gemm = tunable_gemm
        # fused_lmhead: when the lm_head GEMM runs with the sampler in its epilogue
        # (skyrl_lmhead_sample, csrc/lmhead_gemm.hip; no [n, V] logits in HBM) instead of a library
        # GEMM + skyrl_sample. "auto" (default; "greedy" is its older name): unfiltered
        # single-parameter batches without penalties or suppressed ids where the fused kernel
        # measured faster (greedy at >= 192 or <= 16 rows, T > 0 at >= 480 rows; see _fused_ok and
        # profiles/r02_lmhead_sample_bench.json); "always": every unfiltered single-parameter
        # batch; "off". Under "auto" a request's logits come from either GEMM depending on how many
        # rows share its step. Both round fp32 sums to bf16 and agree within one bf16 rounding,
        # argmax included wherever the top-2 margin exceeds it
        # (tests/test_gpu_engine.py::test_lmhead_gemm_vs_flinear_logits_and_argmax); a run that
        # must not depend on batch composition at all (seeded evaluation) sets "off" or "always".
        if fused_lmhead == "greedy":  # the r02 name of "auto"
            fused_lmhead = "auto"
        if fused_lmhead not in ("auto", "always", "off"):
            raise ValueError(f"fused_lmhead must be 'auto', 'always' or 'off', got {fused_lmhead!r}")
        fits = model.spec.hidden_size % 64 == 0 and str(getattr(model, "dtype", "")) == "torch.bfloat16"
        self.fused_lmhead = fused_lmhead if fits else "off"
        self.fused_steps = 0  # decode/prefill steps sampled by the fused kernel
        self._last_nb = 0
        import torch

        self.torch = torch
        self.model = model
        self.device = model.device
        self.seed = int(seed)
        self.num_blocks = num_blocks
        self.max_num_seqs = max_num_seqs
        self.max_blocks = _blocks_needed(model.max_model_len)
        self.use_graphs = use_graphs
        self.buckets = [b for b in self.BUCKETS if b < max_num_seqs] + [max_num_seqs]
        self.cache = None
        R = max_num_seqs
        pin = torch.cuda.is_available()
        self.h_i64 = torch.zeros((3, R), dtype=torch.int64, pin_memory=pin)       # token | position | slot
        self.h_i32 = torch.zeros((R, self.max_blocks), dtype=torch.int32, pin_memory=pin)  # block tables
        self.h_ctx = torch.zeros(R, dtype=torch.int32, pin_memory=pin)
        self.h_keys = torch.zeros(R, dtype=torch.int64, pin_memory=pin)
        self.n_i64, self.n_i32, self.n_keys = self.h_i64.numpy(), self.h_i32.numpy(), self.h_keys.numpy()
        self.n_ctx = self.h_ctx.numpy()
        self.d_i64 = torch.zeros((3, R), dtype=torch.int64, device=self.device)
        self.d_i32 = torch.zeros((R, self.max_blocks), dtype=torch.int32, device=self.device)
        self.d_ctx = torch.ones(R, dtype=torch.int32, device=self.device)
        self.d_keys = torch.zeros(R, dtype=torch.int64, device=self.device)
        self.tokens = torch.empty(R, dtype=torch.int32, device=self.device)
        self.lps = torch.empty(R, dtype=torch.float32, device=self.device)
        self.h_out = torch.zeros((2, R), dtype=torch.float64, pin_memory=pin)
        self._nblk = np.zeros(R, dtype=np.int64)  # table entries already staged per row
        self._graphs: Dict[int, Tuple[Any, Any]] = {}
        self._pool = None
        self._sampler_ws = None
        self.ensure_cache(num_blocks)

    # ---------------------------------------------------------------- memory
    def release_cache(self):
        self._graphs.clear()
        self._pool = None
        self.cache = None

    def ensure_cache(self, num_blocks: int):
        if self.cache is None:
            from .model import PagedKVCache

            s = self.model.spec
            self.cache = PagedKVCache(s.num_layers, num_blocks, s.num_kv_heads, s.head_dim, self.device)
            self._graphs.clear()

    def drop_graphs(self):
        """Weights were re-allocated (sleep level 2 / wake_up): captured graphs point at the old storage."""
        self._graphs.clear()
        self._pool = None

    def _h2d(self, arr: np.ndarray):
        return self.torch.from_numpy(arr).pin_memory().to(self.device, non_blocking=True)

    # ---------------------------------------------------------------- decode inputs
    def _decode_inputs(self, nb: int, fixed: bool):
        from .model import StepInputs

        nparts = max_ctx = None
        if fixed:  # graph: the wave count is baked into the launch (the split adapts on device)
            from . import kernels

            max_ctx = self.model.max_model_len
            nparts = kernels.choose_nparts(nb, self.model.spec.num_kv_heads, max_ctx)
        return StepInputs(tokens=self.d_i64[0, :nb], positions=self.d_i64[1, :nb], slots=self.d_i64[2, :nb],
                          block_tables=self.d_i32[:nb], context_lens=self.d_ctx[:nb], max_ctx=max_ctx or 0,
                          nparts=nparts)

    def _forward_hidden(self, inp):
        return self.model.forward_decode(inp, self.cache)

    def _graph(self, nb: int):
        g = self._graphs.get(nb)
        if g is not None:
            return g
        torch = self.torch
        from . import kernels

        s = self.model.spec
        need = 0  # pre-size the merge workspace for every bucket: a graph must never see it move
        for b in self.buckets:
            nparts = kernels.choose_nparts(b, s.num_kv_heads, self.model.max_model_len)
            need = max(need, _decode_ws_bytes(b, s.num_heads, s.head_dim, nparts))
        self.model.workspace.get(need)
        inp = self._decode_inputs(nb, fixed=True)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self._forward_hidden(inp)  # warm-up outside capture (library handles, workspaces)
        torch.cuda.current_stream(self.device).wait_stream(side)
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self._pool):
            hidden = self._forward_hidden(inp)
        self._graphs[nb] = (graph, hidden)
        return self._graphs[nb]

    def _stage_decode(self, reqs: List["Request"], nb: int) -> None:
        n_i64, n_i32, n_ctx = self.n_i64, self.n_i32, self.n_ctx
        n_i64[:, :nb] = 0
        n_i64[2, :nb] = -1
        n_ctx[:nb] = 1
        rows = np.fromiter((r.row for r in reqs), dtype=np.int64, count=len(reqs))
        L = np.fromiter((r.num_tokens for r in reqs), dtype=np.int64, count=len(reqs))
        for r in reqs:  # table rows: only newly allocated blocks are staged
            k = self._nblk[r.row]
            if len(r.blocks) != k:
                if len(r.blocks) < k:
                    k = 0
                n_i32[r.row, k:len(r.blocks)] = r.blocks[k:]
                self._nblk[r.row] = len(r.blocks)
        n_i64[0, rows] = np.fromiter((r.out_tokens[-1] for r in reqs), dtype=np.int64, count=len(reqs))
        pos = L - 1
        n_i64[1, rows] = pos
        n_i64[2, rows] = n_i32[rows, pos // BLOCK_SIZE].astype(np.int64) * BLOCK_SIZE + pos % BLOCK_SIZE
        n_ctx[rows] = L
        self.d_i64[:, :nb].copy_(self.h_i64[:, :nb], non_blocking=True)
        self.d_i32[:nb].copy_(self.h_i32[:nb], non_blocking=True)
        self.d_ctx[:nb].copy_(self.h_ctx[:nb], non_blocking=True)

    # ---------------------------------------------------------------- execute
    def execute(self, batch: ScheduledBatch):
        if not self.tunable_gemm:
            return self._execute(batch)
        tun = self.torch.cuda.tunable
        tun.set_filename(self.tunable_gemm)
        tun.enable(True)
        tun.tuning_enable(True)
        try:
            return self._execute(batch)
        finally:
            tun.enable(False)

    def _execute(self, batch: ScheduledBatch):
        torch = self.torch
        from .model import StepInputs

        reqs = batch.requests
        n = len(reqs)
        if batch.kind == "prefill":
            cached = [r.num_cached for r in reqs]  # prefix-cache hits: only the suffix is computed
            seqs = [(r.prompt + r.out_tokens)[c:] for r, c in zip(reqs, cached)]
            lens = [len(s) for s in seqs]
            tok = np.fromiter(itertools.chain.from_iterable(seqs), dtype=np.int64, count=sum(lens))
            pos = np.concatenate([np.arange(c, c + L, dtype=np.int64) for c, L in zip(cached, lens)])
            slots = np.concatenate([_slots(r.blocks, c, c + L) for r, c, L in zip(reqs, cached, lens)])
            packed = self._h2d(np.concatenate([tok, pos, slots]))
            T = tok.shape[0]
            bt = None
            if any(cached):
                width = max(len(r.blocks) for r in reqs)
                bt_np = np.zeros((n, width), dtype=np.int32)
                for i, r in enumerate(reqs):
                    bt_np[i, :len(r.blocks)] = r.blocks
                bt = self._h2d(bt_np)
            inp = StepInputs(tokens=packed[:T], positions=packed[T:2 * T], slots=packed[2 * T:], seq_lens=lens,
                             cached_lens=cached, block_tables=bt)
            hidden = self.model.forward_prefill(inp, self.cache)
            for r in reqs:
                self._nblk[r.row] = 0  # (re)admitted row: restage its whole table
            rows = np.arange(n)
        else:
            hi = 1 + max(r.row for r in reqs)
            nb = next(b for b in self.buckets if b >= hi)
            self._stage_decode(reqs, nb)
            self._last_nb = nb
            if self.use_graphs:
                graph, hidden = self._graph(nb)
                graph.replay()
            else:
                inp = self._decode_inputs(nb, fixed=False)
                inp.max_ctx = int(max(r.num_tokens for r in reqs))
                hidden = self._forward_hidden(inp)
            rows = np.fromiter((r.row for r in reqs), dtype=np.int64, count=n)
        return self._sample(hidden, batch, rows)

    def _fused_ok(self, groups, batch: ScheduledBatch) -> bool:
        if self.fused_lmhead == "off" or len(groups) != 1 or any(batch.suppress):
            return False
        if any(r.params.has_penalty() for r in batch.requests):
            return False
        temp, top_k, top_p, min_p = next(iter(groups))
        unfiltered = (top_k is None or top_k < 0) and (top_p is None or top_p >= 1.0) and not min_p
        if self.fused_lmhead == "always":
            return unfiltered
        # where the fused kernel measured faster (256 x 256 tiles waste MFMA work on mid-size
        # batches). Greedy: 143 vs 128 us at 64 rows, 143 vs 175 at 8, 248 vs 292 at 512. T > 0
        # (cross-tile row bar): 314 vs 319 us at 512 rows, 198 vs 188 at 256, so only full tiles.
        nb = len(batch.requests) if batch.kind == "prefill" else self._last_nb
        if temp == 0.0:
            return unfiltered and (nb >= 192 or nb <= 16)
        return unfiltered and nb >= 480

    def _sample(self, hidden, batch: ScheduledBatch, rows: np.ndarray):
        torch = self.torch
        from .. import _ffi, ops
        from ..ops import _ptr, _stream

        nb = hidden.shape[0]
        self.n_keys[:nb] = 0
        self.n_keys[rows] = batch.keys
        self.d_keys[:nb].copy_(self.h_keys[:nb], non_blocking=True)
        groups: Dict[Tuple, List[int]] = {}
        for r_i, r in zip(rows.tolist(), batch.requests):
            groups.setdefault(r.params.sampler_key(), []).append(r_i)
        if self._fused_ok(groups, batch):  # lm_head GEMM with the sampler in its epilogue
            temp = next(iter(groups))[0]
            ops.lmhead_sample(hidden, self.model.lm_head, temperature=float(temp), seed=self.seed,
                              seq_ids=self.d_keys[:nb], step=0, tokens_out=self.tokens[:nb], logp_out=self.lps[:nb])
            self.fused_steps += 1
            return self._fetch(nb, rows)
        logits = self.model.logits(hidden)
        V = logits.shape[1]
        pen = self._apply_penalties(logits, batch, rows)
        for r_i, ids in zip(rows.tolist(), batch.suppress):
            if ids:
                logits[r_i, list(ids)] = float("-inf")
        ws_bytes = _ffi.query("skyrl_sample_workspace_bytes", max(nb, self.max_num_seqs), V)
        if self._sampler_ws is None or self._sampler_ws.numel() < ws_bytes:
            self._sampler_ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=self.device)
        st = _stream(self.device)
        for (temp, top_k, top_p, min_p), grows in groups.items():
            if len(groups) == 1:  # every row of the bucket (idle rows are sampled and dropped)
                lg, ky, to, lo = logits, self.d_keys[:nb], self.tokens[:nb], self.lps[:nb]
            else:
                idx = torch.tensor(grows, dtype=torch.int64).to(self.device, non_blocking=True)
                lg, ky = logits.index_select(0, idx), self.d_keys.index_select(0, idx)
                to = torch.empty(len(grows), dtype=torch.int32, device=self.device)
                lo = torch.empty(len(grows), dtype=torch.float32, device=self.device)
            _ffi.call("skyrl_sample", _ptr(lg), _ffi.BF16, lg.stride(0), lg.shape[0], V, float(temp), int(top_k),
                      float(top_p), float(min_p), self.seed & 0xFFFFFFFFFFFFFFFF, _ptr(ky), 0, _ptr(to), _ptr(lo),
                      _ptr(self._sampler_ws), st)
            if len(groups) != 1:
                self.tokens.index_copy_(0, idx, to)
                self.lps.index_copy_(0, idx, lo)
        if pen is not None:  # raw logprobs of the penalized rows: restore the logits, recompute
            flat, saved, prow = pen
            logits.view(-1).index_copy_(0, flat, saved)
            x = logits.index_select(0, prow)
            lp, _ = ops.logprobs_and_entropy(x[None], self.tokens.index_select(0, prow).long()[None],
                                             compute_entropy=False)
            self.lps.index_copy_(0, prow, lp[0])
        return self._fetch(nb, rows)

    def _apply_penalties(self, logits, batch: ScheduledBatch, rows: np.ndarray):
        """vLLM's apply_penalties on the rows that ask for one (sparse: only the tokens of their
        prompt + output). Returns (flat indices, original values, rows) to restore, or None."""
        torch = self.torch
        V = logits.shape[1]
        fi, rep, add, prow = [], [], [], []
        for r_i, r in zip(rows.tolist(), batch.requests):
            p = r.params
            if not p.has_penalty():
                continue
            prow.append(r_i)
            counts = collections.Counter(r.out_tokens)
            toks = sorted(set(r.prompt) | set(counts)) if p.repetition_penalty != 1.0 else sorted(counts)
            for t in toks:
                if 0 <= t < V:
                    c = counts.get(t, 0)
                    fi.append(r_i * V + t)
                    rep.append(p.repetition_penalty)
                    add.append(-(p.frequency_penalty * c + (p.presence_penalty if c > 0 else 0.0)))
        if not prow:
            return None
        dev = self.device
        flat = torch.tensor(fi, dtype=torch.int64).to(dev, non_blocking=True)
        r = torch.tensor(rep, dtype=torch.float32).to(dev, non_blocking=True)
        a = torch.tensor(add, dtype=torch.float32).to(dev, non_blocking=True)
        saved = logits.view(-1).index_select(0, flat)
        v = saved.float()
        v = torch.where(v > 0, v / r, v * r) + a
        logits.view(-1).index_copy_(0, flat, v.to(logits.dtype))
        return flat, saved, torch.tensor(prow, dtype=torch.int64).to(dev, non_blocking=True)

    def _fetch(self, nb: int, rows: np.ndarray):
        torch = self.torch
        m = max(nb, int(rows.max()) + 1)
        out = self.h_out[:, :m]
        out[0].copy_(self.tokens[:m], non_blocking=True)
        out[1].copy_(self.lps[:m], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        o = out.numpy()
        return o[0, rows].astype(np.int64), o[1, rows].astype(np.float32)


def _decode_ws_bytes(nseq: int, nh: int, head_dim: int, nparts: int) -> int:
    from .. import _ffi

    return int(_ffi.query("skyrl_paged_decode_workspace_bytes", nseq, nh, head_dim, nparts))


def _slots(blocks: List[int], start: int, end: int) -> np.ndarray:
    p = np.arange(start, end, dtype=np.int64)
    b = np.asarray(blocks, dtype=np.int64)
    return b[p // BLOCK_SIZE] * BLOCK_SIZE + p % BLOCK_SIZE


class AMDInferenceEngine(InferenceEngineInterface):
    """One rollout engine on one GPU (tp = pp = dp = 1), asyncio-driven.

    `model` is a PagedDecoder; `num_blocks` sizes the KV cache (default: ``kv_cache_fraction``
    of the free HBM after weights). Decoding runs in a background task while any request is
    unfinished; each step is one prefill or decode batch of every running request."""

    def __init__(self, model, num_blocks: Optional[int] = None, max_num_seqs: int = 512,
                 max_prefill_tokens: int = 32768, seed: int = 0, kv_cache_fraction: float = 0.5,
                 tokenizer=None, runner=None, use_graphs: bool = True, enable_prefix_caching: bool = True,
                 tunable_gemm: Optional[str] = None, fused_lmhead: str = "auto"):
        self.model = model
        self.tokenizer = tokenizer
        if num_blocks is None:
            import torch

            from .model import PagedKVCache

            free, _ = torch.cuda.mem_get_info(model.device)
            s = model.spec
            num_blocks = int(free * kv_cache_fraction) // PagedKVCache.bytes_per_block(
                s.num_layers, s.num_kv_heads, s.head_dim)
        self.num_blocks = num_blocks
        self.runner = runner if runner is not None else ModelRunner(model, num_blocks, max_num_seqs, seed,
                                                                         use_graphs=use_graphs,
                                                                         tunable_gemm=tunable_gemm,
                                                                         fused_lmhead=fused_lmhead)
        self.core = EngineCore(self.runner, num_blocks, max_num_seqs=max_num_seqs,
                               max_model_len=model.max_model_len, max_prefill_tokens=max_prefill_tokens,
                               eos_token_id=model.spec.eos_token_id, seed=seed,
                               detokenize=(lambda ids: tokenizer.decode(ids, skip_special_tokens=True))
                               if tokenizer is not None else None,
                               enable_prefix_caching=enable_prefix_caching)
        self._task: Optional[asyncio.Task] = None
        self._futures: Dict[int, asyncio.Future] = {}
        self._receiver = None
        self._offloaded = None

    # ---------------------------------------------------------------- generation
    def _decode_text(self, r: Request) -> str:
        if self.tokenizer is None:
            return ""
        text = self.tokenizer.decode(r.out_tokens, skip_special_tokens=True)
        if r.finish_reason == "stop" and r.params.stop and r.out_tokens:
            # include_stop_str_in_output: cut after the stop string the last token completed
            # (vLLM searches only the newly added characters plus one stop length back)
            new = len(self.tokenizer.decode(r.out_tokens[-1:], skip_special_tokens=True))
            for s in r.params.stop:
                i = text.find(s, max(0, len(text) - new - len(s)))
                if i >= 0:
                    return text[:i + len(s)]
        return text

    def _submit(self, prompt: List[int], params: RequestParams) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()

        def done(r: Request, fut=fut):
            self._futures.pop(r.rid, None)
            if not fut.done():
                fut.set_result(r)

        req = self.core.add_request(prompt, params, on_finish=done)
        self._futures[req.rid] = fut
        if self._task is None or self._task.done() or self._task.get_loop() is not loop:  # (a previous asyncio.run's loop)
            self._task = loop.create_task(self._run())
        return fut

    async def _run(self):
        try:
            while self.core.has_unfinished():
                self.core.step()
                await asyncio.sleep(0)
        except BaseException as e:  # fail every pending request instead of hanging it
            for fut in list(self._futures.values()):
                if not fut.done():
                    fut.set_exception(e)
            self._futures.clear()
            self.core.abort_all()
            raise

    def _output(self, reqs: List[Request], want_logprobs: bool) -> InferenceEngineOutput:
        return InferenceEngineOutput(
            responses=[self._decode_text(r) for r in reqs],
            stop_reasons=[r.finish_reason for r in reqs],
            response_ids=[list(r.out_tokens) for r in reqs],
            response_logprobs=[list(r.out_logprobs) for r in reqs] if want_logprobs else None,
        )

    async def generate(self, input_batch: InferenceEngineInput) -> InferenceEngineOutput:
        prompts = input_batch.get("prompts")
        ids = input_batch.get("prompt_token_ids")
        if prompts is not None or ids is None:
            raise ValueError("AMDInferenceEngine only accepts `prompt_token_ids`, not `prompts` "
                             "(vllm_engine.py:112-114)")
        params = RequestParams.from_dict(input_batch.get("sampling_params"))
        if params.n > 1:
            # n samples per prompt, prompt-major in the output (the reference copies prompts instead:
            # vllm_engine.py:133-136); a seeded request's j-th sample uses seed + j, as vLLM's
            # parallel sampling does
            subs = []
            for j in range(params.n):
                pj = dataclasses.replace(params, n=1, seed=None if params.seed is None else params.seed + j)
                subs.append(pj)
            futs = [self._submit(p, subs[j]) for p in ids for j in range(params.n)]
        else:
            futs = [self._submit(p, params) for p in ids]
        reqs = await asyncio.gather(*futs)
        return self._output(list(reqs), params.logprobs is not None)

    async def sample(self, prompt_token_ids: List[int], num_samples: int,
                     sampling_params: Dict[str, Any]) -> InferenceEngineOutput:
        """All num_samples requests go into the batch at once (independent keys per request)."""
        return await self.generate({"prompt_token_ids": [list(prompt_token_ids)] * num_samples,
                                    "sampling_params": sampling_params})

    async def abort_generation(self) -> None:
        self.core.abort_all()

    async def chat_completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("OpenAI HTTP endpoints are out of scope for the MI355X engine")

    async def completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("OpenAI HTTP endpoints are out of scope for the MI355X engine")

    # ---------------------------------------------------------------- memory
    async def sleep(self, *args: Any, **kwargs: Any):
        """level 1: offload weights to host and free the KV cache; level 2: discard weights too
        (they come back through update_named_weights) — vllm_engine.py sleep()."""
        if self.core.has_unfinished():
            self.core.abort_all()
        level = kwargs.get("level", 2)
        self.runner.release_cache()
        self.core.reset_prefix_cache()
        if level == 1:
            self._offloaded = [(n, t.detach().to("cpu")) for n, t in self.model.hf_named_tensors()]
        self.model.release()

    async def wake_up(self, *args: Any, **kwargs: Any):
        tags = kwargs.get("tags") or ["weights", "kv_cache"]
        if "weights" in tags and not self.model.layers:
            self.model._alloc(seed=None)
            self.runner.drop_graphs()
            if self._offloaded is not None:
                self.model.load_weights(self._offloaded)
                self._offloaded = None
        if "kv_cache" in tags:
            self.runner.ensure_cache(self.num_blocks)

    # ---------------------------------------------------------------- weights
    async def init_weight_update_communicator(self, init_info):
        """init_info: a ready receiver (has `receive_weights(request)`), or a dict with
        {"group", "src"} for a broadcast receiver (broadcast_strategy.py:173-191)."""
        if hasattr(init_info, "receive_weights"):
            self._receiver = init_info
        else:
            from ..comm import BroadcastWeightReceiver

            info = dict(init_info or {})
            self._receiver = BroadcastWeightReceiver(self.model.dtype, group=info.get("group"),
                                                     src=info.get("src", 0), device=self.model.device)

    async def update_named_weights(self, request):
        """request: a WeightUpdateRequest (data through the receiver), or a dict / object with
        `names` and `tensors` (colocated path: CUDA-IPC handles resolved by the caller)."""
        tensors = request.get("tensors") if isinstance(request, dict) else getattr(request, "tensors", None)
        names = request["names"] if isinstance(request, dict) else request.names
        if tensors is not None:
            n = self.model.load_weights(zip(names, tensors))
        else:
            if self._receiver is None:
                raise RuntimeError("init_weight_update_communicator was not called")
            n = self.model.load_weights(self._receiver.receive_weights(request))
        self.core.reset_prefix_cache()  # cached K/V were computed by the old weights
        return n

    async def reset_prefix_cache(self):
        self.core.reset_prefix_cache()

    async def teardown(self):
        self.core.abort_all()
        self.runner.release_cache()

    def tp_size(self) -> int:
        return 1

    def pp_size(self) -> int:
        return 1

    def dp_size(self) -> int:
        return 1
