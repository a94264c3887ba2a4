"""Decoder-only transformer (HF Qwen2 / Llama semantics) for the rollout engine, with a
paged KV cache.

The reference generates with vLLM (inference_engines/vllm/vllm_engine.py) on HF checkpoints
(policy model `Qwen/Qwen2.5-1.5B-Instruct`, ppo_base_config.yaml:26); this module is the
MI355X engine's model runner. GEMMs are PyTorch-ROCm (hipBLASLt) — the north star keeps the
transformer in PyTorch — while the decode-loop specific ops are HIP: fused RoPE + paged
KV write and MFMA decode attention (csrc/attention.hip), and the sampler (csrc/sampler.hip).

Weights use the HF parameter names on the way in and out (`load_weights`, `hf_named_tensors`),
so the learner's state dict and the weight-sync requests (WeightUpdateRequest names,
weight_sync/base.py) address them directly; q/k/v and gate/up are stored fused, one GEMM
each (the slices are views, as vLLM's stacked parameters).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Iterable, Iterator, List, Optional, Tuple

import torch
import torch.nn.functional as F

from . import kernels

BLOCK_SIZE = kernels.BLOCK_SIZE


@dataclass
class DecoderSpec:
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    rms_norm_eps: float
    qkv_bias: bool
    tie_word_embeddings: bool
    max_position_embeddings: int
    initializer_range: float = 0.02
    eos_token_id: Optional[int] = None

    @classmethod
    def from_hf(cls, cfg) -> "DecoderSpec":
        mt = getattr(cfg, "model_type", "")
        if mt not in ("qwen2", "llama", "mistral", "qwen3"):
            raise ValueError(f"unsupported model_type {mt!r} (qwen2/llama/mistral)")
        nh = cfg.num_attention_heads
        hd = getattr(cfg, "head_dim", None) or cfg.hidden_size // nh
        eos = cfg.eos_token_id
        if isinstance(eos, (list, tuple)):
            eos = eos[0] if eos else None
        return cls(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                   num_layers=cfg.num_hidden_layers, num_heads=nh,
                   num_kv_heads=getattr(cfg, "num_key_value_heads", None) or nh, head_dim=hd,
                   rms_norm_eps=cfg.rms_norm_eps,
                   qkv_bias=(mt == "qwen2") or bool(getattr(cfg, "attention_bias", False)),
                   tie_word_embeddings=bool(getattr(cfg, "tie_word_embeddings", False)),
                   max_position_embeddings=cfg.max_position_embeddings,
                   initializer_range=getattr(cfg, "initializer_range", 0.02), eos_token_id=eos)


def rope_cos_sin(hf_config, max_pos: int, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """[max_pos, D] f32 table: cos | sin halves, computed by the HF rotary module itself and
    rounded to the model dtype as HF's forward does (cos.to(x.dtype))."""
    import importlib

    mt = hf_config.model_type
    mod = importlib.import_module(f"transformers.models.{mt}.modeling_{mt}")
    rot_cls = getattr(mod, {"qwen2": "Qwen2RotaryEmbedding", "llama": "LlamaRotaryEmbedding",
                            "mistral": "MistralRotaryEmbedding", "qwen3": "Qwen3RotaryEmbedding"}[mt])
    rot = rot_cls(hf_config)
    pos = torch.arange(max_pos, dtype=torch.int64)[None]
    x = torch.zeros(1, dtype=dtype)
    cos, sin = rot(x, pos)
    cos, sin = cos[0].to(dtype).float(), sin[0].to(dtype).float()
    h = cos.shape[-1] // 2
    return torch.cat([cos[:, :h], sin[:, :h]], dim=-1).contiguous()


class PagedKVCache:
    """Per-layer K [blocks, nkv, 16, D] and V [blocks, nkv, D, 16] bf16, zero-initialised
    (masked tail slots of a block are read by the MFMA: they must hold finite values)."""

    def __init__(self, num_layers: int, num_blocks: int, nkv: int, head_dim: int, device,
                 dtype: torch.dtype = torch.bfloat16):
        self.num_layers, self.num_blocks, self.nkv, self.head_dim = num_layers, num_blocks, nkv, head_dim
        self.k = torch.zeros((num_layers, num_blocks, nkv, BLOCK_SIZE, head_dim), dtype=dtype, device=device)
        self.v = torch.zeros((num_layers, num_blocks, nkv, head_dim, BLOCK_SIZE), dtype=dtype, device=device)

    @staticmethod
    def bytes_per_block(num_layers: int, nkv: int, head_dim: int, dtype=torch.bfloat16) -> int:
        return 2 * num_layers * nkv * BLOCK_SIZE * head_dim * torch.tensor([], dtype=dtype).element_size()


@dataclass
class StepInputs:
    """Device inputs of one forward over T tokens of n sequences."""

    tokens: torch.Tensor        # int64 [T]
    positions: torch.Tensor     # int64 [T]
    slots: torch.Tensor         # int64 [T]
    # decode only
    block_tables: Optional[torch.Tensor] = None  # int32 [n, max_blocks]
    context_lens: Optional[torch.Tensor] = None  # int32 [n]
    max_ctx: int = 0
    nparts: Optional[int] = None  # decode waves per (sequence, kv head); None: chosen per call
    # prefill only: tokens computed per sequence (host) and the cached prefix each starts after
    seq_lens: Optional[List[int]] = None
    cached_lens: Optional[List[int]] = None


class PagedDecoder:
    """Weights + forward of a Qwen2/Llama decoder over a paged KV cache."""

    def __init__(self, hf_config, device, dtype: torch.dtype = torch.bfloat16, seed: Optional[int] = 0,
                 max_model_len: Optional[int] = None):
        self.hf_config = hf_config
        self.spec = s = DecoderSpec.from_hf(hf_config)
        self.device = torch.device(device)
        self.dtype = dtype
        self.max_model_len = min(max_model_len or s.max_position_embeddings, s.max_position_embeddings)
        self.scale = 1.0 / math.sqrt(s.head_dim)
        self.cos_sin = rope_cos_sin(hf_config, self.max_model_len, dtype).to(self.device)
        self.workspace = kernels.DecodeWorkspace(self.device)
        self._alloc(seed)

    # ---------------------------------------------------------------- weights
    def _alloc(self, seed: Optional[int]):
        s, dev, dt = self.spec, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(0 if seed is None else seed)
        std = s.initializer_range

        def w(*shape):
            t = torch.empty(shape, dtype=dt, device=dev)
            return t.normal_(0.0, std, generator=g) if seed is not None else t.zero_()

        qkv_out = (s.num_heads + 2 * s.num_kv_heads) * s.head_dim
        self.embed = w(s.vocab_size, s.hidden_size)
        self.layers: List[Dict[str, torch.Tensor]] = []
        for _ in range(s.num_layers):
            self.layers.append({
                "ln1": torch.ones(s.hidden_size, dtype=dt, device=dev),
                "wqkv": w(qkv_out, s.hidden_size),
                "bqkv": torch.zeros(qkv_out, dtype=dt, device=dev) if s.qkv_bias else None,
                "wo": w(s.hidden_size, s.num_heads * s.head_dim),
                "ln2": torch.ones(s.hidden_size, dtype=dt, device=dev),
                "wgu": w(2 * s.intermediate_size, s.hidden_size),
                "wd": w(s.hidden_size, s.intermediate_size),
            })
        self.norm = torch.ones(s.hidden_size, dtype=dt, device=dev)
        self.lm_head = self.embed if s.tie_word_embeddings else w(s.vocab_size, s.hidden_size)

    def _param_views(self) -> Dict[str, torch.Tensor]:
        """HF name -> view into the (fused) storage."""
        s = self.spec
        q, kv = s.num_heads * s.head_dim, s.num_kv_heads * s.head_dim
        I = s.intermediate_size
        out = {"model.embed_tokens.weight": self.embed, "model.norm.weight": self.norm}
        if not s.tie_word_embeddings:
            out["lm_head.weight"] = self.lm_head
        for i, L in enumerate(self.layers):
            p = f"model.layers.{i}."
            out[p + "input_layernorm.weight"] = L["ln1"]
            out[p + "post_attention_layernorm.weight"] = L["ln2"]
            out[p + "self_attn.q_proj.weight"] = L["wqkv"][:q]
            out[p + "self_attn.k_proj.weight"] = L["wqkv"][q:q + kv]
            out[p + "self_attn.v_proj.weight"] = L["wqkv"][q + kv:]
            if L["bqkv"] is not None:
                out[p + "self_attn.q_proj.bias"] = L["bqkv"][:q]
                out[p + "self_attn.k_proj.bias"] = L["bqkv"][q:q + kv]
                out[p + "self_attn.v_proj.bias"] = L["bqkv"][q + kv:]
            out[p + "self_attn.o_proj.weight"] = L["wo"]
            out[p + "mlp.gate_proj.weight"] = L["wgu"][:I]
            out[p + "mlp.up_proj.weight"] = L["wgu"][I:]
            out[p + "mlp.down_proj.weight"] = L["wd"]
        return out

    def hf_named_tensors(self) -> Iterator[Tuple[str, torch.Tensor]]:
        yield from self._param_views().items()

    def load_weights(self, named: Iterable[Tuple[str, torch.Tensor]]) -> int:
        """Copy HF-named tensors into place (WorkerWrap.load_weights, inference_servers/vllm_worker.py:74-96).
        `lm_head.weight` of a tied model is accepted and ignored, as vLLM does. Unknown names raise."""
        views = self._param_views()
        n = 0
        with torch.no_grad():
            for name, t in named:
                dst = views.get(name)
                if dst is None:
                    if name == "lm_head.weight" and self.spec.tie_word_embeddings:
                        continue
                    if name.endswith("rotary_emb.inv_freq"):
                        continue
                    raise KeyError(f"unknown parameter {name!r}")
                if tuple(t.shape) != tuple(dst.shape):
                    raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(dst.shape)}")
                dst.copy_(t, non_blocking=True)
                n += 1
        return n

    def num_params(self) -> int:
        return sum(int(t.numel()) for t in self._param_views().values())

    def release(self):
        """Drop the weights (sleep level 2 discards them, vllm_engine.py sleep())."""
        self.embed = self.lm_head = self.norm = None
        self.layers = []

    # ---------------------------------------------------------------- forward
    def _run_layers(self, h: torch.Tensor, attention) -> torch.Tensor:
        """Residual stream h [T, H] (bf16, updated in place) through every layer; `attention(li, L,
        qkv)` returns the attention output [T, nh*D]. Norms and the SiLU gate are the fused HIP
        kernels (csrc/decoder_ops.hip); GEMMs are hipBLASLt through torch. Returns the final-norm
        output [T, H]."""
        s = self.spec
        eps = s.rms_norm_eps
        x = torch.empty_like(h)
        kernels.add_rmsnorm(None, h, self.layers[0]["ln1"], eps, x)
        for li, L in enumerate(self.layers):
            qkv = F.linear(x, L["wqkv"], L["bqkv"])
            a = attention(li, L, qkv)
            kernels.add_rmsnorm(F.linear(a, L["wo"]), h, L["ln2"], eps, x)
            act = kernels.silu_mul(F.linear(x, L["wgu"]))
            nxt = self.layers[li + 1]["ln1"] if li + 1 < len(self.layers) else self.norm
            kernels.add_rmsnorm(F.linear(act, L["wd"]), h, nxt, eps, x)
        return x

    def forward_decode(self, inp: StepInputs, cache: PagedKVCache) -> torch.Tensor:
        """One token per sequence: returns the final hidden states [n, H]."""
        s = self.spec
        h = F.embedding(inp.tokens, self.embed)
        n = h.shape[0]
        q_buf = torch.empty((n, s.num_heads, s.head_dim), dtype=self.dtype, device=self.device)
        a_buf = torch.empty_like(q_buf)

        def attention(li, L, qkv):
            q = kernels.rope_kv_write(qkv, inp.positions, inp.slots, self.cos_sin, s.num_heads, s.num_kv_heads,
                                      s.head_dim, cache.k[li], cache.v[li], q_out=q_buf)
            a = kernels.paged_decode(q, cache.k[li], cache.v[li], inp.block_tables, inp.context_lens, inp.max_ctx,
                                     self.scale, out=a_buf, workspace=self.workspace, nparts=inp.nparts)
            return a.view(n, -1)

        return self._run_layers(h, attention)

    def forward_prefill(self, inp: StepInputs, cache: PagedKVCache) -> torch.Tensor:
        """Ragged prefill (total T tokens; per sequence inp.seq_lens tokens starting at position
        inp.cached_lens[i]): writes their K/V into the cache and returns the final hidden state of
        each sequence's last token [B, H].

        Sequences without a cached prefix attend with causal SDPA on a right-padded batch of
        their own tokens. Sequences whose leading blocks came from the prefix cache compute
        only their suffix: each suffix token is one query row of the paged decode kernel over
        its sequence's block table with context = position + 1 (its K/V, and those of the
        suffix tokens before it, are written by rope_kv_write first)."""
        s = self.spec
        lens = list(inp.seq_lens)
        cached = list(inp.cached_lens) if inp.cached_lens is not None else [0] * len(lens)
        T = int(sum(lens))
        dev = self.device
        starts = torch.tensor([0] + lens[:-1], dtype=torch.int64).cumsum(0)
        lens_t = torch.tensor(lens, dtype=torch.int64)
        last = (starts + lens_t - 1).to(dev, non_blocking=True)
        full = [i for i, c in enumerate(cached) if c == 0]
        part = [i for i, c in enumerate(cached) if c > 0]
        nhd = s.num_heads * s.head_dim
        k_out = torch.empty((T, s.num_kv_heads, s.head_dim), dtype=self.dtype, device=dev) if full else None
        rep = s.num_heads // s.num_kv_heads
        if full:  # padded layout of the uncached sequences (T indexes a zero row)
            fl = lens_t[full]
            Lmax = int(fl.max())
            j = torch.arange(Lmax, dtype=torch.int64)
            inside = j[None] < fl[:, None]
            pad_idx = torch.where(inside, starts[full][:, None] + j[None], torch.full((1, 1), T)).to(dev)
            valid = inside.reshape(-1).nonzero().squeeze(1).to(dev)
            tok_full = (starts[full][:, None] + j[None])[inside].to(dev)
        if part:  # one decode-kernel row per suffix token
            tok_part = torch.cat([torch.arange(int(starts[i]), int(starts[i]) + lens[i]) for i in part])
            seq_of = torch.cat([torch.full((lens[i],), i, dtype=torch.int64) for i in part])
            ctx = torch.cat([torch.arange(cached[i] + 1, cached[i] + lens[i] + 1, dtype=torch.int32) for i in part])
            max_ctx = int(ctx.max())
            bt = inp.block_tables.index_select(0, seq_of.to(dev))[:, :-(-max_ctx // BLOCK_SIZE)].contiguous()
            tok_part, ctx = tok_part.to(dev), ctx.to(dev)

        def attention(li, L, qkv):
            q = kernels.rope_kv_write(qkv, inp.positions, inp.slots, self.cos_sin, s.num_heads, s.num_kv_heads,
                                      s.head_dim, cache.k[li], cache.v[li], k_out=k_out)
            if not part:
                o = self._sdpa(q, k_out, qkv, T, pad_idx, rep)
                return o.transpose(1, 2).reshape(-1, nhd)[valid]
            o = torch.empty((T, nhd), dtype=self.dtype, device=dev)
            if full:
                of = self._sdpa(q, k_out, qkv, T, pad_idx, rep)
                o.index_copy_(0, tok_full, of.transpose(1, 2).reshape(-1, nhd)[valid])
            op = kernels.paged_decode(q.index_select(0, tok_part), cache.k[li], cache.v[li], bt, ctx, max_ctx,
                                      self.scale, workspace=self.workspace)
            o.index_copy_(0, tok_part, op.view(-1, nhd))
            return o

        h = F.embedding(inp.tokens, self.embed)
        return self._run_layers(h, attention)[last]

    def _sdpa(self, q, k, qkv, T, pad_idx, rep):
        s = self.spec
        v = qkv[:, (s.num_heads + s.num_kv_heads) * s.head_dim:].reshape(T, s.num_kv_heads, s.head_dim)

        def padded(t):
            z = torch.cat([t, t.new_zeros((1,) + tuple(t.shape[1:]))], 0)
            return z[pad_idx].transpose(1, 2)  # [B, heads, Lmax, D]

        return F.scaled_dot_product_attention(padded(q), padded(k), padded(v), is_causal=True, scale=self.scale,
                                              enable_gqa=rep > 1)

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """lm_head: bf16 [n, V] (the sampler's input)."""
        return F.linear(hidden, self.lm_head)
