"""§8(f)2 rollout decode loop on the GPU: paged-attention kernels vs a torch fp32 reference of
the same op, the paged decoder vs the HF transformers model of record (Qwen2 / Llama, the
reference's model classes), and the engine end to end (greedy tokens vs HF argmax, rollout
logprobs vs HF log_softmax, seeded reproducibility, weight update, sleep/wake_up).

Tolerances: attention output is bf16 with bf16 P in the P.V MFMA (rel. error ~2^-8 per
term): 2e-2 abs on unit-scale V. Model logits: bf16 end to end in both implementations with
different GEMM/attention kernels: compared by relative L2 error < 3e-2. Greedy tokens must
equal HF's argmax wherever HF's top-2 margin exceeds 0.1 (nearer ties may legitimately flip).
"""

import asyncio
import math

import pytest
import torch

from skyrl_amd.inference_engines import kernels
from skyrl_amd.inference_engines.engine import AMDInferenceEngine
from skyrl_amd.inference_engines.model import PagedDecoder, PagedKVCache, StepInputs

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
BS = kernels.BLOCK_SIZE


def torch_rope(x, cos_sin, pos):
    h = x.shape[-1] // 2
    c, s = cos_sin[pos, :h][:, None], cos_sin[pos, h:][:, None]
    x1, x2 = x[..., :h].float(), x[..., h:].float()
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


@pytest.mark.parametrize("nh,nkv,D", [(12, 2, 128), (4, 4, 64), (32, 8, 128)])
def test_rope_kv_write(nh, nkv, D):
    g = torch.Generator(device=DEV).manual_seed(0)
    T, nblk = 37, 20
    qkv = torch.randn(T, (nh + 2 * nkv) * D, device=DEV, generator=g).to(torch.bfloat16)
    pos = torch.randint(0, 500, (T,), device=DEV, generator=g)
    slots = torch.randperm(nblk * BS, device=DEV, generator=g)[:T]
    slots[3] = -1  # skipped
    ang = pos.new_tensor(range(512)).float()[:, None] * (1e-3 * torch.arange(1, D // 2 + 1, device=DEV))[None]
    cos_sin = torch.cat([ang.cos(), ang.sin()], -1).float().contiguous()
    kc = torch.zeros(nblk, nkv, BS, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nblk, nkv, D, BS, dtype=torch.bfloat16, device=DEV)
    k_out = torch.empty(T, nkv, D, dtype=torch.bfloat16, device=DEV)
    q = kernels.rope_kv_write(qkv, pos, slots, cos_sin, nh, nkv, D, kc, vc, k_out=k_out)
    x = qkv.view(T, nh + 2 * nkv, D)
    q_ref = torch_rope(x[:, :nh], cos_sin, pos).to(torch.bfloat16)
    k_ref = torch_rope(x[:, nh:nh + nkv], cos_sin, pos).to(torch.bfloat16)
    # the kernel may contract x1*c - x2*s into one fma: at most one bf16 ulp from the unfused form
    torch.testing.assert_close(q.float(), q_ref.float(), atol=1e-6, rtol=2 ** -7)
    torch.testing.assert_close(k_out.float(), k_ref.float(), atol=1e-6, rtol=2 ** -7)
    for t in range(T):
        s = int(slots[t])
        if s < 0:
            continue
        b, o = divmod(s, BS)
        assert torch.equal(kc[b, :, o], k_out[t])
        assert torch.equal(vc[b, :, :, o], x[t, nh + nkv:])
    # the skipped token wrote nothing: cache holds exactly T-1 nonzero K rows
    assert int((kc.abs().sum(-1) > 0).sum()) == (T - 1) * nkv


def build_paged(ctx_lens, nkv, D, g, extra_blocks=7):
    """Random K/V per sequence scattered into shuffled blocks; returns caches, table, dense K/V."""
    nb_seq = [math.ceil(c / BS) for c in ctx_lens]
    nblk = sum(nb_seq) + extra_blocks
    perm = torch.randperm(nblk, device=DEV, generator=g)
    kc = torch.randn(nblk, nkv, BS, D, device=DEV, generator=g).to(torch.bfloat16)  # stale junk everywhere
    vc = torch.randn(nblk, nkv, D, BS, device=DEV, generator=g).to(torch.bfloat16)
    maxb = max(nb_seq) + 2
    bt = torch.full((len(ctx_lens), maxb), 10 ** 6, dtype=torch.int32, device=DEV)  # junk past the context
    dense = []
    used = 0
    for i, c in enumerate(ctx_lens):
        blocks = perm[used:used + nb_seq[i]]
        used += nb_seq[i]
        bt[i, :nb_seq[i]] = blocks.int()
        K = kc[blocks].permute(1, 0, 2, 3).reshape(nkv, -1, D)[:, :c]
        Vv = vc[blocks].permute(1, 0, 3, 2).reshape(nkv, -1, D)[:, :c]
        dense.append((K.float(), Vv.float()))
    return kc, vc, bt, dense


def attn_ref(q, dense, scale):
    outs = []
    nh = q.shape[1]
    for i, (K, Vv) in enumerate(dense):
        rep = nh // K.shape[0]
        Kr, Vr = K.repeat_interleave(rep, 0), Vv.repeat_interleave(rep, 0)
        s = torch.einsum("hd,htd->ht", q[i].float(), Kr) * scale
        outs.append(torch.einsum("ht,htd->hd", torch.softmax(s, -1), Vr))
    return torch.stack(outs)


@pytest.mark.parametrize("nh,nkv,D", [(12, 2, 128), (28, 4, 128), (32, 8, 128), (8, 8, 64), (16, 1, 64)])
@pytest.mark.parametrize("nparts,part_min", [(None, 64), (1, 64), (3, 16), (64, 16)])
def test_paged_decode_matches_fp32_reference(nh, nkv, D, nparts, part_min):
    g = torch.Generator(device=DEV).manual_seed(nh * 7 + D)
    ctx = [1, 15, 16, 17, 33, 200, 1000, 2051]
    kc, vc, bt, dense = build_paged(ctx, nkv, D, g)
    q = torch.randn(len(ctx), nh, D, device=DEV, generator=g).to(torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    out = kernels.paged_decode(q, kc, vc, bt, cl, max(ctx), scale, nparts=nparts, part_min=part_min)
    ref = attn_ref(q, dense, scale)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    if nparts is None:  # the split depends only on the per-sequence context: a larger grid is a no-op
        big = kernels.paged_decode(q, kc, vc, bt, cl, max(ctx), scale, nparts=4096 // 64)
        assert torch.equal(big, kernels.paged_decode(q, kc, vc, bt, cl, max(ctx), scale, nparts=4096 // 64 + 5))


@pytest.mark.parametrize("pf", [4, 6, 8])
def test_paged_decode_prefetch_depths(pf):
    """Every K/V prefetch depth of the D = 128 kernel (skyrl_variant attn_pf: blocks in flight per
    wave, a register ring unrolled by the depth) matches the fp32 reference and the default
    bit for bit: ragged contexts that end mid-ring and past the 64-entry block-table window
    (2051 tokens = 129 blocks in one wave), unsplit and split."""
    g = torch.Generator(device=DEV).manual_seed(pf)
    ctx = [1, 16, 47, 63 * 16, 64 * 16 + 1, 129 * 16 - 13, 2051, 5]
    kc, vc, bt, dense = build_paged(ctx, 2, 128, g)
    q = torch.randn(len(ctx), 12, 128, device=DEV, generator=g).to(torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(128)
    ref = attn_ref(q, dense, scale)
    for nparts in (1, 3):
        base = kernels.paged_decode(q, kc, vc, bt, cl, max(ctx), scale, nparts=nparts)
        with kernels._ffi.variant(attn_pf=pf):
            out = kernels.paged_decode(q, kc, vc, bt, cl, max(ctx), scale, nparts=nparts)
        torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
        assert torch.equal(out, base)


@pytest.mark.parametrize("nh,nkv,D", [(12, 2, 128), (28, 4, 128), (16, 1, 64)])
@pytest.mark.parametrize("waves", [1, 3, 7, 64, 1024, 5000])
def test_paged_decode_balanced_matches_fp32_reference(nh, nkv, D, waves):
    """Block-balanced decode (every wave streams total_blocks / waves blocks across sequence
    boundaries; split sequences merged from per-wave records) vs the fp32 reference: one wave
    (everything in it), a few waves (long sequences split 2-3 ways, short ones whole), one per
    block, and more waves than blocks (empty waves). Contexts end mid-block and span > 64 blocks."""
    g = torch.Generator(device=DEV).manual_seed(waves * 3 + D)
    ctx = [1, 15, 16, 17, 33, 200, 1000, 2051, 5, 64 * 16 + 1, 700]
    kc, vc, bt, dense = build_paged(ctx, nkv, D, g)
    q = torch.randn(len(ctx), nh, D, device=DEV, generator=g).to(torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    out = kernels.paged_decode_balanced(q, kc, vc, bt, cl, scale, waves=waves)
    torch.testing.assert_close(out.float(), attn_ref(q, dense, scale), atol=2e-2, rtol=2e-2)
    # a strided q (a view into a fused qkv row) and a reused workspace give the same answer
    qkv = torch.zeros(len(ctx), (nh + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
    qkv[:, :nh * D] = q.reshape(len(ctx), -1)
    ws = kernels.DecodeWorkspace(DEV)
    for _ in range(2):
        again = kernels.paged_decode_balanced(qkv[:, :nh * D].view(len(ctx), nh, D), kc, vc, bt, cl, scale,
                                              waves=waves, workspace=ws)
        assert torch.equal(again, out)


def test_paged_decode_balanced_large_ragged_batch():
    g = torch.Generator(device=DEV).manual_seed(9)
    ctx = torch.randint(1, 1537, (512,), generator=torch.Generator().manual_seed(2)).tolist()
    kc, vc, bt, dense = build_paged(ctx, 2, 128, g)
    q = torch.randn(len(ctx), 12, 128, device=DEV, generator=g).to(torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    out = kernels.paged_decode_balanced(q, kc, vc, bt, cl, 1 / math.sqrt(128))
    torch.testing.assert_close(out.float(), attn_ref(q, dense, 1 / math.sqrt(128)), atol=2e-2, rtol=2e-2)


def test_paged_decode_large_batch_and_strided_q():
    g = torch.Generator(device=DEV).manual_seed(5)
    ctx = torch.randint(1, 1500, (300,), generator=torch.Generator().manual_seed(1)).tolist()
    kc, vc, bt, dense = build_paged(ctx, 2, 128, g)
    qkv = torch.randn(len(ctx), 16 * 128, device=DEV, generator=g).to(torch.bfloat16)
    q = qkv[:, :12 * 128].view(len(ctx), 12, 128)  # row stride 16*128: a view into the fused qkv
    out = kernels.paged_decode(q, kc, vc, bt, torch.tensor(ctx, dtype=torch.int32, device=DEV), max(ctx),
                               1 / math.sqrt(128))
    torch.testing.assert_close(out.float(), attn_ref(q, dense, 1 / math.sqrt(128)), atol=2e-2, rtol=2e-2)


def test_paged_decode_rejects_bad_shapes():
    q = torch.zeros(2, 12, 128, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(4, 2, BS, 128, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(4, 2, 128, BS, dtype=torch.bfloat16, device=DEV)
    bt = torch.zeros(2, 1, dtype=torch.int32, device=DEV)
    cl = torch.ones(2, dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):
        kernels.paged_decode(q, kc, vc, bt, cl, 40, 0.1)  # table too narrow for max_ctx
    with pytest.raises(ValueError):
        kernels.paged_decode(q, kc.transpose(2, 3), vc, bt, cl, 16, 0.1)


# ------------------------------------------------------------------ model vs HF
def tiny_hf(model_type="qwen2", seed=0):
    from transformers import LlamaConfig, Qwen2Config

    kw = dict(vocab_size=1031, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
              num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512, rms_norm_eps=1e-6,
              tie_word_embeddings=(model_type == "qwen2"), eos_token_id=2)
    cfg = Qwen2Config(**kw) if model_type == "qwen2" else LlamaConfig(**kw)
    cfg._attn_implementation = "eager"
    torch.manual_seed(seed)
    from transformers import AutoModelForCausalLM

    hf = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    with torch.no_grad():  # HF inits biases/norms to 0/1: perturb so they are exercised
        for n, p in hf.named_parameters():
            if n.endswith("bias") or "norm" in n:
                p.add_(0.1 * torch.randn_like(p))
        # std-0.02 init gives near-uniform logits (top-2 margins ~1e-2): scale the output
        # projection so greedy decisions are well separated and comparable across kernels
        hf.lm_head.weight.mul_(20.0)
    return cfg, hf


def our_model(cfg, hf, max_len=512):
    m = PagedDecoder(cfg, DEV, seed=None, max_model_len=max_len)
    n = m.load_weights(hf.state_dict().items())
    assert n >= len(list(m.hf_named_tensors()))
    return m


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("model_type", ["qwen2", "llama"])
def test_decoder_prefill_and_decode_logits_match_hf(model_type):
    cfg, hf = tiny_hf(model_type)
    m = our_model(cfg, hf)
    g = torch.Generator().manual_seed(3)
    lens = [5, 17, 40]
    seqs = [torch.randint(3, cfg.vocab_size, (L + 6,), generator=g).tolist() for L in lens]
    cache = PagedKVCache(cfg.num_hidden_layers, 64, 2, 128, DEV)
    blocks = [list(range(i * 8, i * 8 + 8))[::-1] for i in range(3)]  # non-contiguous order

    def slots(i, start, end):
        return [blocks[i][p // BS] * BS + p % BS for p in range(start, end)]

    toks = sum((s[:L] for s, L in zip(seqs, lens)), [])
    pos = sum((list(range(L)) for L in lens), [])
    sl = sum((slots(i, 0, L) for i, L in enumerate(lens)), [])
    t = lambda x: torch.tensor(x, dtype=torch.int64, device=DEV)  # noqa: E731
    with torch.no_grad():
        h = m.forward_prefill(StepInputs(tokens=t(toks), positions=t(pos), slots=t(sl), seq_lens=lens), cache)
        ours = m.logits(h)
        for i, L in enumerate(lens):
            ref = hf(t(seqs[i][:L])[None]).logits[0, -1]
            assert rel(ours[i], ref) < 3e-2
        for k in range(6):  # decode 6 tokens from the cache
            cur = [L + k for L in lens]
            bt = torch.tensor([b + [0] * 0 for b in blocks], dtype=torch.int32, device=DEV)
            inp = StepInputs(tokens=t([s[c] for s, c in zip(seqs, cur)]), positions=t(cur),
                             slots=t([slots(i, c, c + 1)[0] for i, c in enumerate(cur)]), block_tables=bt,
                             context_lens=torch.tensor([c + 1 for c in cur], dtype=torch.int32, device=DEV),
                             max_ctx=max(cur) + 1)
            ours = m.logits(m.forward_decode(inp, cache))
            for i, c in enumerate(cur):
                ref = hf(t(seqs[i][:c + 1])[None]).logits[0, -1]
                assert rel(ours[i], ref) < 3e-2, (i, k, rel(ours[i], ref))


def hf_greedy_check(hf, prompt, ids, margin=0.1):
    """Every engine token equals HF's argmax wherever HF's top-2 margin exceeds `margin`."""
    seq = list(prompt)
    checked = 0
    with torch.no_grad():
        for tok in ids:
            logits = hf(torch.tensor(seq, device=DEV)[None]).logits[0, -1].float()
            top2 = torch.topk(logits, 2)
            if float(top2.values[0] - top2.values[1]) < margin:
                break
            assert tok == int(top2.indices[0])
            checked += 1
            seq.append(tok)
    return checked


def test_engine_greedy_matches_hf_and_logprobs():
    cfg, hf = tiny_hf("qwen2", seed=1)
    m = our_model(cfg, hf)
    eng = AMDInferenceEngine(m, num_blocks=256, max_num_seqs=8)
    g = torch.Generator().manual_seed(4)
    prompts = [torch.randint(3, cfg.vocab_size, (L,), generator=g).tolist() for L in (3, 9, 30, 64, 1)]
    sp = {"temperature": 0.0, "max_tokens": 24, "logprobs": 0, "ignore_eos": True}
    out = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    total = 0
    for p, ids, lps in zip(prompts, out["response_ids"], out["response_logprobs"]):
        assert len(ids) == 24 and len(lps) == 24
        total += hf_greedy_check(hf, p, ids)
        with torch.no_grad():  # rollout logprob = log_softmax of the raw logits at the sampled token
            full = torch.tensor(p + ids, device=DEV)[None]
            lsm = torch.log_softmax(hf(full).logits[0, len(p) - 1:-1].float(), -1)
            ref_lp = lsm.gather(1, torch.tensor(ids, device=DEV)[:, None])[:, 0]
        torch.testing.assert_close(torch.tensor(lps), ref_lp.cpu(), atol=5e-2, rtol=0)
    assert total >= 60  # most positions are far from ties
    assert out["stop_reasons"] == ["length"] * 5


def test_engine_sampling_reproducible_and_eos():
    cfg, hf = tiny_hf("llama", seed=2)
    m = our_model(cfg, hf)
    prompts = [[5, 6, 7, 8]] * 4 + [[9] * 20]
    sp = {"temperature": 1.0, "max_tokens": 40, "min_tokens": 1, "seed": 11, "stop_token_ids": [17, 23]}
    outs = []
    for _ in range(2):
        eng = AMDInferenceEngine(m, num_blocks=64, max_num_seqs=3)  # forces waves of admission
        outs.append(asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp})))
    assert outs[0]["response_ids"] == outs[1]["response_ids"]
    for ids, reason in zip(outs[0]["response_ids"], outs[0]["stop_reasons"]):
        assert reason in ("stop", "length")
        if reason == "stop":
            assert ids[-1] in (17, 23, 2)
        assert all(t not in (17, 23, 2) for t in ids[:-1])
    # a per-request seed (vLLM SamplingParams.seed) makes equal prompts draw equal tokens
    assert outs[0]["response_ids"][0] == outs[0]["response_ids"][1]
    sp2 = dict(sp)
    sp2.pop("seed")
    eng = AMDInferenceEngine(m, num_blocks=64, max_num_seqs=8)
    o = asyncio.run(eng.generate({"prompt_token_ids": prompts[:4], "sampling_params": sp2}))
    assert len({tuple(x) for x in o["response_ids"]}) > 1  # unseeded requests differ


def test_engine_weight_update_and_sleep_wake():
    cfg, hf = tiny_hf("qwen2", seed=3)
    m = our_model(cfg, hf)
    eng = AMDInferenceEngine(m, num_blocks=128, max_num_seqs=4)
    sp = {"temperature": 0.0, "max_tokens": 8, "ignore_eos": True}
    prompts = [[4, 5, 6], [7, 8, 9, 10, 11]]
    before = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))["response_ids"]
    asyncio.run(eng.sleep(level=1))
    asyncio.run(eng.wake_up())
    again = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))["response_ids"]
    assert again == before
    cfg2, hf2 = tiny_hf("qwen2", seed=4)  # "learner" weights after an update
    sd = hf2.state_dict()
    names = list(sd)
    asyncio.run(eng.sleep(level=2))
    asyncio.run(eng.wake_up(tags=["weights"]))
    asyncio.run(eng.update_named_weights({"names": names, "tensors": [sd[n] for n in names]}))
    asyncio.run(eng.wake_up(tags=["kv_cache"]))
    after = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))["response_ids"]
    for p, ids in zip(prompts, after):
        assert hf_greedy_check(hf2, p, ids) >= 4


@pytest.mark.parametrize("H", [1536, 3584, 4096, 512])
def test_add_rmsnorm_matches_hf(H):
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RMSNorm

    g = torch.Generator(device=DEV).manual_seed(H)
    n = 37
    h = torch.randn(n, H, device=DEV, generator=g).to(torch.bfloat16)
    d = torch.randn(n, H, device=DEV, generator=g).to(torch.bfloat16)
    norm = Qwen2RMSNorm(H, eps=1e-6).to(DEV, torch.bfloat16)
    with torch.no_grad():
        norm.weight.copy_(1 + 0.1 * torch.randn(H, device=DEV, generator=g))
        ref_h = h + d
        ref = norm(ref_h)
    hh, out = h.clone(), torch.empty_like(h)
    kernels.add_rmsnorm(d, hh, norm.weight.data, 1e-6, out)
    assert torch.equal(hh, ref_h)  # residual stream: the same bf16 add
    torch.testing.assert_close(out.float(), ref.float(), atol=1e-6, rtol=2 ** -7)  # <= 1 bf16 ulp
    assert float((out != ref).float().mean()) < 0.01
    out2 = torch.empty_like(h)
    kernels.add_rmsnorm(None, hh, norm.weight.data, 1e-6, out2)  # no delta: plain norm
    torch.testing.assert_close(out2, out, atol=0, rtol=0)


def test_silu_mul_matches_torch():
    g = torch.Generator(device=DEV).manual_seed(1)
    gu = (3 * torch.randn(53, 2 * 8960, device=DEV, generator=g)).to(torch.bfloat16)
    ref = torch.nn.functional.silu(gu[:, :8960]) * gu[:, 8960:]
    out = kernels.silu_mul(gu)
    torch.testing.assert_close(out.float(), ref.float(), atol=1e-6, rtol=2 ** -7)
    assert float((out != ref).float().mean()) < 0.01


def test_engine_graph_and_eager_decode_agree():
    """Decode through captured HIP graphs (fixed partitions, bucketed rows, idle rows) and
    eagerly (exact rows, tight partitions) — both equal HF greedy where HF is decisive."""
    cfg, hf = tiny_hf("qwen2", seed=5)
    m = our_model(cfg, hf)
    g = torch.Generator().manual_seed(9)
    prompts = [torch.randint(3, cfg.vocab_size, (L,), generator=g).tolist() for L in (2, 7, 19, 33, 50, 4)]
    sp = {"temperature": 0.0, "max_tokens": 20, "ignore_eos": True, "logprobs": 0}
    outs = {}
    for graphs in (True, False):
        eng = AMDInferenceEngine(m, num_blocks=96, max_num_seqs=5, use_graphs=graphs)  # 6 prompts > 5 rows
        outs[graphs] = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    for p, a, b in zip(prompts, outs[True]["response_ids"], outs[False]["response_ids"]):
        assert hf_greedy_check(hf, p, a) >= 5 and hf_greedy_check(hf, p, b) >= 5
    la = torch.tensor(outs[True]["response_logprobs"])
    lb = torch.tensor(outs[False]["response_logprobs"])
    same = torch.tensor(outs[True]["response_ids"]) == torch.tensor(outs[False]["response_ids"])
    torch.testing.assert_close(la[same], lb[same], atol=2e-2, rtol=0)


def test_engine_prefix_cache_matches_uncached_prefill():
    """GRPO-shaped batch (4 prompts x 4 samples): with the prefix cache the siblings compute only
    their tail through the paged kernel (query rows over the shared cached blocks); greedy tokens
    and rollout logprobs match the uncached engine and HF."""
    cfg, hf = tiny_hf("qwen2", seed=6)
    m = our_model(cfg, hf)
    g = torch.Generator().manual_seed(11)
    base = [torch.randint(3, cfg.vocab_size, (L,), generator=g).tolist() for L in (16, 33, 47, 70)]
    prompts = [p for p in base for _ in range(4)]
    sp = {"temperature": 0.0, "max_tokens": 12, "ignore_eos": True, "logprobs": 0}
    outs = {}
    for caching in (False, True):
        eng = AMDInferenceEngine(m, num_blocks=256, max_num_seqs=16, enable_prefix_caching=caching)
        outs[caching] = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
        if caching:
            assert eng.core.allocator.hits >= 12 * 1  # every sibling reused its prompt's full blocks
            again = asyncio.run(eng.generate({"prompt_token_ids": prompts[:2], "sampling_params": sp}))
            assert again["response_ids"] == outs[True]["response_ids"][:2]  # served from the cache
    for p, a, b in zip(prompts, outs[True]["response_ids"], outs[False]["response_ids"]):
        assert hf_greedy_check(hf, p, a) >= 4 and hf_greedy_check(hf, p, b) >= 4
    la, lb = torch.tensor(outs[True]["response_logprobs"]), torch.tensor(outs[False]["response_logprobs"])
    same = torch.tensor(outs[True]["response_ids"]) == torch.tensor(outs[False]["response_ids"])
    assert float(same.float().mean()) > 0.9
    torch.testing.assert_close(la[same], lb[same], atol=3e-2, rtol=0)


@pytest.mark.parametrize("temp", [0.0, 1.0])
def test_engine_fused_lmhead_sampler_equals_unfused(temp):
    """§8(f)1 decode side inside the engine: the lm_head GEMM with the sampler in its epilogue
    (fused_lmhead) gives the same tokens as the library GEMM + skyrl_sample whenever the bf16
    logits agree (the GEMMs' fp32 sums round to bf16; compared here against the fused kernel's own
    plain-GEMM output, skyrl_lmhead_gemm), and logprobs to 1e-4; the fused path really ran."""
    from skyrl_amd import ops

    cfg, hf = tiny_hf("qwen2", seed=2)
    m = our_model(cfg, hf)
    g = torch.Generator().manual_seed(6)
    prompts = [torch.randint(3, cfg.vocab_size, (L,), generator=g).tolist() for L in (4, 11, 27, 2)]
    sp = {"temperature": temp, "max_tokens": 16, "logprobs": 0, "ignore_eos": True, "seed": 5}
    fused = AMDInferenceEngine(m, num_blocks=256, max_num_seqs=8, fused_lmhead="always")
    a = asyncio.run(fused.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    assert fused.runner.fused_steps >= 16
    # reference: the unfused sampler over the fused kernel's own logits (identical bf16 values)
    plain = AMDInferenceEngine(m, num_blocks=256, max_num_seqs=8, fused_lmhead="off")
    plain.runner.model.logits = lambda h: ops.lmhead_gemm(h.contiguous(), m.lm_head)
    b = asyncio.run(plain.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    assert plain.runner.fused_steps == 0
    assert a["response_ids"] == b["response_ids"]
    for x, y in zip(a["response_logprobs"], b["response_logprobs"]):
        torch.testing.assert_close(torch.tensor(x), torch.tensor(y), atol=1e-4, rtol=0)


def _penalized(logits, prompt, out, rep, pres, freq):
    """vLLM apply_penalties on one row (repetition over prompt + output, presence / frequency
    over output counts)."""
    from collections import Counter

    x = logits.clone()
    c = Counter(out)
    seen = set(prompt) | set(c)
    if rep != 1.0:
        idx = torch.tensor(sorted(seen), device=x.device)
        v = x[idx]
        x[idx] = torch.where(v > 0, v / rep, v * rep)
    if c:
        idx = torch.tensor(sorted(c), device=x.device)
        cnt = torch.tensor([c[t] for t in sorted(c)], device=x.device, dtype=x.dtype)
        x[idx] -= freq * cnt + pres
    return x


@pytest.mark.parametrize("pen", [(1.3, 0.0, 0.0), (1.0, 0.8, 0.3), (0.7, -0.5, 0.2)])
def test_engine_penalties_greedy_vs_hf(pen):
    """repetition / presence / frequency penalties (vLLM semantics) on greedy decoding: every token
    is the argmax of HF's penalized logits wherever that margin exceeds 0.1, and the returned
    logprob is the RAW one (vLLM's default logprobs_mode), not the penalized one."""
    rep, pres, freq = pen
    cfg, hf = tiny_hf("qwen2", seed=3)
    m = our_model(cfg, hf)
    eng = AMDInferenceEngine(m, num_blocks=256, max_num_seqs=8)
    g = torch.Generator().manual_seed(8)
    prompts = [torch.randint(3, cfg.vocab_size, (L,), generator=g).tolist() for L in (5, 13)]
    sp = {"temperature": 0.0, "max_tokens": 20, "logprobs": 0, "ignore_eos": True, "repetition_penalty": rep,
          "presence_penalty": pres, "frequency_penalty": freq}
    out = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    assert eng.runner.fused_steps == 0  # penalties take the unfused path
    checked = 0
    with torch.no_grad():
        for p, ids, lps in zip(prompts, out["response_ids"], out["response_logprobs"]):
            for k, tok in enumerate(ids):
                raw = hf(torch.tensor(p + ids[:k], device=DEV)[None]).logits[0, -1].float()
                x = _penalized(raw, p, ids[:k], rep, pres, freq)
                top2 = torch.topk(x, 2)
                if float(top2.values[0] - top2.values[1]) < 0.1:
                    break
                assert tok == int(top2.indices[0]), (k, tok, int(top2.indices[0]))
                assert abs(lps[k] - float(torch.log_softmax(raw, -1)[tok])) < 5e-2
                checked += 1
    assert checked >= 10


def test_engine_n_samples_and_top_logprobs():
    """n > 1: n consecutive samples per prompt; a seeded request's j-th sample is the n = 1
    request with seed + j (vLLM parallel sampling). logprobs = 5 returns the sampled token's
    logprob, as logprobs = 0 does (the reference reads only that one, vllm_engine.py:139-149)."""
    cfg, hf = tiny_hf("qwen2", seed=4)
    with torch.no_grad():  # undo tiny_hf's sharpening: samples at T = 1 should differ
        hf.lm_head.weight.div_(20.0)
    m = our_model(cfg, hf)
    eng = AMDInferenceEngine(m, num_blocks=256, max_num_seqs=16)
    prompts = [[5, 6, 7, 8], [9, 10, 11]]
    sp = {"temperature": 1.0, "max_tokens": 12, "logprobs": 0, "ignore_eos": True, "seed": 7}
    a = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": dict(sp, n=3)}))
    assert len(a["response_ids"]) == 6
    for i, p in enumerate(prompts):
        for j in range(3):
            b = asyncio.run(eng.generate({"prompt_token_ids": [p], "sampling_params": dict(sp, seed=7 + j)}))
            assert a["response_ids"][3 * i + j] == b["response_ids"][0]
        assert len({tuple(x) for x in a["response_ids"][3 * i:3 * i + 3]}) > 1
    c = asyncio.run(eng.generate({"prompt_token_ids": prompts[:1], "sampling_params": dict(sp, logprobs=5)}))
    d = asyncio.run(eng.generate({"prompt_token_ids": prompts[:1], "sampling_params": sp}))
    assert c["response_ids"] == d["response_ids"] and c["response_logprobs"] == d["response_logprobs"]


@pytest.mark.parametrize("shape", [(192, 1536, 151936), (16, 1536, 151936), (512, 896, 50257)])
def test_lmhead_gemm_vs_flinear_logits_and_argmax(shape):
    """The engine's default fused_lmhead="auto" picks the MFMA GEMM (with or without the sampler
    in its epilogue) or F.linear by batch occupancy, so a request's logits can come from either.
    Both round fp32 sums to bf16: they agree within one bf16 rounding (rtol 2^-7), almost all
    elements bit for bit, and the greedy token (argmax) is the same wherever the F.linear top-2
    margin exceeds that rounding."""
    import torch.nn.functional as F

    from skyrl_amd import ops

    M, H, V = shape
    g = torch.Generator(device="cuda").manual_seed(M + V)
    h = torch.randn(M, H, device="cuda", generator=g).to(torch.bfloat16)
    w = (0.02 * torch.randn(V, H, device="cuda", generator=g)).to(torch.bfloat16)
    a = ops.lmhead_gemm(h, w).float()
    b = F.linear(h, w).float()
    torch.testing.assert_close(a, b, atol=1e-3, rtol=2 ** -7)
    assert float((a != b).float().mean()) < 0.02
    top2 = b.topk(2, dim=-1).values
    decisive = (top2[:, 0] - top2[:, 1]) > 2 ** -6 * top2[:, 0].abs().clamp(min=1e-3)
    assert bool(decisive.any())
    assert torch.equal(a.argmax(-1)[decisive], b.argmax(-1)[decisive])
