"""Rollout decode-loop measurements (§8(f)2) on one MI355X.

1. paged decode attention (csrc/attention.hip) at the configs' GQA shapes: algorithmic bytes =
   the K and V of every context token of every sequence (nkv * D * 2 B each) + q and out, per
   launch (one layer), / HIP-event launch time;
2. the engine end to end on a random-init Qwen2.5-1.5B-shaped decoder: 512 prompts (uniform
   [16, 512] tokens) x max_tokens decode steps (ignore_eos), tokens/s and ms per decode step.

Prints one JSON object.
"""

import argparse
import asyncio
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from skyrl_amd.inference_engines import kernels  # noqa: E402

DEV = torch.device("cuda:0")
BS = kernels.BLOCK_SIZE


def qwen15b_config(layers=28):
    from transformers import Qwen2Config

    return Qwen2Config(vocab_size=151936, hidden_size=1536, intermediate_size=8960, num_hidden_layers=layers,
                       num_attention_heads=12, num_key_value_heads=2, max_position_embeddings=32768,
                       rope_theta=1000000.0, rms_norm_eps=1e-6, tie_word_embeddings=True, eos_token_id=151645)


def attn_bench(nseq, ctx, nh, nkv, D=128, reps=20):
    g = torch.Generator(device=DEV).manual_seed(0)
    nb_seq = math.ceil(ctx / BS)
    nblk = nseq * nb_seq
    kc = torch.randn(nblk, nkv, BS, D, device=DEV, generator=g).to(torch.bfloat16)
    vc = torch.randn(nblk, nkv, D, BS, device=DEV, generator=g).to(torch.bfloat16)
    bt = torch.randperm(nblk, device=DEV, generator=g).int().view(nseq, nb_seq)
    cl = torch.full((nseq,), ctx, dtype=torch.int32, device=DEV)
    q = torch.randn(nseq, nh, D, device=DEV, generator=g).to(torch.bfloat16)
    out = torch.empty_like(q)
    ws = kernels.DecodeWorkspace(DEV)
    res = {}
    auto = kernels.choose_nparts(nseq, nkv, ctx)
    for nparts in sorted({auto, max(1, auto // 2), 2 * auto}):
        f = lambda: kernels.paged_decode(q, kc, vc, bt, cl, ctx, 1 / math.sqrt(D), out=out, workspace=ws,  # noqa
                                         nparts=nparts)
        f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record()
        b.synchronize()
        us = a.elapsed_time(b) * 1e3 / reps
        nbytes = nseq * ctx * nkv * D * 2 * 2 + 2 * nseq * nh * D * 2
        res[f"nparts={nparts}" + (" (auto)" if nparts == auto else "")] = {
            "us": round(us, 2), "GBps": round(nbytes / (us * 1e-6) / 1e9, 1), "bytes": nbytes}
    return res


def decode_step_bench(nseq, ctx, layers, reps=10):
    """One decode forward (+ lm_head) of nseq sequences at context ctx: eager wall time vs the
    same forward captured in a HIP graph and replayed (= GPU time without host launch cost)."""
    from skyrl_amd.inference_engines.model import PagedDecoder, PagedKVCache, StepInputs

    cfg = qwen15b_config(layers)
    m = PagedDecoder(cfg, DEV, seed=0, max_model_len=2048)
    nb = math.ceil((ctx + 1) / BS)
    cache = PagedKVCache(layers, nseq * nb, 2, 128, DEV)
    bt = torch.arange(nseq * nb, device=DEV, dtype=torch.int32).view(nseq, nb)
    pos = torch.full((nseq,), ctx - 1, dtype=torch.int64, device=DEV)
    inp = StepInputs(tokens=torch.randint(0, cfg.vocab_size, (nseq,), device=DEV), positions=pos,
                     slots=(bt[:, (ctx - 1) // BS].long() * BS + (ctx - 1) % BS), block_tables=bt,
                     context_lens=torch.full((nseq,), ctx, dtype=torch.int32, device=DEV), max_ctx=ctx)
    f = lambda: m.logits(m.forward_decode(inp, cache))  # noqa: E731
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t0) / reps * 1e3
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        f()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    graph_ms = (time.perf_counter() - t0) / reps * 1e3
    return {"nseq": nseq, "ctx": ctx, "layers": layers, "eager_ms": round(eager_ms, 3), "graph_ms": round(graph_ms, 3)}


def engine_bench(nprompts, max_tokens, layers, use_graphs=True):
    from skyrl_amd.inference_engines.engine import AMDInferenceEngine
    from skyrl_amd.inference_engines.model import PagedDecoder

    cfg = qwen15b_config(layers)
    t0 = time.time()
    model = PagedDecoder(cfg, DEV, seed=0, max_model_len=2048)
    torch.cuda.synchronize()
    init_s = time.time() - t0
    g = torch.Generator().manual_seed(1234)
    lens = torch.randint(16, 513, (nprompts,), generator=g).tolist()
    prompts = [torch.randint(0, cfg.vocab_size, (L,), generator=g).tolist() for L in lens]
    eng = AMDInferenceEngine(model, num_blocks=None, max_num_seqs=nprompts, kv_cache_fraction=0.3,
                             use_graphs=use_graphs)
    sp = {"temperature": 1.0, "max_tokens": max_tokens, "ignore_eos": True, "logprobs": 0}
    # warm-up: the full batch for a few tokens captures the decode graph of its bucket
    asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": {"max_tokens": 3}}))
    eng.core.stats.clear()
    torch.cuda.synchronize()
    steps0 = eng.core.num_steps
    t0 = time.time()
    out = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    torch.cuda.synchronize()
    dt = time.time() - t0
    ntok = sum(len(x) for x in out["response_ids"])
    steps = eng.core.num_steps - steps0
    return {"prompts": nprompts, "max_tokens": max_tokens, "layers": layers, "params": model.num_params(),
            "kv_blocks": eng.num_blocks, "seconds": round(dt, 3), "generated_tokens": ntok,
            "tokens_per_s": round(ntok / dt, 1), "engine_steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 3), "preemptions": eng.core.num_preemptions,
            "init_s": round(init_s, 2), "graphs": use_graphs,
            "stats": {k: round(v, 4) for k, v in eng.core.stats.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompts", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--layers", type=int, default=28)
    ap.add_argument("--skip-engine", action="store_true")
    ap.add_argument("--skip-attn", action="store_true")
    args = ap.parse_args()
    res = {"attention": {}, "decode_step": []}
    for nseq, ctx in ((512, 400), (512, 1280), (64, 1024), (8, 512)):
        res["decode_step"].append(decode_step_bench(nseq, ctx, args.layers))
        print(json.dumps(res["decode_step"][-1]), file=sys.stderr, flush=True)
    for name, nh, nkv in () if args.skip_attn else (("qwen2.5-1.5b", 12, 2), ("qwen2.5-7b", 28, 4), ("llama3-8b", 32, 8)):
        for nseq, ctx in ((512, 1280), (64, 4096), (8, 2048)):
            res["attention"][f"{name} nseq={nseq} ctx={ctx}"] = attn_bench(nseq, ctx, nh, nkv)
            print(json.dumps({name: res["attention"][f"{name} nseq={nseq} ctx={ctx}"]}), file=sys.stderr, flush=True)
    if not args.skip_engine:
        res["engine"] = engine_bench(args.prompts, args.max_tokens, args.layers)
        print(json.dumps(res["engine"]), file=sys.stderr, flush=True)
        res["engine_eager"] = engine_bench(args.prompts, args.max_tokens, args.layers, use_graphs=False)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
