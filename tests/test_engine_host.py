"""Rollout engine host logic on CPU: scheduler, block allocation and recompute preemption,
stop conditions, abort, the async InferenceEngineInterface and the client's pause/resume retry
(inference_engines/inference_engine_client.py:223-330,597-628). The device runner is replaced
by a deterministic fake whose next token is a function of the whole token history, so any
scheduling error (lost tokens, wrong positions after preemption) changes the outputs."""

import asyncio
from types import SimpleNamespace

import numpy as np
import pytest

from skyrl_amd.inference_engines.client import InferenceEngineClient, route_prompts_to_engines
from skyrl_amd.inference_engines.engine import BLOCK_SIZE, AMDInferenceEngine, EngineCore, RequestParams

V = 97


def next_token(history, suppress=()):
    t = (sum((i + 1) * x for i, x in enumerate(history)) * 31 + 7) % V
    while t in suppress:
        t = (t + 1) % V
    return t


class FakeRunner:
    def __init__(self, num_blocks):
        self.owner = {}  # block -> rid, to catch double allocation
        self.batches = []
        self.num_blocks = num_blocks

    def execute(self, batch):
        self.batches.append((batch.kind, len(batch.requests)))
        seen = {}
        rows = [r.row for r in batch.requests]
        assert len(set(rows)) == len(rows) and min(rows) >= 0, "persistent rows must be unique"
        written = {}
        for r in batch.requests:
            need = (r.num_tokens + (1 if batch.kind == "prefill" else 0) + BLOCK_SIZE - 1) // BLOCK_SIZE
            assert len(r.blocks) >= min(need, (r.num_tokens + BLOCK_SIZE - 1) // BLOCK_SIZE)
            first = r.num_cached if batch.kind == "prefill" else r.num_tokens - 1  # first position written
            for i, b in enumerate(r.blocks):
                assert 0 <= b < self.num_blocks
                seen.setdefault(b, set()).add(r.rid)
                if (i + 1) * BLOCK_SIZE > first and i * BLOCK_SIZE < r.num_tokens:
                    assert written.setdefault(b, r.rid) == r.rid, "a block written this step is written twice"
        for b, rid in written.items():  # shared (prefix-cached) blocks are read-only
            assert seen[b] == {rid}, "a block written this step is also read by another request"
        toks = np.array([next_token(r.prompt + r.out_tokens, sup) for r, sup in zip(batch.requests, batch.suppress)],
                        dtype=np.int64)
        lps = -np.arange(len(toks), dtype=np.float32) / 10
        return toks, lps

    def release_cache(self):
        pass

    def ensure_cache(self, n):
        pass

    def drop_graphs(self):
        pass


def run_all(core):
    while core.has_unfinished():
        core.step()


def reference_output(prompt, params, eos=None):
    out = []
    while True:
        sup = ()
        if len(out) < params.min_tokens:
            sup = tuple(sorted(set(params.stop_token_ids) | ({eos} if eos is not None else set())))
        t = next_token(prompt + out, sup)
        out.append(t)
        if len(out) >= params.min_tokens and (t in params.stop_token_ids or t == eos):
            return out, "stop"
        if len(out) >= params.max_tokens:
            return out, "length"


def test_request_params_parse():
    p = RequestParams.from_dict({"max_tokens": 8, "min_tokens": 1, "temperature": 0.7, "top_p": 0.9, "top_k": 50,
                                 "min_p": 0.0, "logprobs": 0, "stop": None, "skip_special_tokens": True,
                                 "include_stop_str_in_output": True})
    assert (p.max_tokens, p.min_tokens, p.top_k, p.logprobs) == (8, 1, 50, 0)
    q = RequestParams.from_dict({"n": 3, "repetition_penalty": 1.1, "presence_penalty": 0.5,
                                 "frequency_penalty": -0.2, "logprobs": 5})
    assert (q.n, q.repetition_penalty, q.presence_penalty, q.frequency_penalty, q.logprobs) == (3, 1.1, 0.5, -0.2, 5)
    assert q.has_penalty() and not p.has_penalty()
    for bad in ({"n": 0}, {"repetition_penalty": 0.0}, {"presence_penalty": 2.5}, {"frequency_penalty": -3}):
        with pytest.raises(ValueError):
            RequestParams.from_dict(bad)
    assert RequestParams.from_dict({"stop": ["</sql>", "x"]}).stop == ("</sql>", "x")
    assert RequestParams.from_dict({"stop": "\n"}).stop == ("\n",)
    with pytest.raises(ValueError):  # stop strings need a tokenizer in the engine
        EngineCore(FakeRunner(10), 10).add_request([1], RequestParams(stop=("\n",)))
    with pytest.raises(ValueError):
        RequestParams.from_dict({"bogus": 1})


def test_stop_strings_end_a_request_and_cut_the_text():
    """vLLM semantics: a stop string in the decoded output finishes the request with "stop" (not
    before min_tokens); the response text ends with it (include_stop_str_in_output)."""
    chars = "abcdefghijklmnopqrstuvwxyz</>"

    class CharTok:
        def decode(self, ids, skip_special_tokens=True):
            return "".join(chars[i % len(chars)] for i in ids)

    class ScriptRunner(FakeRunner):
        def execute(self, batch):
            toks = [chars.index("</sql>"[len(r.out_tokens) % 6]) if r.prompt[0] == 0 else 0 for r in batch.requests]
            return np.array(toks, dtype=np.int64), np.zeros(len(toks), dtype=np.float32)

    model = SimpleNamespace(max_model_len=256, spec=SimpleNamespace(eos_token_id=None))
    eng = AMDInferenceEngine(model, num_blocks=50, max_num_seqs=4, runner=ScriptRunner(50), tokenizer=CharTok())
    out = asyncio.run(eng.generate({"prompt_token_ids": [[0, 1], [1, 2]],
                                    "sampling_params": {"max_tokens": 20, "stop": ["sql>"], "min_tokens": 1}}))
    assert out["stop_reasons"] == ["stop", "length"]
    assert out["responses"][0] == "</sql>" and len(out["response_ids"][0]) == 6
    out = asyncio.run(eng.generate({"prompt_token_ids": [[0, 1]],
                                    "sampling_params": {"max_tokens": 20, "stop": ["sql>"], "min_tokens": 9}}))
    assert out["stop_reasons"] == ["stop"] and out["responses"][0] == "</sql></sql>" and len(out["response_ids"][0]) == 12


@pytest.mark.parametrize("num_blocks", [400, 12])
def test_scheduler_outputs_independent_of_cache_pressure(num_blocks):
    """With 12 blocks the running set must be preempted and recomputed repeatedly; outputs must
    equal the unconstrained sequential answer."""
    rng = np.random.default_rng(0)
    runner = FakeRunner(num_blocks)
    core = EngineCore(runner, num_blocks, max_num_seqs=6, max_model_len=200, max_prefill_tokens=64,
                      eos_token_id=3)
    reqs, expect = [], []
    for i in range(10):
        prompt = rng.integers(0, V, size=int(rng.integers(1, 30))).tolist()
        params = RequestParams(max_tokens=int(rng.integers(1, 40)), min_tokens=int(rng.integers(0, 3)),
                               stop_token_ids=(5,))
        reqs.append(core.add_request(prompt, params))
        expect.append(reference_output(prompt, params, eos=3))
    run_all(core)
    for r, (toks, reason) in zip(reqs, expect):
        assert r.out_tokens == toks and r.finish_reason == reason
    assert core.allocator.num_free == num_blocks
    if num_blocks == 12:
        assert core.num_preemptions > 0
    kinds = {k for k, _ in runner.batches}
    assert kinds == {"prefill", "decode"}
    assert max(n for _, n in runner.batches) <= 6


def test_max_model_len_and_validation():
    core = EngineCore(FakeRunner(100), 100, max_model_len=20)
    with pytest.raises(ValueError):
        core.add_request(list(range(20)), RequestParams(max_tokens=5))
    with pytest.raises(ValueError):
        core.add_request([], RequestParams())
    r = core.add_request(list(range(15)), RequestParams(max_tokens=50, ignore_eos=True))
    run_all(core)
    assert r.finish_reason == "length" and r.num_tokens == 20


def test_abort_returns_partial_tokens():
    core = EngineCore(FakeRunner(100), 100, max_num_seqs=1)
    a = core.add_request([1, 2, 3], RequestParams(max_tokens=50, ignore_eos=True))
    b = core.add_request([4, 5], RequestParams(max_tokens=50, ignore_eos=True))
    for _ in range(4):
        core.step()
    core.abort_all()
    assert a.finish_reason == "abort" and len(a.out_tokens) == 4
    assert b.finish_reason == "abort" and b.out_tokens == []  # was waiting (max_num_seqs=1)
    assert core.allocator.num_free == 100 and not core.has_unfinished()


def fake_engine(num_blocks=200, max_num_seqs=8, eos=None, max_model_len=256):
    model = SimpleNamespace(max_model_len=max_model_len, spec=SimpleNamespace(eos_token_id=eos))
    return AMDInferenceEngine(model, num_blocks=num_blocks, max_num_seqs=max_num_seqs,
                              runner=FakeRunner(num_blocks))


def test_async_generate_and_sample():
    eng = fake_engine(eos=3)
    prompts = [[1, 2], [3, 4, 5], [6]]
    sp = {"max_tokens": 10, "min_tokens": 1, "logprobs": 0}
    out = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": sp}))
    for p, ids, reason in zip(prompts, out["response_ids"], out["stop_reasons"]):
        exp, er = reference_output(p, RequestParams.from_dict(sp), eos=3)
        assert ids == exp and reason == er
    assert len(out["response_logprobs"]) == 3 and len(out["response_logprobs"][0]) == len(out["response_ids"][0])
    out2 = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": {"max_tokens": 2}}))
    assert out2["response_logprobs"] is None
    s = asyncio.run(eng.sample([1, 2], 3, {"max_tokens": 4}))
    assert len(s["response_ids"]) == 3
    with pytest.raises(ValueError):
        asyncio.run(eng.generate({"prompts": [[{"role": "user", "content": "x"}]], "prompt_token_ids": None}))


def test_concurrent_generate_calls_share_the_engine():
    eng = fake_engine(max_num_seqs=4)

    async def main():
        calls = [eng.generate({"prompt_token_ids": [[i, i + 1]], "sampling_params": {"max_tokens": 6 + i}})
                 for i in range(7)]
        return await asyncio.gather(*calls)

    outs = asyncio.run(main())
    for i, o in enumerate(outs):
        exp, _ = reference_output([i, i + 1], RequestParams(max_tokens=6 + i))
        assert o["response_ids"][0] == exp


def test_route_prompts_to_engines():
    assert route_prompts_to_engines(5, 2, None) == {0: [0, 1, 2], 1: [3, 4]}
    r = route_prompts_to_engines(4, 3, ["a", "b", "a", 7])
    assert sorted(i for v in r.values() for i in v) == [0, 1, 2, 3]
    assert [k for k, v in r.items() if 0 in v] == [k for k, v in r.items() if 2 in v]
    assert len(route_prompts_to_engines(1, 4, None)) == 1


def test_client_pause_abort_resume_retry():
    """A single-prompt generate() interrupted by pause_generation returns the same tokens as
    an uninterrupted one: the aborted partial is resent as prompt + accumulated tokens."""
    eng = fake_engine()
    client = InferenceEngineClient([eng], abort_grace_seconds=0.0)
    sp = {"max_tokens": 40, "logprobs": 0, "ignore_eos": True}
    exp, _ = reference_output([9, 8, 7], RequestParams.from_dict(sp))

    async def main():
        task = asyncio.create_task(client.generate({"prompt_token_ids": [[9, 8, 7]], "sampling_params": sp}))
        for _ in range(10):
            await asyncio.sleep(0)
        await client.pause_generation()
        assert eng.core.num_steps > 0
        await asyncio.sleep(0.01)
        await client.resume_generation()
        return await task

    out = asyncio.run(main())
    assert out["response_ids"][0] == exp and out["stop_reasons"] == ["length"]
    assert len(out["response_logprobs"][0]) == 40
    with pytest.raises(RuntimeError):
        asyncio.run(client.resume_generation())


def test_client_batched_generate_over_two_engines():
    engines = [fake_engine(), fake_engine()]
    client = InferenceEngineClient(engines)
    prompts = [[i, 2 * i + 1] for i in range(5)]
    out = asyncio.run(client.generate({"prompt_token_ids": prompts, "sampling_params": {"max_tokens": 5}}))
    for p, ids in zip(prompts, out["response_ids"]):
        assert ids == reference_output(p, RequestParams(max_tokens=5))[0]
    assert client.dp_size() == 2


def test_decoder_hf_weight_names_round_trip():
    """PagedDecoder stores q/k/v and gate/up fused; HF state-dict names load into the right
    slices and come back out unchanged (host-side mapping only, CPU tensors)."""
    import torch
    from transformers import AutoModelForCausalLM, Qwen2Config

    from skyrl_amd.inference_engines.model import PagedDecoder

    cfg = Qwen2Config(vocab_size=101, hidden_size=256, intermediate_size=384, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=64,
                      tie_word_embeddings=True)
    torch.manual_seed(0)
    hf = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    sd = {k: v + 0.01 * torch.randn_like(v) for k, v in hf.state_dict().items()}
    m = PagedDecoder(cfg, "cpu", seed=None)
    assert m.load_weights(sd.items()) == len(sd) - 1  # tied lm_head is skipped, as vLLM does
    ours = dict(m.hf_named_tensors())
    for k, v in sd.items():
        if k != "lm_head.weight":
            assert torch.equal(ours[k], v), k
    with pytest.raises(KeyError):
        m.load_weights([("model.layers.9.mlp.up_proj.weight", sd["model.layers.0.mlp.up_proj.weight"])])
    with pytest.raises(ValueError):
        m.load_weights([("model.norm.weight", torch.zeros(3))])


def test_model_runner_stages_decode_rows():
    """ModelRunner's host staging (CPU tensors, no kernel call): idle rows get slot -1 and
    context 1; running rows get their last token, position, slot and block-table row."""
    import torch
    from transformers import Qwen2Config

    from skyrl_amd.inference_engines.engine import ModelRunner, Request
    from skyrl_amd.inference_engines.model import PagedDecoder

    cfg = Qwen2Config(vocab_size=64, hidden_size=256, intermediate_size=256, num_hidden_layers=1,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=128)
    m = PagedDecoder(cfg, "cpu", seed=None)
    runner = ModelRunner(m, num_blocks=40, max_num_seqs=6)
    a = Request(rid=0, prompt=list(range(20)), params=RequestParams(), key=0, out_tokens=[7], blocks=[5, 9],
                row=0)
    b = Request(rid=1, prompt=[1, 2], params=RequestParams(), key=1, out_tokens=[3, 4], blocks=[11], row=3)
    runner._stage_decode([a, b], 4)
    tok, pos, slot = runner.d_i64[:, :4].tolist()
    assert tok == [7, 0, 0, 4] and pos == [20, 0, 0, 3]
    assert slot == [9 * 16 + 4, -1, -1, 11 * 16 + 3]
    t = runner.d_i32[:4].tolist()
    assert runner.d_ctx[:4].tolist() == [21, 1, 1, 4]
    assert t[0][0:2] == [5, 9] and t[3][0] == 11
    a.blocks.append(17)  # a new block is staged incrementally
    a.out_tokens += [1] * 12
    runner._stage_decode([a], 1)
    assert runner.d_i32[0, 0:3].tolist() == [5, 9, 17] and runner.d_i64[2, 0].item() == 17 * 16 + 0
    assert torch.equal(runner.d_ctx[:1], torch.tensor([33], dtype=torch.int32))


def test_block_allocator_prefix_cache():
    from skyrl_amd.inference_engines.engine import BlockAllocator, block_hashes

    a = BlockAllocator(4, enable_caching=True)
    b = a.allocate(2)
    h = block_hashes(list(range(40)), 2)
    assert h == block_hashes(list(range(32)) + [9] * 8, 2) and h != block_hashes(list(range(1, 41)), 2)
    a.register(b[0], h[0])
    a.register(b[1], h[1])
    a.free(b)
    assert a.num_free == 4 and a.lookup(h[0]) == b[0]  # released but still cached (evictable)
    a.acquire(b[0])
    assert a.num_free == 3
    c = a.allocate(3)  # 2 plain free blocks, then evicts the LRU cached block (b[1])
    assert b[1] in c and a.lookup(h[1]) is None and a.lookup(h[0]) == b[0]
    a.free(c + [b[0]])
    a.reset()
    assert a.lookup(h[0]) is None and a.num_free == 4


def test_prefix_caching_shares_prompt_blocks_and_keeps_outputs():
    """GRPO shape: 3 prompts x 4 samples. With the prefix cache the siblings of a prompt reuse
    its full prompt blocks (read-only) and compute only the tail; the tokens are unchanged."""
    rng = np.random.default_rng(3)
    prompts = [rng.integers(0, V, size=int(n)).tolist() for n in (40, 17, 70)]
    results = {}
    for caching in (False, True):
        runner = FakeRunner(200)
        seen_cached = []
        orig = runner.execute

        def execute(batch, orig=orig, seen=seen_cached, caching=caching):
            if batch.kind == "prefill":
                for r in batch.requests:
                    seen.append(r.num_cached)
                    k = r.num_cached // BLOCK_SIZE
                    assert r.num_cached % BLOCK_SIZE == 0 and r.num_cached < r.num_tokens
                    if caching:
                        assert len(r.block_hashes) == (r.num_tokens - 1) // BLOCK_SIZE and k <= len(r.block_hashes)
            return orig(batch)

        runner.execute = execute
        core = EngineCore(runner, 200, max_num_seqs=16, max_model_len=200, enable_prefix_caching=caching)
        reqs = [core.add_request(p, RequestParams(max_tokens=12, ignore_eos=True)) for p in prompts for _ in range(4)]
        first_blocks = {}
        while core.has_unfinished():
            core.step()
            for r in core.running:
                first_blocks.setdefault(tuple(r.prompt[:16]), set()).add(r.blocks[0])
        results[caching] = [r.out_tokens for r in reqs]
        assert core.allocator.num_free == 200
        if caching:
            assert seen_cached.count(0) == 3 and sum(c > 0 for c in seen_cached) == 9
            assert all(len(v) == 1 for v in first_blocks.values())  # siblings share block 0
            assert core.allocator.hits >= 9
    assert results[True] == results[False]


def test_apply_penalties_matches_vllm_formula():
    """ModelRunner._apply_penalties (CPU tensors, no kernel): repetition over prompt + output,
    presence / frequency over output counts, only on rows that ask for them; the saved values
    restore the raw logits exactly."""
    import torch
    from collections import Counter

    from transformers import Qwen2Config

    from skyrl_amd.inference_engines.engine import ModelRunner, Request, ScheduledBatch
    from skyrl_amd.inference_engines.model import PagedDecoder

    cfg = Qwen2Config(vocab_size=64, hidden_size=256, intermediate_size=256, num_hidden_layers=1,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=128)
    runner = ModelRunner(PagedDecoder(cfg, "cpu", seed=None), num_blocks=8, max_num_seqs=4)
    g = torch.Generator().manual_seed(2)
    V = 64
    raw = (torch.randn(3, V, generator=g) * 2).to(torch.bfloat16)
    pen = RequestParams(repetition_penalty=1.3, presence_penalty=0.5, frequency_penalty=0.25)
    reqs = [Request(rid=0, prompt=[1, 2, 3], params=pen, key=0, out_tokens=[3, 3, 9, 40], row=0),
            Request(rid=1, prompt=[5], params=RequestParams(), key=1, out_tokens=[5, 6], row=1),
            Request(rid=2, prompt=[7, 8], params=RequestParams(presence_penalty=-1.0), key=2, out_tokens=[8, 8],
                    row=2)]
    logits = raw.clone()
    batch = ScheduledBatch("decode", reqs, np.zeros(3, dtype=np.int64), [(), (), ()])
    flat, saved, prow = runner._apply_penalties(logits, batch, np.arange(3))
    assert prow.tolist() == [0, 2]
    exp = raw.float().clone()
    for i, r in ((0, reqs[0]), (2, reqs[2])):
        p, c = r.params, Counter(r.out_tokens)
        for t in sorted(set(r.prompt) | set(c)) if p.repetition_penalty != 1.0 else sorted(c):
            x = exp[i, t]
            x = x / p.repetition_penalty if x > 0 else x * p.repetition_penalty
            exp[i, t] = x - (p.frequency_penalty * c[t] + (p.presence_penalty if c[t] else 0.0))
    torch.testing.assert_close(logits.float(), exp.to(torch.bfloat16).float())
    assert torch.equal(logits[1], raw[1])  # no penalty, untouched
    logits.view(-1).index_copy_(0, flat, saved)
    assert torch.equal(logits, raw)
