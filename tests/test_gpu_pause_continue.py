"""Pause / continue / abort through the client, mirroring the reference's
`tests/gpu/gpu_ci/test_pause_and_continue_generation.py`:

* test_continue_generation_generate (ref :171-262): 6 concurrent single-prompt generate() calls
  over 2 engines with max_num_seqs=2 (per engine 2 run, 1 waits), paused and resumed twice
  mid-flight; every output finishes "length" with exactly max_tokens ids and logprobs, and the
  text is the decode of the ids.
* test_abort_generation (ref :265-356): 4 long requests straight to engine 0 with
  max_num_seqs=2, then pause: all 4 come back "abort", the 2 that never ran with 0 tokens.

The reference waits a fixed second before pausing; here the test waits until the running rows
have produced tokens, so the outcome does not depend on how fast the box decodes.
"""

import asyncio

import pytest
import torch

from skyrl_amd.inference_engines.client import InferenceEngineClient
from skyrl_amd.inference_engines.engine import AMDInferenceEngine
from skyrl_amd.inference_engines.model import PagedDecoder

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


class IdTokenizer:
    """decode() only (what the engine and the client's retry path call)."""

    def decode(self, ids, skip_special_tokens=True):
        return " ".join(str(int(i)) for i in ids)


def make_engine(seed, max_num_seqs=2, max_len=2048):
    from transformers import Qwen2Config

    cfg = Qwen2Config(vocab_size=1031, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=max_len,
                      tie_word_embeddings=True, eos_token_id=2)
    m = PagedDecoder(cfg, DEV, seed=7, max_model_len=max_len)  # same weights on every engine
    return AMDInferenceEngine(m, num_blocks=1024, max_num_seqs=max_num_seqs, seed=seed, tokenizer=IdTokenizer())


async def wait_for_progress(engines, min_tokens, timeout=60.0):
    """Until every engine holding requests has its running rows at >= min_tokens each (the
    client routes single prompts at random, so an engine may hold none)."""
    loop = asyncio.get_running_loop()
    t0 = loop.time()
    while True:
        cores = [e.core for e in engines if e.core.has_unfinished()]
        if cores and all(c.running and all(len(r.out_tokens) >= min_tokens for r in c.running) for c in cores):
            return
        assert loop.time() - t0 < timeout, "engines made no progress"
        await asyncio.sleep(0.005)


def test_continue_generation_generate():
    engines = [make_engine(0), make_engine(1)]
    tok = IdTokenizer()
    client = InferenceEngineClient(engines, tok, abort_grace_seconds=0.0)
    max_tokens = 768
    sp = {"max_tokens": max_tokens, "ignore_eos": True, "temperature": 0.0, "logprobs": 0}
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(3, 1031, (int(n),), generator=g).tolist() for n in (5, 17, 33, 9, 64, 12)]

    async def run():
        tasks = [asyncio.create_task(client.generate({"prompt_token_ids": [p], "sampling_params": sp}))
                 for p in prompts]
        for k in range(2):  # pause and resume twice in the middle
            await wait_for_progress(engines, 32 * (k + 1))
            await client.pause_generation()
            for e in engines:
                assert not e.core.has_unfinished()  # everything aborted back to the client
            await asyncio.sleep(0.05)
            await client.resume_generation()
        return await asyncio.gather(*tasks)

    outs = asyncio.run(run())
    assert len(outs) == len(prompts)
    for i, out in enumerate(outs):
        assert len(out["responses"]) == len(out["response_ids"]) == len(out["stop_reasons"]) == 1
        assert out["stop_reasons"][0] == "length", (i, out["stop_reasons"])
        ids = out["response_ids"][0]
        assert len(ids) == max_tokens, (i, len(ids))
        assert out["response_logprobs"] is not None and len(out["response_logprobs"][0]) == max_tokens
        assert all(lp <= 0.0 for lp in out["response_logprobs"][0])
        assert out["responses"][0] == tok.decode(ids)


def test_abort_generation():
    engine = make_engine(0)
    client = InferenceEngineClient([engine], IdTokenizer(), abort_grace_seconds=0.0)
    sp = {"max_tokens": 1900, "ignore_eos": True}
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(3, 1031, (20,), generator=g).tolist() for _ in range(4)]

    async def run_requests_then_pause():
        tasks = [asyncio.create_task(engine.generate({"prompt_token_ids": [p], "sampling_params": sp}))
                 for p in prompts]
        await wait_for_progress([engine], 4)
        assert len(engine.core.running) == 2 and len(engine.core.waiting) == 2
        await client.pause_generation()
        return await asyncio.gather(*tasks)

    outs = asyncio.run(run_requests_then_pause())
    assert all(o["stop_reasons"] == ["abort"] for o in outs)
    n_zero = sum(len(o["response_ids"][0]) == 0 for o in outs)
    assert n_zero == 2, [len(o["response_ids"][0]) for o in outs]
    assert all(0 < len(o["response_ids"][0]) < 1900 for o in outs if o["response_ids"][0])
    asyncio.run(client.resume_generation())
    # the engine serves again after the abort
    out = asyncio.run(engine.generate({"prompt_token_ids": [prompts[0]], "sampling_params": {"max_tokens": 5}}))
    assert out["stop_reasons"] == ["length"] and len(out["response_ids"][0]) == 5
