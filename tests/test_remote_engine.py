"""Separated placement protocol (skyrl_amd/inference_engines/remote.py) on CPU over gloo.

Three ranks: learners 0 and 1 (both source the weight broadcast, rank 0 also drives the
control channel), engine rank 2 serving a host-memory stand-in engine whose next token is a
function of the sequence so far (so an aborted and retried request must end with exactly the
tokens of an uninterrupted one). Checked, against the reference's semantics
(inference_engine_client.py:223-330 retry, :597-628 pause/abort, broadcast_strategy.py:98-191,
fully_async_trainer.py:415-419):
  * concurrent generate calls are answered by id, in any order;
  * an abort overtakes in-flight generations (stop reason "abort", partial tokens);
  * pause -> update -> resume through InferenceEngineClient: the paused request is retried with
    its accumulated tokens and ends identical to an uninterrupted one;
  * the engine's weights after the two-source sharded broadcast equal the learners' bit for bit;
  * errors raised on the engine rank reach the caller; teardown ends the server.
The GPU version (a real AMDInferenceEngine fed by GRPOTrainer / FullyAsyncGRPOTrainer) is
tests/test_gpu_separated.py.
"""

import asyncio
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Model:
    dtype = torch.bfloat16
    device = torch.device("cpu")

    def __init__(self):
        self.w = {"a.weight": torch.zeros(3, 5, dtype=torch.bfloat16), "b.bias": torch.zeros(7, dtype=torch.bfloat16)}

    def hf_named_tensors(self):
        return list(self.w.items())

    def load_weights(self, named):
        n = 0
        for name, t in named:
            self.w[name].copy_(t)
            n += 1
        return n


def _next_token(seq):
    return (sum(seq) * 31 + len(seq)) % 97 + 2


class _FakeEngine:
    """Emits one token per 5 ms of asyncio time; abort_generation ends the running requests."""

    def __init__(self):
        self.model = _Model()
        self.epoch = 0
        self._rcv = None

    async def generate(self, batch):
        mt = int(batch["sampling_params"].get("max_tokens", 8))
        if batch["sampling_params"].get("raise"):
            raise ValueError("bad sampling params")
        ep = self.epoch
        outs, reasons = [], []
        for p in batch["prompt_token_ids"]:
            seq, out, reason = list(p), [], "length"
            while len(out) < mt:
                await asyncio.sleep(0.005)
                if self.epoch != ep:
                    reason = "abort"
                    break
                out.append(_next_token(seq))
                seq.append(out[-1])
            outs.append(out)
            reasons.append(reason)
        return {"responses": [""] * len(outs), "stop_reasons": reasons, "response_ids": outs,
                "response_logprobs": [[-1.0] * len(o) for o in outs]}

    async def abort_generation(self):
        self.epoch += 1

    async def init_weight_update_communicator(self, rcv):
        self._rcv = rcv

    async def update_named_weights(self, request):
        return self.model.load_weights(self._rcv.receive_weights(request))

    async def reset_prefix_cache(self):
        return None


def _uninterrupted(prompt, n):
    seq, out = list(prompt), []
    for _ in range(n):
        out.append(_next_token(seq))
        seq.append(out[-1])
    return out


def _case(rank, world):
    from skyrl_amd.inference_engines.client import InferenceEngineClient
    from skyrl_amd.inference_engines.remote import RemoteEngine, serve_engine

    req = dist.new_group([0, 2], backend="gloo")
    rep = dist.new_group([0, 2], backend="gloo")
    wg = dist.new_group([0, 1, 2], backend="gloo")
    g = torch.Generator().manual_seed(3)
    new_w = [("a.weight", torch.randn(3, 5, generator=g).to(torch.bfloat16)),
             ("b.bias", torch.randn(7, generator=g).to(torch.bfloat16))]
    request = {"names": [n for n, _ in new_w], "tensors": [t for _, t in new_w]}
    if rank == 2:
        serve_engine(_FakeEngine(), 0, req, rep, wg)
        return
    if rank == 1:  # second learner: joins the broadcasts only
        remote = RemoteEngine(2, None, None, wg, weight_src_ranks=[0, 1], control=False)
        for _ in range(2):
            assert asyncio.run(remote.update_named_weights(request)) == 2
        return

    remote = RemoteEngine(2, req, rep, wg, weight_src_ranks=[0, 1])

    async def main():
        await remote.init_weight_update_communicator(None)
        # concurrent calls, replies matched by id
        prompts = [[5, 6, 7], [9], [11, 12], [4, 4, 4, 4]]
        outs = await asyncio.gather(*[remote.generate({"prompt_token_ids": [p], "sampling_params": {"max_tokens": 6}})
                                      for p in prompts])
        for p, o in zip(prompts, outs):
            assert o["response_ids"][0] == _uninterrupted(p, 6) and o["stop_reasons"] == ["length"]
        # an abort overtakes in-flight generations
        slow = [asyncio.create_task(remote.generate({"prompt_token_ids": [p], "sampling_params": {"max_tokens": 400}}))
                for p in prompts]
        await asyncio.sleep(0.2)
        await remote.abort_generation()
        got = await asyncio.gather(*slow)
        for p, o in zip(prompts, got):
            assert o["stop_reasons"] == ["abort"] and 0 < len(o["response_ids"][0]) < 400
            assert o["response_ids"][0] == _uninterrupted(p, len(o["response_ids"][0]))
        # callers cancelled while their requests are in flight (stopped generation workers): the
        # late replies are dropped and the channel keeps serving
        gone = [asyncio.create_task(remote.generate({"prompt_token_ids": [p], "sampling_params": {"max_tokens": 400}}))
                for p in prompts]
        await asyncio.sleep(0.1)
        for t in gone:
            t.cancel()
        await asyncio.gather(*gone, return_exceptions=True)
        await remote.abort_generation()
        o = await remote.generate({"prompt_token_ids": [[3]], "sampling_params": {"max_tokens": 5}})
        assert o["response_ids"][0] == _uninterrupted([3], 5)
        # pause -> update -> resume with a request in flight (client retry, token-in/token-out)
        client = InferenceEngineClient([remote], abort_grace_seconds=0.0)
        t = asyncio.create_task(client.generate({"prompt_token_ids": [[8, 1]], "sampling_params": {"max_tokens": 60}}))
        await asyncio.sleep(0.1)
        await client.pause_generation()
        assert await client.update_named_weights(request) == [2]
        await client.resume_generation()
        out = await t
        assert out["stop_reasons"] == ["length"] and out["response_ids"][0] == _uninterrupted([8, 1], 60)
        w = await remote.named_weights()
        for n, ten in new_w:
            assert torch.equal(w[n].view(torch.int16), ten.view(torch.int16)), n
        # an update without a pause, then a remote error surfaces here
        assert await remote.update_named_weights(request) == 2
        with pytest.raises(RuntimeError, match="bad sampling params"):
            await remote.generate({"prompt_token_ids": [[1]], "sampling_params": {"raise": True}})
        await remote.teardown()

    asyncio.run(main())


def _entry(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _case(rank, world)
    finally:
        dist.destroy_process_group()


def test_remote_engine_protocol_three_ranks():
    mp.spawn(_entry, args=(3, _free_port()), nprocs=3, join=True)
