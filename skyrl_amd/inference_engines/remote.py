"""Separated placement without Ray or HTTP: a rollout engine hosted by another rank.

The reference places vLLM engines on their own GPUs and reaches them through Ray actors or an
HTTP server (remote_inference_engine.py:126-326, ray_wrapped_inference_engine.py); weights go
from the policy ranks to the engines' workers by collective broadcast
(weight_sync/broadcast_strategy.py:98-191, inference_servers/vllm_worker.py:43-96), and the
fully-async trainer pauses generation, updates and resumes it (fully_async_trainer.py:415-419).

Here the engine rank runs :func:`serve_engine` around its AMDInferenceEngine, and the trainer
rank talks to it through :class:`RemoteEngine`, an InferenceEngineInterface whose calls are
small pickled control messages over two torch.distributed point-to-point groups (requests one
way, replies the other; gloo -- they carry only token lists and metadata). Replies carry the
request id, so many generate calls can be in flight at once and an abort overtakes them, as the
in-flight weight update needs. The weights themselves never travel on the control channel:
update_named_weights sends the metadata, then every learner rank broadcasts the packed bf16
stream on the weight group (comm.ShardedBroadcastWeightSender, one shard per learner rank;
RCCL on a multi-GPU node), straight into the engine's receive buffer, whose views the engine
loads (comm.ShardedBroadcastWeightReceiver).
"""

from __future__ import annotations

import asyncio
import concurrent.futures
import itertools
import threading
from typing import Any, Dict, List, Optional, Sequence

import torch.distributed as dist

from .base import InferenceEngineInput, InferenceEngineInterface, InferenceEngineOutput


def _send(obj: Any, dst: int, group) -> None:
    dist.send_object_list([obj], dst=dst, group=group)


def _recv(src: int, group) -> Any:
    box = [None]
    dist.recv_object_list(box, src=src, group=group)
    return box[0]


class RemoteEngine(InferenceEngineInterface):
    """Trainer-side handle of an engine served by rank `peer` (global rank). `req_group` /
    `rep_group`: two gloo groups holding this rank and the peer (requests, replies);
    `weight_group` + `weight_src_ranks`: the broadcast group and the learner ranks that source
    it (every learner rank calls update_named_weights; only the one with `control=True` sends
    the control messages, once per engine)."""

    def __init__(self, peer: int, req_group, rep_group, weight_group=None, weight_src_ranks: Sequence[int] = (0,),
                 control: bool = True):
        self.peer, self.req_group, self.rep_group = peer, req_group, rep_group
        self.weight_group, self.weight_src_ranks, self.control = weight_group, list(weight_src_ranks), control
        self._ids = itertools.count()
        self._pending: Dict[int, concurrent.futures.Future] = {}
        self._lock = threading.Lock()
        self._reader: Optional[threading.Thread] = None
        self._closed = False

    # ------------------------------------------------------------------ transport
    def _read_replies(self) -> None:
        while True:
            rep = _recv(self.peer, self.rep_group)
            fut = self._pending.pop(rep["id"], None)
            # a caller that was cancelled meanwhile (a generation worker stopped while its request
            # was in flight) has cancelled the future: drop the reply, keep reading
            if fut is not None and fut.set_running_or_notify_cancel():
                if rep["ok"]:
                    fut.set_result(rep["result"])
                else:
                    fut.set_exception(RuntimeError(f"remote engine (rank {self.peer}): {rep['error']}"))
            if rep.get("last"):
                return

    def _post(self, op: str, *args: Any) -> concurrent.futures.Future:
        if not self.control:
            raise RuntimeError("this RemoteEngine handle only joins the weight broadcast (control=False)")
        if self._closed:
            raise RuntimeError("remote engine was torn down")
        fut: concurrent.futures.Future = concurrent.futures.Future()
        with self._lock:  # one sender at a time on the request group, ids in send order
            rid = next(self._ids)
            self._pending[rid] = fut
            if self._reader is None:
                self._reader = threading.Thread(target=self._read_replies, name="remote-engine-replies", daemon=True)
                self._reader.start()
            _send({"id": rid, "op": op, "args": args}, self.peer, self.req_group)
        return fut

    async def _call(self, op: str, *args: Any) -> Any:
        loop = asyncio.get_running_loop()
        fut = await loop.run_in_executor(None, self._post, op, *args)  # the send blocks until received
        return await asyncio.wrap_future(fut)

    # ------------------------------------------------------------------ interface
    async def generate(self, input_batch: InferenceEngineInput) -> InferenceEngineOutput:
        if input_batch.get("prompts") is not None or input_batch.get("prompt_token_ids") is None:
            raise ValueError("RemoteEngine only accepts `prompt_token_ids`, not `prompts` "
                             "(remote_inference_engine.py:173-175)")
        return await self._call("generate", {"prompt_token_ids": [list(p) for p in input_batch["prompt_token_ids"]],
                                             "sampling_params": dict(input_batch.get("sampling_params") or {})})

    async def sample(self, prompt_token_ids: List[int], num_samples: int,
                     sampling_params: Dict[str, Any]) -> InferenceEngineOutput:
        return await self._call("sample", list(prompt_token_ids), int(num_samples), dict(sampling_params))

    async def abort_generation(self) -> None:
        await self._call("abort_generation")

    async def init_weight_update_communicator(self, init_info=None):
        """Tell the engine rank to receive from `weight_src_ranks` on its weight group."""
        if self.control:
            await self._call("init_weight_update_communicator", {"src_ranks": self.weight_src_ranks})

    async def update_named_weights(self, request):
        """request: {"names", "tensors"} (GRPOTrainer.weight_update_request). The control
        message goes first (the engine enters its receive), then this rank broadcasts its shard."""
        from ..comm import ShardedBroadcastWeightSender, WeightUpdateRequest

        names = request["names"] if isinstance(request, dict) else request.names
        tensors = request["tensors"] if isinstance(request, dict) else request.tensors
        named = list(zip(names, tensors))
        sender = ShardedBroadcastWeightSender(self.weight_src_ranks, group=self.weight_group)
        meta = WeightUpdateRequest(list(names), [str(sender.dtype)] * len(named), [list(t.shape) for t in tensors])
        fut = None
        if self.control:
            loop = asyncio.get_running_loop()
            fut = await loop.run_in_executor(None, self._post, "update_named_weights", meta.to_json_dict())
        sender.send(named)
        return await asyncio.wrap_future(fut) if fut is not None else len(named)

    async def reset_prefix_cache(self):
        return await self._call("reset_prefix_cache")

    async def sleep(self, *args: Any, **kwargs: Any):
        return await self._call("sleep", kwargs)

    async def wake_up(self, *args: Any, **kwargs: Any):
        return await self._call("wake_up", kwargs)

    async def named_weights(self) -> Dict[str, Any]:
        """The engine's weights under their HF names, as host tensors (checks and debugging)."""
        return await self._call("named_weights")

    async def teardown(self):
        if self.control and not self._closed:
            await self._call("shutdown")
            self._closed = True
            if self._reader is not None:
                self._reader.join(timeout=30)

    async def chat_completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("OpenAI HTTP endpoints are out of scope for the MI355X engine")

    async def completion(self, request_payload: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError("OpenAI HTTP endpoints are out of scope for the MI355X engine")

    def tp_size(self) -> int:
        return 1

    def pp_size(self) -> int:
        return 1

    def dp_size(self) -> int:
        return 1


async def _serve(engine, trainer_rank: int, req_group, rep_group, weight_group) -> None:
    loop = asyncio.get_running_loop()
    inbox: asyncio.Queue = asyncio.Queue()
    send_lock = asyncio.Lock()

    def reader():
        while True:
            msg = _recv(trainer_rank, req_group)
            loop.call_soon_threadsafe(inbox.put_nowait, msg)
            if msg["op"] == "shutdown":
                return

    threading.Thread(target=reader, name="engine-requests", daemon=True).start()

    async def reply(msg, ok, result=None, error=None, last=False):
        rep = {"id": msg["id"], "ok": ok, "result": result, "error": error, "last": last}
        async with send_lock:
            await loop.run_in_executor(None, _send, rep, trainer_rank, rep_group)

    async def run(msg):
        op, args = msg["op"], msg["args"]
        try:
            if op == "generate":
                out = await engine.generate(args[0])
                res = {k: out.get(k) for k in ("responses", "stop_reasons", "response_ids", "response_logprobs")}
            elif op == "sample":
                out = await engine.sample(*args)
                res = {k: out.get(k) for k in ("responses", "stop_reasons", "response_ids", "response_logprobs")}
            elif op == "abort_generation":
                res = await engine.abort_generation()
            elif op == "init_weight_update_communicator":
                from ..comm import ShardedBroadcastWeightReceiver

                rcv = ShardedBroadcastWeightReceiver(args[0]["src_ranks"], model_dtype=engine.model.dtype,
                                                     group=weight_group, device=engine.model.device)
                res = await engine.init_weight_update_communicator(rcv)
            elif op == "update_named_weights":
                from ..comm import WeightUpdateRequest

                # runs on this loop: the broadcast receive blocks generation, which the trainer
                # has paused (or not started) around an update
                res = await engine.update_named_weights(WeightUpdateRequest.from_json_dict(args[0]))
            elif op == "reset_prefix_cache":
                res = await engine.reset_prefix_cache()
            elif op == "sleep":
                res = await engine.sleep(**args[0])
            elif op == "wake_up":
                res = await engine.wake_up(**args[0])
            elif op == "named_weights":
                res = {n: t.detach().cpu() for n, t in engine.model.hf_named_tensors()}
            else:
                raise ValueError(f"unknown op {op!r}")
        except Exception as e:  # noqa: BLE001 -- reported to the caller, the server keeps serving
            await reply(msg, False, error=f"{type(e).__name__}: {e}")
            return
        await reply(msg, True, res)

    tasks = set()
    while True:
        msg = await inbox.get()
        if msg["op"] == "shutdown":
            if tasks:
                await asyncio.gather(*tasks, return_exceptions=True)
            await engine.abort_generation()
            await reply(msg, True, None, last=True)
            return
        if msg["op"] in ("update_named_weights", "init_weight_update_communicator"):
            await run(msg)  # in order with the broadcasts that follow it
        else:
            t = asyncio.create_task(run(msg))
            tasks.add(t)
            t.add_done_callback(tasks.discard)


def serve_engine(engine, trainer_rank: int, req_group, rep_group, weight_group=None) -> None:
    """Engine-rank main loop: serve `engine` to the RemoteEngine on `trainer_rank` until it
    tears the handle down."""
    asyncio.run(_serve(engine, trainer_rank, req_group, rep_group, weight_group))
