"""Ray-free mesh dispatch (reference: skyrl_train/distributed/dispatch.py).

The reference's driver holds Ray actor handles. `MeshDispatch.dispatch` cuts a
TrainingInputBatch into dp_size chunks, `ray.put`s each chunk once and calls the method on
every actor. Actors that share a DP rank (its SP/TP/PP replicas) get the same chunk
(`:123-141`). `sync_collect` / `async_collect` concatenate, in DP order, the outputs of the
actors with (sp=0, tp=0, pp=last) (`:289-307`). `dispatch_from_staged` sends one staged
full batch plus per-DP slice indices (`:164-205`). PassThroughDispatch calls every actor with
the same arguments.

Here there is one process per GPU and no Ray. The "actors" are the ranks of a
torch.distributed group, each holding its own worker object, and every call is collective
(SPMD):

  stage(data, src)                    the source rank's batch reaches every rank, once. Over
                                      RCCL it goes one broadcast per tensor, device to device
                                      (xGMI), after a pinned host -> HBM copy on the source.
                                      Over gloo it goes host to host. The metadata (keys,
                                      dtypes, shapes, batch metadata) travels as one small
                                      object broadcast.
  MeshDispatch.dispatch(...)          stage, then each rank calls worker.method(its DP chunk).
  MeshDispatch.dispatch_from_staged   no communication: each rank calls
                                      method(staged, start_idx, end_idx) on its DP slice.
  collect(...)                        gather to dst; dst concatenates the collection ranks'
                                      outputs in DP order. Other ranks get None.

The registry (`DispatchRegistry`, `register_dispatch_type`) keeps the reference's names and
errors.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple, Type

import torch
import torch.distributed as dist

from .training_batch import TensorBatch, TrainingInputBatch, TrainingOutputBatch


@dataclass
class MeshRank:
    """(DP, SP, TP, PP) coordinates of a rank (dispatch.py:14-43)."""

    dp: int
    sp: int
    tp: int
    pp: int
    world_size: int
    dp_size: int
    pp_size: int

    def is_collection_dp_rank(self) -> bool:
        """The rank whose output represents its DP group: sp = 0, tp = 0, pp = last stage."""
        return self.tp == 0 and self.pp == self.pp_size - 1 and self.sp == 0


def mesh_rank(rank: int, world_size: int, dp_size: int, sp_size: int = 1, tp_size: int = 1,
              pp_size: int = 1) -> MeshRank:
    """Coordinates of a global rank with tp fastest, then sp, then pp, then dp. TP peers are
    then neighbouring ranks, i.e. neighbouring GPUs of one node on its xGMI links."""
    if dp_size * sp_size * tp_size * pp_size != world_size:
        raise ValueError(f"dp*sp*tp*pp = {dp_size * sp_size * tp_size * pp_size} != world_size {world_size}")
    tp = rank % tp_size
    sp = (rank // tp_size) % sp_size
    pp = (rank // (tp_size * sp_size)) % pp_size
    dp = rank // (tp_size * sp_size * pp_size)
    return MeshRank(dp=dp, sp=sp, tp=tp, pp=pp, world_size=world_size, dp_size=dp_size, pp_size=pp_size)


@dataclass
class ActorInfo:
    """A rank's local worker object and its mesh coordinates (the reference's actor handle
    becomes the object the method is called on in this process)."""

    handle: Any
    rank: MeshRank


def _world(group) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def stage(data: Optional[TensorBatch], group=None, src: int = 0, device: Optional[torch.device] = None) -> TensorBatch:
    """Every rank gets the src rank's batch (the staged object of dispatch_from_staged).

    With an "nccl" (RCCL) group the tensors land on ``device`` (default: the current GPU). The
    source copies them host -> HBM from pinned memory, then one broadcast per tensor runs over
    xGMI. With gloo they stay on the host."""
    rank, world = _world(group)
    if world == 1:
        if data is None:
            raise ValueError("stage: the source rank must pass the batch")
        return data
    backend = dist.get_backend(group)
    on_gpu = backend == "nccl"
    if on_gpu and device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    gsrc = dist.get_global_rank(group, src) if group is not None else src
    if rank == src:
        if data is None:
            raise ValueError("stage: the source rank must pass the batch")
        header = {"cls": type(data).__name__, "metadata": data.metadata,
                  "fields": [(k, None if v is None else (str(v.dtype).replace("torch.", ""), tuple(v.shape)))
                             for k, v in data.items()]}
    else:
        header = None
    box = [header]
    dist.broadcast_object_list(box, src=gsrc, group=group)
    header = box[0]
    out: Dict[str, Optional[torch.Tensor]] = {}
    for key, spec in header["fields"]:
        if spec is None:
            out[key] = None
            continue
        dtype, shape = getattr(torch, spec[0]), spec[1]
        if rank == src:
            t = data[key].contiguous()
            if on_gpu and t.device.type != "cuda":
                t = t.pin_memory().to(device, non_blocking=True)
            elif not on_gpu and t.device.type != "cpu":
                t = t.cpu()
        else:
            t = torch.empty(shape, dtype=dtype, device=device if on_gpu else "cpu")
        dist.broadcast(t, src=gsrc, group=group)
        out[key] = t
    cls = {"TrainingInputBatch": TrainingInputBatch, "TrainingOutputBatch": TrainingOutputBatch}.get(
        header["cls"], TensorBatch)
    batch = cls(out)
    batch.metadata = header["metadata"]
    return batch


def concatenate_outputs_after_mesh_dispatch(mesh_ranks: List[MeshRank],
                                            data_batches: List[Optional[TensorBatch]]) -> TensorBatch:
    """dispatch.py:289-307: the collection ranks' outputs, concatenated in DP order."""
    assert len(mesh_ranks) == len(data_batches), "`mesh_ranks` and `data_batches` must have the same length"
    by_dp = {}
    for r, b in zip(mesh_ranks, data_batches):
        if r.is_collection_dp_rank():
            by_dp[r.dp] = b
    return TrainingOutputBatch.cat([by_dp[i] for i in range(mesh_ranks[0].dp_size)])


def collect(me: MeshRank, output: Optional[TensorBatch], group=None, dst: int = 0) -> Optional[TensorBatch]:
    """Gather every rank's output (host wire format) to dst and concatenate there; None on the
    other ranks, or everywhere when every rank returned None. A mix of None and batches is an
    error, as sync_collect (:154-161)."""
    rank, world = _world(group)
    if output is not None and output.device is not None and output.device.type != "cpu":
        output = output.to("cpu")
    if world == 1:
        gathered, ranks = [output], [me]
    else:
        gathered = [None] * world if rank == dst else None
        gdst = dist.get_global_rank(group, dst) if group is not None else dst
        dist.gather_object((me, output), gathered, dst=gdst, group=group)
        if rank != dst:
            return None
        ranks = [g[0] for g in gathered]
        gathered = [g[1] for g in gathered]
    if all(g is None for g in gathered):
        return None
    assert all(g is not None for g in gathered), "Got a mix of `None` and non-`None` objects"
    return concatenate_outputs_after_mesh_dispatch(ranks, gathered)


class Dispatch(ABC):
    """dispatch.py:56-93, collective form: every rank of the group calls dispatch with its own
    ActorInfo (local worker + mesh rank) and gets its local result back. collect is
    collective too."""

    @classmethod
    @abstractmethod
    def dispatch(cls, actor_info: ActorInfo, method: str, *args, **kwargs) -> Any:
        ...

    @classmethod
    def sync_collect(cls, actor_info: ActorInfo, output: Any, group=None, dst: int = 0) -> Optional[TensorBatch]:
        return collect(actor_info.rank, output, group, dst)

    @classmethod
    async def async_collect(cls, actor_info: ActorInfo, output: Any, group=None, dst: int = 0):
        return collect(actor_info.rank, output, group, dst)

    @classmethod
    def validate_dispatch_args(cls, *args, **kwargs) -> Tuple[Tuple, Dict[str, Any]]:
        return args, kwargs


class MeshDispatch(Dispatch):
    """Data-parallel dispatch (dispatch.py:96-222): the batch is cut into dp_size equal chunks
    and every rank of DP group d runs the method on chunk d."""

    @classmethod
    def dispatch(cls, actor_info: ActorInfo, method: str, data: Optional[TrainingInputBatch] = None, group=None,
                 src: int = 0, **kwargs) -> Any:
        staged = stage(data, group, src)
        dp_size = actor_info.rank.dp_size
        assert len(staged) % dp_size == 0, "data batch size must be divisible by dp_size, got {} and {}".format(
            len(staged), dp_size)
        chunk = len(staged) // dp_size
        d = actor_info.rank.dp
        return getattr(actor_info.handle, method)(staged.slice(d * chunk, (d + 1) * chunk), **kwargs)

    @classmethod
    def dispatch_from_staged(cls, actor_info: ActorInfo, method: str, data_ref: TensorBatch, start_idx: int,
                             end_idx: int, **kwargs) -> Any:
        """:164-205 without the object store: ``data_ref`` is the staged batch every rank
        already holds; the method receives it with this DP rank's slice indices."""
        dp_size = actor_info.rank.dp_size
        mini = end_idx - start_idx
        assert mini % dp_size == 0, f"mini_batch_size must be divisible by dp_size, got {mini} and {dp_size}"
        chunk = mini // dp_size
        ws = start_idx + actor_info.rank.dp * chunk
        return getattr(actor_info.handle, method)(data_ref, start_idx=ws, end_idx=ws + chunk, **kwargs)

    @classmethod
    def validate_dispatch_args(cls, *args, **kwargs) -> Tuple[Tuple, Dict[str, Any]]:
        if args:
            data, rest = args[0], kwargs
        elif "data" in kwargs:
            data = kwargs.pop("data")
            rest = kwargs
        else:
            raise ValueError("MeshDispatch requires 'data' as first positional argument or keyword argument")
        if not isinstance(data, TrainingInputBatch):
            raise ValueError(f"For MeshDispatch, `data` entry should be a `TrainingInputBatch`, got {type(data)}")
        return (data,), rest


class PassThroughDispatch(Dispatch):
    """The same arguments on every rank (dispatch.py:225-260)."""

    @classmethod
    def dispatch(cls, actor_info: ActorInfo, method: str, *args, **kwargs) -> Any:
        return getattr(actor_info.handle, method)(*args, **kwargs)


class DispatchRegistry:
    _registry: Dict[str, Type[Dispatch]] = {"mesh": MeshDispatch, "pass_through": PassThroughDispatch}

    @classmethod
    def register(cls, name: str, dispatch_class: Type[Dispatch]) -> None:
        assert issubclass(dispatch_class, Dispatch)
        cls._registry[name] = dispatch_class

    @classmethod
    def get(cls, name: str) -> Type[Dispatch]:
        if name not in cls._registry:
            raise KeyError(f"Dispatch type '{name}' not registered")
        return cls._registry[name]

    @classmethod
    def list_registered(cls) -> Dict[str, Type[Dispatch]]:
        return cls._registry


def register_dispatch_type(name: str, dispatch_class: Type) -> None:
    DispatchRegistry.register(name, dispatch_class)
