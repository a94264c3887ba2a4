"""a12–a14: the learner's data-parallel exchanges over RCCL (xGMI), one process per GPU.

Reference call sites (skyrl-train/skyrl_train/):
  a12 DP gradient reduce   FSDP2 reduce-scatter, fp32 reduce dtype (distributed/fsdp_strategy.py:216-226,
                           253-271), 1/n_micro scaling (workers/worker.py:900-925), clip
                           (distributed/fsdp_utils.py:388-401), AdamW (fsdp_strategy.py:284-296)
  a13 metric all-reduce    workers/worker_utils.py:25-35 -> distributed/strategy.py:70-95 (one
                           collective per scalar, mean = pre-divide + SUM)
  a14 weight sync          weight_sync/broadcast_strategy.py:98-191 (per-parameter broadcast + RPC),
                           weight_sync/base.py (WeightChunk / WeightUpdateRequest),
                           workers/fsdp/fsdp_worker.py:201-228 (learner -> rollout)

MI355X design:
  * The flat fp32 gradient is cut into buckets (default 256 MiB: xGMI rings are per-link
    bound, so few large collectives beat many small ones). Each bucket is reduce-scattered
    on a dedicated comm stream as soon as the compute stream marks it ready, so the
    exchange overlaps whatever the compute stream does next.
  * The optimizer is sharded like FSDP2: rank r owns piece r of every bucket. Its master
    fp32 weights, Adam moments and gradient shard are one contiguous buffer in that
    bucket-interleaved order, so one HIP launch updates the whole shard (skyrl_adamw_*).
  * The same update pass writes the bf16 copy of the shard; per-bucket all-gathers of it
    ARE the colocated learner -> rollout weight sync (a14) -- no separate extraction
    pass and no per-parameter RPC.
  * Metrics: every mean goes into one packed SUM all-reduce, min and max share one MAX
    all-reduce (min x = -max -x): two collectives per call instead of one per scalar.
  * Separated placement (rollout GPUs outside the learner group): parameters are packed
    into ~1 GiB bf16 chunks and broadcast once per chunk (BroadcastWeightSender /
    BroadcastWeightReceiver), receivers get zero-copy views of the chunk buffer.

Everything here is stream-ordered: no host synchronisation except where the reference
itself reads a scalar (grad_norm().item() in optim_step).
"""

from __future__ import annotations

import ctypes
import math
import os
from dataclasses import asdict, dataclass
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 256 << 20
_ALIGN = 64  # elements: keeps every shard piece 256-B aligned for the 16-B vector kernels


def _world(group) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _collective(world: int) -> bool:
    """True when the exchanges must run as collectives. World size 1 normally short-cuts them;
    ``SKYRL_FORCE_COLLECTIVES=1`` under an initialized one-rank group keeps them, so the RCCL
    code path (comm-stream reduce-scatter / all-gather / all-reduce) runs on a one-GPU box."""
    if world > 1:
        return True
    return (os.environ.get("SKYRL_FORCE_COLLECTIVES", "0") == "1" and dist.is_available()
            and dist.is_initialized())


# ------------------------------------------------------------------------------------ a13
def all_reduce_metrics(metrics: Dict[str, float], group=None, device=None) -> Dict[str, float]:
    """Mirror of ``all_reduce_metrics`` (worker_utils.py:25-35): keys ending in ``_min`` are
    min-reduced, ``_max`` max-reduced, the rest averaged over ranks. Two collectives total."""
    world, _ = _world(group)
    if not _collective(world) or not metrics:
        return {k: float(v) for k, v in metrics.items()}
    keys = list(metrics)
    mean_keys = [k for k in keys if not (k.endswith("_min") or k.endswith("_max"))]
    ext_keys = [k for k in keys if k.endswith("_min") or k.endswith("_max")]
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    out: Dict[str, float] = {}
    if mean_keys:
        t = torch.tensor([float(metrics[k]) for k in mean_keys], dtype=torch.float32, device=device)
        t /= world  # strategy.py:85-87: pre-divide, then SUM
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        out.update(zip(mean_keys, t.tolist()))
    if ext_keys:
        sign = [-1.0 if k.endswith("_min") else 1.0 for k in ext_keys]
        t = torch.tensor([s * float(metrics[k]) for s, k in zip(sign, ext_keys)], dtype=torch.float32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        out.update({k: s * v for s, k, v in zip(sign, ext_keys, t.tolist())})
    return {k: out[k] for k in keys}


# ------------------------------------------------------------------------------------ a12
class FlatLayout:
    """Flat parameter index space cut into buckets, each a multiple of world * _ALIGN elements.

    Shard layout: rank r owns piece r of every bucket, concatenated in bucket order.
    """

    def __init__(self, numel: int, world: int, bucket_numel: int):
        if numel <= 0:
            raise ValueError("numel must be positive")
        unit = world * _ALIGN
        self.numel = numel
        self.world = world
        self.padded = int(math.ceil(numel / unit) * unit)
        bucket_numel = max(unit, (bucket_numel // unit) * unit)
        self.buckets: List[Tuple[int, int]] = []
        s = 0
        while s < self.padded:
            e = min(self.padded, s + bucket_numel)
            self.buckets.append((s, e))
            s = e
        self.shard_numel = self.padded // world
        # shard offset of each bucket's piece
        self.piece_off = []
        off = 0
        for s, e in self.buckets:
            self.piece_off.append(off)
            off += (e - s) // world

    def piece(self, b: int, rank: int) -> Tuple[int, int]:
        """Global [start, end) of bucket b's piece owned by rank."""
        s, e = self.buckets[b]
        n = (e - s) // self.world
        return s + rank * n, s + (rank + 1) * n

    def shard_index(self, rank: int) -> torch.Tensor:
        """Global flat index of every element of rank's shard (int64), in shard order."""
        parts = [torch.arange(*self.piece(b, rank), dtype=torch.int64) for b in range(len(self.buckets))]
        return torch.cat(parts)


class GradReducer:
    """Bucketed DP gradient reduction on a side stream (a12).

    ``grad`` is the flat fp32 gradient buffer the model's ``.grad`` tensors view. After the
    last micro-batch, :meth:`launch` reduce-scatters every bucket (SUM) on the comm stream
    into ``grad_shard``; :meth:`wait` makes the current stream wait for it. World size 1:
    the shard is the gradient itself and nothing is launched.
    """

    def __init__(self, numel: int, device, group=None, bucket_bytes: int = DEFAULT_BUCKET_BYTES,
                 dtype: torch.dtype = torch.float32):
        self.group = group
        self.world, self.rank = _world(group)
        self.collective = _collective(self.world)
        self.device = torch.device(device)
        self.layout = FlatLayout(numel, self.world, bucket_bytes // torch.tensor([], dtype=dtype).element_size())
        self.grad = torch.zeros(self.layout.padded, dtype=dtype, device=self.device)
        if self.collective:
            self.grad_shard = torch.zeros(self.layout.shard_numel, dtype=dtype, device=self.device)
        else:
            self.grad_shard = self.grad
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._done = None
        self._works = []

    def launch(self, buckets: Optional[Sequence[int]] = None) -> None:
        """Reduce-scatter the given buckets (default: all) after the work already queued on the
        current stream. Asynchronous with respect to the current stream."""
        if not self.collective:
            return
        lay = self.layout
        idx = range(len(lay.buckets)) if buckets is None else buckets
        if self.stream is not None:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(self.device))
            self.stream.wait_event(ready)
            ctx = torch.cuda.stream(self.stream)
        else:
            ctx = _null_ctx()
        with ctx:
            for b in idx:
                s, e = lay.buckets[b]
                po = lay.piece_off[b]
                out = self.grad_shard[po:po + (e - s) // self.world]
                self._works.append(dist.reduce_scatter_tensor(out, self.grad[s:e], op=dist.ReduceOp.SUM,
                                                              group=self.group, async_op=self.stream is None))
            if self.stream is not None:
                self._done = torch.cuda.Event()
                self._done.record(self.stream)

    def wait(self) -> None:
        if self._done is not None:
            torch.cuda.current_stream(self.device).wait_event(self._done)
            self._done = None
        for w in self._works:
            if w is not None and self.stream is None:
                w.wait()
        self._works = []

    def zero_grad(self) -> None:
        self.grad.zero_()


class _null_ctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


@dataclass
class AdamWConfig:
    """optimizer_config of the reference (ppo_base_config.yaml:37-44)."""

    lr: float = 1e-6
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 1e-2
    max_grad_norm: float = 1.0


class ShardedAdamW:
    """FSDP2-style sharded AdamW whose update is one HIP pass per step (a12), writing the
    bf16 rollout weights in the same pass and all-gathering them per bucket (a14).

    ``step(n_micro)`` mirrors PolicyWorkerBase.optim_step: grads *= 1/n_micro (folded into
    the update), DP mean (SUM reduce-scatter / world), clip at max_grad_norm, skip on a
    non-finite norm, AdamW. Returns the pre-clip grad norm as a device scalar.
    """

    def __init__(self, reducer: GradReducer, init_params: torch.Tensor, config: AdamWConfig = AdamWConfig(),
                 shadow_bf16: bool = True, gather_bf16: bool = True):
        from . import _ffi
        from .ops import _require_gpu

        self._ffi = _ffi
        dev = _require_gpu(reducer.grad)
        self._dev = dev
        self._gathered = None
        self.reducer = reducer
        self.cfg = config
        lay = reducer.layout
        if init_params.numel() != lay.numel:
            raise ValueError(f"init_params has {init_params.numel()} elements, layout expects {lay.numel}")
        flat = torch.zeros(lay.padded, dtype=torch.float32, device=dev)
        flat[: lay.numel] = init_params.reshape(-1).to(device=dev, dtype=torch.float32)
        if reducer.collective:
            self.param = torch.cat([flat[slice(*lay.piece(b, reducer.rank))] for b in range(len(lay.buckets))])
            del flat
        else:
            self.param = flat
        self.exp_avg = torch.zeros_like(self.param)
        self.exp_avg_sq = torch.zeros_like(self.param)
        self.weights_bf16 = torch.empty(lay.padded, dtype=torch.bfloat16, device=dev) if shadow_bf16 else None
        # gather_bf16=False (world > 1): the owner fills weights_bf16 itself (ShardedModuleOptimizer
        # casts it from the gathered fp32 master), so the update pass writes no bf16 shard
        self.gather_bf16 = gather_bf16
        if shadow_bf16 and not reducer.collective:
            self.weights_bf16.copy_(flat)
            self.shard_bf16 = self.weights_bf16
        elif shadow_bf16 and gather_bf16:
            self.shard_bf16 = self.param.to(torch.bfloat16)
            self._all_gather_weights(sync=True)
        else:
            self.shard_bf16 = None
        self.step_count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.plan = torch.zeros(int(_ffi.query("skyrl_adamw_plan_floats")), dtype=torch.float32, device=dev)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = torch.zeros(int(_ffi.query("skyrl_sumsq_workspace_bytes", lay.shard_numel)), dtype=torch.uint8,
                               device=dev)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self._dev).cuda_stream)

    def step(self, n_micro: int = 1, lr: Optional[float] = None, zero_grad: bool = True,
             seg: Optional["ParamSegments"] = None) -> torch.Tensor:
        """With ``seg`` (a module's parameters) the update is per parameter: ``seg.touched``
        (device, already reduced over ranks) selects the parameters to update, each with its own
        step count, as torch.optim.AdamW does for named parameters (skyrl_adamw_seg_*)."""
        from .ops import _ptr

        cfg = self.cfg
        r = self.reducer
        r.wait()
        g = r.grad_shard
        self._ffi.call("skyrl_sumsq", _ptr(g), g.numel(), _ptr(self.sumsq), _ptr(self._ws), self._stream())
        if r.collective:
            dist.all_reduce(self.sumsq, op=dist.ReduceOp.SUM, group=r.group)
        hp = self._ffi.AdamWParams(float(cfg.lr if lr is None else lr), float(cfg.betas[0]), float(cfg.betas[1]),
                                   float(cfg.eps), float(cfg.weight_decay), float(cfg.max_grad_norm),
                                   1.0 / (max(1, n_micro) * r.world))
        if seg is None:
            self._ffi.call("skyrl_adamw_plan", _ptr(self.sumsq), ctypes.byref(hp), _ptr(self.step_count),
                           _ptr(self.plan), _ptr(self.grad_norm), self._stream())
            self._ffi.call("skyrl_adamw_update", _ptr(self.param), _ptr(g), _ptr(self.exp_avg), _ptr(self.exp_avg_sq),
                           _ptr(self.shard_bf16), self.param.numel(), _ptr(self.plan), float(cfg.betas[0]),
                           float(cfg.betas[1]), self._stream())
        else:
            self._ffi.call("skyrl_adamw_seg_plan", _ptr(self.sumsq), ctypes.byref(hp), _ptr(seg.touched),
                           seg.nparams, _ptr(seg.param_step), _ptr(self.plan), _ptr(seg.coef), _ptr(self.grad_norm),
                           self._stream())
            self._ffi.call("skyrl_adamw_seg_update", _ptr(self.param), _ptr(g), _ptr(self.exp_avg),
                           _ptr(self.exp_avg_sq), _ptr(self.shard_bf16), self.param.numel(), _ptr(self.plan),
                           _ptr(seg.coef), _ptr(seg.start), _ptr(seg.owner), seg.nseg, _ptr(seg.tile_seg),
                           float(cfg.betas[0]), float(cfg.betas[1]), self._stream())
        if zero_grad:  # strategy.optimizer_step ends with optimizer.zero_grad()
            r.zero_grad()
        return self.grad_norm

    def sync_weights(self) -> None:
        """Start the learner -> rollout weight all-gather (bf16) on the comm stream; the rollout
        side calls :meth:`wait_weights` before it reads ``weights_bf16``."""
        if self.weights_bf16 is None or not self.reducer.collective or not self.gather_bf16:
            return
        self._all_gather_weights(sync=False)

    def wait_weights(self) -> None:
        if self._gathered is not None:
            torch.cuda.current_stream(self._dev).wait_event(self._gathered)
            self._gathered = None

    def _all_gather_weights(self, sync: bool) -> None:
        r = self.reducer
        lay = r.layout
        stream = r.stream
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self._dev))
        stream.wait_event(ready)
        with torch.cuda.stream(stream):
            for b, (s, e) in enumerate(lay.buckets):
                po = lay.piece_off[b]
                n = (e - s) // r.world
                dist.all_gather_into_tensor(self.weights_bf16[s:e], self.shard_bf16[po:po + n], group=r.group)
            self._gathered = torch.cuda.Event()
            self._gathered.record(stream)
        if sync:
            self.wait_weights()


# ------------------------------------------------------------------------------------ a14
@dataclass
class WeightChunk:
    """Mirror of weight_sync/base.py WeightChunk: one or more parameters moved together."""

    names: List[str]
    dtypes: List[str]
    shapes: List[List[int]]
    tensors: List[torch.Tensor]

    def __post_init__(self):
        if len({len(self.names), len(self.dtypes), len(self.shapes), len(self.tensors)}) != 1:
            raise ValueError("names, dtypes, shapes, tensors must have the same length")

    def __len__(self):
        return len(self.names)

    @property
    def total_numel(self) -> int:
        return sum(int(t.numel()) for t in self.tensors)


@dataclass
class WeightUpdateRequest:
    """Mirror of weight_sync/base.py WeightUpdateRequest (metadata only; data moves by broadcast)."""

    names: List[str]
    dtypes: List[str]
    shapes: List[List[int]]

    def __post_init__(self):
        if len({len(self.names), len(self.dtypes), len(self.shapes)}) != 1:
            raise ValueError(
                f"names, dtypes, shapes must have the same length. Got names={len(self.names)}, "
                f"dtypes={len(self.dtypes)}, shapes={len(self.shapes)}")

    def __len__(self):
        return len(self.names)

    def to_json_dict(self):
        return asdict(self)

    @classmethod
    def from_json_dict(cls, d):
        return cls(**d)


_DTYPES = {"torch.bfloat16": torch.bfloat16, "bfloat16": torch.bfloat16, "torch.float16": torch.float16,
           "torch.float32": torch.float32, "float32": torch.float32}


def pack_chunks(named: Iterable[Tuple[str, torch.Tensor]], chunk_bytes: int = 1 << 30,
                dtype: torch.dtype = torch.bfloat16) -> Iterator[WeightChunk]:
    """Group parameters into chunks of about ``chunk_bytes`` (reference IPC path packs 1 GB)."""
    names, shapes, tensors, nbytes = [], [], [], 0
    es = torch.tensor([], dtype=dtype).element_size()
    for name, t in named:
        if tensors and nbytes + t.numel() * es > chunk_bytes:
            yield WeightChunk(names, [str(dtype)] * len(names), shapes, tensors)
            names, shapes, tensors, nbytes = [], [], [], 0
        names.append(name)
        shapes.append(list(t.shape))
        tensors.append(t)
        nbytes += t.numel() * es
    if tensors:
        yield WeightChunk(names, [str(dtype)] * len(names), shapes, tensors)


class BroadcastWeightSender:
    """Separated placement: one broadcast per packed chunk from ``src`` over ``group``
    (reference: per-parameter broadcast + barrier, broadcast_strategy.py:98-142)."""

    def __init__(self, group=None, src: int = 0, dtype: torch.dtype = torch.bfloat16,
                 on_request: Optional[Callable[[WeightUpdateRequest], None]] = None):
        self.group, self.src, self.dtype, self.on_request = group, src, dtype, on_request

    def send_chunks(self, chunks: Iterable[WeightChunk]) -> int:
        """Returns the number of broadcasts issued."""
        n = 0
        for chunk in chunks:
            req = WeightUpdateRequest(list(chunk.names), list(chunk.dtypes), [list(s) for s in chunk.shapes])
            if self.on_request is not None:
                self.on_request(req)
            flat = torch.cat([t.detach().reshape(-1).to(self.dtype) for t in chunk.tensors])
            dist.broadcast(flat, self.src, group=self.group)
            n += 1
        return n


class BroadcastWeightReceiver:
    """Receives one packed chunk per request and yields zero-copy per-parameter views."""

    def __init__(self, model_dtype: torch.dtype = torch.bfloat16, group=None, src: int = 0, device=None):
        self.dtype, self.group, self.src = model_dtype, group, src
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))

    def receive_weights(self, request: WeightUpdateRequest) -> Iterator[Tuple[str, torch.Tensor]]:
        for d in request.dtypes:
            if _DTYPES.get(d, None) != self.dtype:
                raise AssertionError(f"dtype mismatch: request {d}, model {self.dtype}")
        sizes = [int(math.prod(s)) for s in request.shapes]
        flat = torch.empty(sum(sizes), dtype=self.dtype, device=self.device)
        dist.broadcast(flat, self.src, group=self.group)
        off = 0
        for name, shape, n in zip(request.names, request.shapes, sizes):
            yield name, flat[off:off + n].view(shape)
            off += n


# ------------------------------------------------------------- a14 sharded-source broadcast
class ShardedBroadcastWeightSender:
    """Separated placement with every learner rank as a source: the packed bf16
    parameter stream is cut into `len(src_ranks)` contiguous shards and learner rank i
    broadcasts shard i, all shards in flight at once (async collectives), so the traffic
    leaves from every learner GPU's links instead of one rank's. The reference broadcasts
    each parameter from rank 0 (broadcast_strategy.py:98-142)."""

    def __init__(self, src_ranks: Sequence[int], group=None, dtype: torch.dtype = torch.bfloat16):
        self.src_ranks, self.group, self.dtype = list(src_ranks), group, dtype

    @staticmethod
    def shard_bounds(total: int, nshards: int) -> List[Tuple[int, int]]:
        per = -(-total // nshards)
        per = -(-per // _ALIGN) * _ALIGN
        return [(min(i * per, total), min((i + 1) * per, total)) for i in range(nshards)]

    def send(self, named: Sequence[Tuple[str, torch.Tensor]]) -> "WeightUpdateRequest":
        """Every learner rank calls this with the same (name, tensor) list; returns the metadata
        the receivers need (the reference sends it by RPC)."""
        req = WeightUpdateRequest([n for n, _ in named], [str(self.dtype)] * len(named),
                                  [list(t.shape) for _, t in named])
        flat = torch.cat([t.detach().reshape(-1).to(self.dtype) for _, t in named])
        _sharded_broadcast(flat, self.src_ranks, self.group)
        return req


class ShardedBroadcastWeightReceiver:
    """Receiving side of ShardedBroadcastWeightSender: one buffer, per-shard async broadcasts
    into slices of it, then zero-copy per-parameter views."""

    def __init__(self, src_ranks: Sequence[int], model_dtype: torch.dtype = torch.bfloat16, group=None, device=None):
        self.src_ranks, self.dtype, self.group = list(src_ranks), model_dtype, group
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))

    def receive_weights(self, request: "WeightUpdateRequest") -> Iterator[Tuple[str, torch.Tensor]]:
        sizes = [int(math.prod(s)) for s in request.shapes]
        flat = torch.empty(sum(sizes), dtype=self.dtype, device=self.device)
        _sharded_broadcast(flat, self.src_ranks, self.group)
        off = 0
        for name, shape, n in zip(request.names, request.shapes, sizes):
            yield name, flat[off:off + n].view(shape)
            off += n


def _sharded_broadcast(flat: torch.Tensor, src_ranks: Sequence[int], group) -> None:
    works = []
    for (a, b), src in zip(ShardedBroadcastWeightSender.shard_bounds(flat.numel(), len(src_ranks)), src_ranks):
        if b > a:
            works.append(dist.broadcast(flat[a:b], src, group=group, async_op=True))
    for w in works:
        w.wait()


# ------------------------------------------------------------- a12 for module parameters
class BucketedGradAllReduce:
    """DP gradient mean for a module's parameters (the HF learner), overlapped with the backward.

    Every trainable fp32 parameter's ``.grad`` is a view into one of a few flat fp32 buckets
    (~``bucket_bytes``, filled in reverse parameter order, the order the backward produces
    them). :meth:`arm` before the LAST micro-batch's backward; from then on a
    post-accumulate-grad hook counts each bucket's parameters, and when a bucket is complete
    its SUM all-reduce (x 1/world) is launched on a dedicated comm stream while the backward
    continues with the earlier layers -- the reference's FSDP2 reduce-scatter per wrapped
    layer during the backward (fsdp_strategy.py:216-226,253-271). Buckets are launched
    strictly in index order, so every rank issues the same collective sequence. :meth:`wait`
    (before clipping) launches any bucket whose parameters got no gradient and makes the
    compute stream wait for the comm stream. World size 1: the buckets are still the grads'
    storage and nothing is launched.

    torch semantics are kept: a parameter that got no gradient on ANY rank during the
    mini-batch (one MAX all-reduce of per-parameter flags) has ``.grad = None`` after
    :meth:`wait`, so AdamW skips it as it would at world size 1, and :meth:`zero_grad`
    re-attaches the bucket views. :meth:`wait` raises if a ``.grad`` was detached from its
    bucket meanwhile (``zero_grad(set_to_none=True)``, a restore that assigned new tensors):
    the all-reduce would then average the stale buckets while each rank kept its own grads.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], group=None, bucket_bytes: int = 64 << 20):
        self.group = group
        self.world, _ = _world(group)
        self.collective = _collective(self.world)
        ps = [p for p in params if p.requires_grad]
        if not ps:
            raise ValueError("no trainable parameters")
        for p in ps:
            if p.dtype != torch.float32:
                raise TypeError(f"BucketedGradAllReduce keeps fp32 grads; got a {p.dtype} parameter")
        self.device = ps[0].device
        groups: List[List[torch.nn.Parameter]] = []
        cur: List[torch.nn.Parameter] = []
        size = 0
        for p in reversed(ps):
            cur.append(p)
            size += p.numel() * 4
            if size >= bucket_bytes:
                groups.append(cur)
                cur, size = [], 0
        if cur:
            groups.append(cur)
        self.buckets: List[Tuple[torch.Tensor, List[torch.nn.Parameter]]] = []
        self._bucket_of: Dict[int, int] = {}
        self._views: List[Tuple[torch.nn.Parameter, torch.Tensor]] = []
        for b, plist in enumerate(groups):
            flat = torch.zeros(sum(p.numel() for p in plist), dtype=torch.float32, device=self.device)
            off = 0
            for p in plist:
                view = flat[off:off + p.numel()].view_as(p)
                p.grad = view
                self._views.append((p, view))
                self._bucket_of[id(p)] = b
                off += p.numel()
            self.buckets.append((flat, plist))
        self._touched: set = set()  # params whose grad hook fired since the last zero_grad
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in ps]
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._armed = False
        self._pending: List[int] = []
        self._ready: List[bool] = []
        self._next = 0
        self.launched_during_backward = 0

    def arm(self) -> None:
        """Call before the backward of the mini-batch's last micro-batch."""
        if not self.collective:
            return
        self._armed = True
        self._pending = [len(pl) for _, pl in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self.launched_during_backward = 0

    def _on_grad(self, p) -> None:
        self._touched.add(id(p))
        if not self._armed:
            return
        b = self._bucket_of[id(p)]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._ready[b] = True
            while self._next < len(self.buckets) and self._ready[self._next]:
                self._launch(self._next)
                self._next += 1
                self.launched_during_backward += 1

    def _launch(self, b: int) -> None:
        flat = self.buckets[b][0]
        if self.stream is None:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            flat.mul_(1.0 / self.world)
            return
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ready)
        with torch.cuda.stream(self.stream):
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            flat.mul_(1.0 / self.world)

    def wait(self) -> int:
        """Finish the exchange (launching buckets that got no gradient); returns the number of
        buckets launched from inside the backward."""
        if not self._armed:
            return 0
        for p, view in self._views:
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                raise RuntimeError("BucketedGradAllReduce: a parameter's .grad is no longer its bucket view "
                                   "(zero_grad(set_to_none=True) or a reassigned grad); use "
                                   "BucketedGradAllReduce.zero_grad() between steps")
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        self._armed = False
        # parameters no rank produced a gradient for: None, as at world size 1
        flags = torch.tensor([1 if id(p) in self._touched else 0 for p, _ in self._views], dtype=torch.int32,
                             device=self.device)
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.group)
        for (p, _), f in zip(self._views, flags.tolist()):
            if not f:
                p.grad = None
        return self.launched_during_backward

    def zero_grad(self) -> None:
        for flat, _ in self.buckets:
            flat.zero_()
        for p, view in self._views:
            p.grad = view
        self._touched.clear()



class ParamSegments:
    """The per-parameter map of one rank's optimizer shard (skyrl_adamw_seg_update): segment s
    covers shard elements [start[s], start[s+1]) of parameter owner[s]; the shard's padding
    belongs to a pseudo-parameter (index nparams - 1) that is always updated (zeros stay zeros).
    ``touched`` i32[nparams] is written per step from the host flags (pinned, non-blocking) and
    MAX-reduced over the DP group on the device; ``param_step`` holds each parameter's AdamW
    step count (torch.optim.AdamW's per-parameter ``state["step"]``)."""

    def __init__(self, pieces: Sequence[Tuple[int, int, int]], n_real: int, shard_numel: int, device):
        import numpy as np

        from . import _ffi

        pad = n_real  # the padding's pseudo-parameter
        starts, owners = [], []
        pos = 0
        for off, n, i in sorted(pieces):
            if n <= 0:
                continue
            if off > pos:
                starts.append(pos)
                owners.append(pad)
            starts.append(off)
            owners.append(i)
            pos = off + n
        if pos < shard_numel or not starts:
            starts.append(pos)
            owners.append(pad)
        start = np.asarray(starts + [shard_numel], dtype=np.int64)
        tile = int(_ffi.query("skyrl_adamw_seg_tile"))
        tiles = np.arange(0, max(1, -(-shard_numel // tile)), dtype=np.int64) * tile
        tile_seg = np.searchsorted(start, tiles, side="right") - 1
        self.nparams = n_real + 1
        self.nseg = len(owners)
        self.start = torch.from_numpy(start).to(device)
        self.owner = torch.tensor(owners, dtype=torch.int32, device=device)
        self.tile_seg = torch.from_numpy(tile_seg.astype(np.int32)).to(device)
        self.touched = torch.ones(self.nparams, dtype=torch.int32, device=device)
        self.param_step = torch.zeros(self.nparams, dtype=torch.int32, device=device)
        self.coef = torch.zeros(2 * self.nparams, dtype=torch.float32, device=device)
        # pinned staging buffers for the host flags, each with the event of the copy that read
        # it: upload() takes a buffer whose copy has completed (event.query(), never a wait) and
        # pins a new one when none has, so the host never blocks on the device here
        self._host: List[torch.Tensor] = []
        self._ev: List[Optional[torch.cuda.Event]] = []

    def _free_buffer(self) -> int:
        for k, ev in enumerate(self._ev):
            if ev is None or ev.query():
                return k
        self._host.append(torch.ones(self.nparams, dtype=torch.int32).pin_memory())
        self._ev.append(None)
        return len(self._host) - 1

    def upload(self, flags: Sequence[bool], group=None, collective: bool = False) -> None:
        """Stage this rank's flags and (collective) MAX-reduce them over the group: no host sync
        (the staging buffer is one whose previous copy has completed; the flags are written into
        its numpy view, no per-step list -> tensor)."""
        import numpy as np

        k = self._free_buffer()
        h = self._host[k]
        hv = h.numpy()
        n = self.nparams - 1
        hv[:n] = np.fromiter(flags, dtype=np.bool_, count=n)
        hv[n] = 1  # the shard's padding pseudo-parameter is always updated
        self.touched.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.touched.device))
        self._ev[k] = ev
        if collective:
            dist.all_reduce(self.touched, op=dist.ReduceOp.MAX, group=group)


class ShardedModuleOptimizer:
    """The HIP a12/a14 path for a module's parameters (the HF learner of GRPOTrainer): the
    reference's FSDP2 reduce-scatter + clip + AdamW (fsdp_strategy.py:155-191, 216-271) with
    the grad scale of optim_step (workers/worker.py:902-924), and the bf16 copy the rollout
    engine loads (broadcast_to_inference_engines, fsdp_worker.py:201-228).

    Every trainable parameter becomes a view into flat buffers laid out in reverse parameter
    order (the order the backward produces gradients) and cut into FlatLayout buckets:
      * ``.grad``  -> GradReducer.grad (fp32); the backward accumulates into it in place;
      * ``.data``  -> the fp32 master (world 1: ShardedAdamW.param itself; world > 1 a full copy
                      re-assembled from the updated shards by an fp32 all-gather per bucket);
      * the engine -> ShardedAdamW.weights_bf16 (written by the update pass at world 1, the bf16
                      all-gather at world > 1): :meth:`named_bf16` hands out named views, no copy.
    :meth:`arm` before the last micro-batch's backward: from then on a post-accumulate-grad hook
    counts each bucket's parameters and fires the bucket's SUM reduce-scatter on the comm stream
    as soon as it is complete (buckets strictly in index order, the same collective sequence on
    every rank). :meth:`step` (n_micro) = wait, sharded grad norm + clip + AdamW in one HIP pass
    (non-finite norm: skipped on device), zero grads, re-assemble. Every parameter is updated
    step, except a parameter no rank's backward reached since the last step: like a None grad in
    torch.optim.AdamW its master weights and moments are left as they were.
    """

    def __init__(self, module: torch.nn.Module, config: AdamWConfig, group=None,
                 bucket_bytes: int = DEFAULT_BUCKET_BYTES):
        named = []
        seen = set()
        for n, p in module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                named.append((n, p))
        if not named:
            raise ValueError("no trainable parameters")
        for n, p in named:
            if p.dtype != torch.float32:
                raise TypeError(f"ShardedModuleOptimizer keeps an fp32 master; {n} is {p.dtype}")
        self.named = list(reversed(named))  # backward order
        dev = self.named[0][1].device
        numel = sum(p.numel() for _, p in self.named)
        self.reducer = GradReducer(numel, dev, group=group, bucket_bytes=bucket_bytes)
        lay = self.reducer.layout
        self.world, self.rank = self.reducer.world, self.reducer.rank
        self.collective = self.reducer.collective
        self.offsets = []
        off = 0
        init = torch.empty(numel, dtype=torch.float32, device=dev)
        for _, p in self.named:
            self.offsets.append(off)
            init[off:off + p.numel()] = p.detach().reshape(-1)
            off += p.numel()
        # world > 1: the bf16 engine copy is cast from the gathered fp32 master on every rank
        # (_gather_full), so ShardedAdamW keeps no bf16 shard of its own to all-gather
        self.opt = ShardedAdamW(self.reducer, init, config, shadow_bf16=True, gather_bf16=not self.collective)
        del init
        self._weights_ready = None
        if not self.collective:
            self.full = self.opt.param
        else:
            self.full = torch.zeros(lay.padded, dtype=torch.float32, device=dev)
            self._gather_full(sync=True)
        self._bucket_count = [0] * len(lay.buckets)  # parameters overlapping each bucket
        self._param_buckets: List[Tuple[int, int]] = []  # first / last bucket of each parameter
        for (_, p), o in zip(self.named, self.offsets):
            p.data = self.full[o:o + p.numel()].view_as(p)
            p.grad = self.reducer.grad[o:o + p.numel()].view_as(p)
            b0, b1 = self._bucket_at(o), self._bucket_at(o + p.numel() - 1)
            self._param_buckets.append((b0, b1))
            for b in range(b0, b1 + 1):
                self._bucket_count[b] += 1
        self._index = {id(p): i for i, (_, p) in enumerate(self.named)}
        self._touched = [False] * len(self.named)  # parameters a backward reached since the last step
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for _, p in self.named]
        # every piece of this rank's shard that belongs to a parameter: the per-parameter update
        # (skip untouched parameters, per-parameter step counts) runs on this map on the device
        pieces = []
        for i, ((_, p), o) in enumerate(zip(self.named, self.offsets)):
            b0, b1 = self._param_buckets[i]
            for b in range(b0, b1 + 1):
                ps, pe = lay.piece(b, self.rank) if self.collective else lay.buckets[b]
                lo, hi = max(o, ps), min(o + p.numel(), pe)
                if hi > lo:
                    pieces.append(((lay.piece_off[b] + lo - ps) if self.collective else lo, hi - lo, i))
        self.segments = ParamSegments(pieces, len(self.named), lay.shard_numel, dev)
        # the module's next forward reads the re-assembled master: it waits for the in-flight gather
        # (callers that read the weights without calling the module -- the trainer's base_model /
        # lm_head passes -- call wait_weights() themselves; base_model gets the same hook)
        self._fwd_hooks = [module.register_forward_pre_hook(lambda m, a: self.wait_weights())]
        base = getattr(module, "base_model", None)
        if isinstance(base, torch.nn.Module) and base is not module:
            self._fwd_hooks.append(base.register_forward_pre_hook(lambda m, a: self.wait_weights()))
        self._armed = False
        self.launched_during_backward = 0

    def _bucket_at(self, x: int) -> int:
        for b, (s, e) in enumerate(self.reducer.layout.buckets):
            if s <= x < e:
                return b
        raise IndexError(x)

    # ---------------------------------------------------------------- gradient exchange
    def arm(self) -> None:
        """Call before the backward of the mini-batch's last micro-batch."""
        if not self.collective:
            return
        self._armed = True
        self._pending = list(self._bucket_count)
        self._fired = [False] * len(self.named)
        self._ready = [n == 0 for n in self._pending]
        self._next = 0
        self.launched_during_backward = 0
        self._launch_ready()

    def _launch_ready(self) -> None:
        while self._next < len(self._ready) and self._ready[self._next]:
            self.reducer.launch([self._next])
            self._next += 1
            self.launched_during_backward += 1

    def _on_grad(self, p) -> None:
        i = self._index[id(p)]
        self._touched[i] = True
        if not self._armed:
            return
        if self._fired[i]:
            return
        self._fired[i] = True
        b0, b1 = self._param_buckets[i]
        for b in range(b0, b1 + 1):
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._ready[b] = True
        self._launch_ready()

    def _finish_exchange(self) -> None:
        if not self.collective or not self._armed:
            return
        while self._next < len(self._ready):  # buckets whose parameters got no gradient
            self.reducer.launch([self._next])
            self._next += 1
        self._armed = False

    # ---------------------------------------------------------------- step
    def step(self, n_micro: int = 1, lr: Optional[float] = None) -> torch.Tensor:
        """optim_step: grads * 1/n_micro (and 1/world), clip, AdamW, zero grads; then (world > 1)
        the updated master is re-assembled on every rank by one fp32 all-gather per bucket and the
        engine's bf16 copy is cast from it on the same comm stream (each rank casts locally: no
        second, bf16 all-gather over xGMI). Both are left in flight: the module's next forward
        (a forward pre-hook), :meth:`named_bf16` and :meth:`wait_weights` make the current stream
        wait for them, so the exchange overlaps whatever the host issues next (the engine's
        rollout in the fully-async loop, fully_async_trainer.py:415-419). Returns the pre-clip grad
        norm (device scalar)."""
        self._finish_exchange()
        self._check_grad_views()  # the .grad views must still be the buckets' storage
        # which parameters some rank's backward reached: this rank's flags staged from pinned host
        # memory and MAX-reduced on the device (no host read). torch.optim.AdamW skips a parameter
        # whose .grad is None and keeps a step count per parameter: the update pass does the same
        # per shard segment (master, moments and bf16 copy of a skipped parameter untouched)
        self.segments.upload(self._touched, group=self.reducer.group, collective=self.collective)
        gn = self.opt.step(n_micro=n_micro, lr=lr, zero_grad=True, seg=self.segments)
        self._touched = [False] * len(self.named)
        if self.collective:
            self._gather_full(sync=False)
        return gn

    def wait_weights(self) -> None:
        """Make the current stream wait for the last step's all-gather + bf16 cast (no host sync)."""
        ev = self._weights_ready
        if ev is not None:
            torch.cuda.current_stream(self.full.device).wait_event(ev)
            self._weights_ready = None

    def _check_grad_views(self) -> None:
        base = self.reducer.grad.data_ptr()
        for (n, p), o in zip(self.named, self.offsets):
            if p.grad is None or p.grad.data_ptr() != base + 4 * o:
                raise RuntimeError(f"{n}.grad is no longer a view of the flat gradient buffer "
                                   "(set_to_none / reassigned); the exchange would miss it")

    def _gather_full(self, sync: bool) -> None:
        """fp32 all-gather of the updated shards into the full master (one per bucket, comm stream),
        then the bf16 engine copy cast from it on that stream; records ``_weights_ready``."""
        from . import _ffi
        from .ops import _ptr

        r = self.reducer
        lay = r.layout
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.full.device))
        r.stream.wait_event(ready)
        with torch.cuda.stream(r.stream):
            for b, (s, e) in enumerate(lay.buckets):
                po = lay.piece_off[b]
                nb = (e - s) // r.world
                dist.all_gather_into_tensor(self.full[s:e], self.opt.param[po:po + nb], group=r.group)
            w = self.opt.weights_bf16
            _ffi.call("skyrl_cast_bf16", _ptr(self.full), _ptr(w), w.numel(), ctypes.c_void_p(r.stream.cuda_stream))
            self._weights_ready = torch.cuda.Event()
            self._weights_ready.record(r.stream)
        if sync:
            self.wait_weights()

    # ---------------------------------------------------------------- weight sync
    def named_bf16(self) -> List[Tuple[str, torch.Tensor]]:
        """(HF name, bf16 view) of every parameter in the engine copy: the weight update request
        of broadcast_to_inference_engines without a per-parameter cast."""
        self.wait_weights()
        w = self.opt.weights_bf16
        return [(n, w[o:o + p.numel()].view(p.shape)) for (n, p), o in zip(reversed(self.named),
                                                                          reversed(self.offsets))]


def allreduce_grads(params: Iterable[torch.Tensor], group=None, bucket_bytes: int = 64 << 20) -> int:
    """Mean of `.grad` over the DP group for parameters that are not views of a flat buffer
    (a HF module under the GRPOTrainer): grads are packed into ~bucket_bytes fp32 buckets, one
    SUM all-reduce per bucket, scaled by 1/world and copied back (FSDP's mean reduce,
    fsdp_strategy.py:216-226). Returns the number of collectives issued."""
    world, _ = _world(group)
    grads = [p.grad for p in params if p.grad is not None]
    if not _collective(world) or not grads:
        return 0
    n = 0
    bucket: List[torch.Tensor] = []
    size = 0

    def flush():
        nonlocal n
        flat = torch.cat([g.reshape(-1).to(torch.float32) for g in bucket])
        dist.all_reduce(flat, group=group)
        flat.mul_(1.0 / world)
        off = 0
        for g in bucket:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()
        n += 1

    for g in grads:
        bucket.append(g)
        size += g.numel() * 4
        if size >= bucket_bytes:
            flush()
            bucket, size = [], 0
    if bucket:
        flush()
    return n
