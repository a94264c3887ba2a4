"""a11: TensorBatch / TrainingInputBatch — a dict of equal-length tensors plus metadata.

Mirror of skyrl-train/skyrl_train/training_batch.py:14-383 (same method names, argument
meaning and error messages): select / slice / chunk / cat / repeat / repeat_interleave /
to / contiguous, int and slice indexing, batch-size and device consistency checks.

Wire format (reference :136-199 pickles raw numpy bytes + shape + dtype, bf16 via torch.save):
here every tensor, bf16 included, travels as raw little-endian bytes with a JSON header
(``to_bytes`` / ``from_bytes``), so loading never executes anything from the payload.
Pickle support (``__getstate__``/``__setstate__``) uses the same raw-bytes records.
Host -> device moves go through pinned staging buffers when ``non_blocking`` is set, so the
copy overlaps the caller's work instead of blocking on pageable memory.
"""

from __future__ import annotations

import json
import struct
from typing import Any, Dict, Generic, List, Optional, TypeVar

import numpy as np
import torch

DictType = TypeVar("DictType")

_MAGIC = b"SKTB1\0"
_DT = {
    torch.float32: "float32", torch.float64: "float64", torch.float16: "float16", torch.bfloat16: "bfloat16",
    torch.int64: "int64", torch.int32: "int32", torch.int16: "int16", torch.int8: "int8", torch.uint8: "uint8",
    torch.bool: "bool",
}
_DT_INV = {v: k for k, v in _DT.items()}


def _tensor_record(t: torch.Tensor) -> Dict[str, Any]:
    t = t.detach().contiguous().cpu()
    raw = t.view(torch.int16) if t.dtype == torch.bfloat16 else t
    return {"dtype": _DT[t.dtype], "shape": list(t.shape), "data": raw.numpy().tobytes()}


def _tensor_from_record(rec: Dict[str, Any]) -> torch.Tensor:
    dt = _DT_INV[rec["dtype"]]
    np_dt = np.int16 if dt == torch.bfloat16 else torch.empty((), dtype=dt).numpy().dtype
    arr = np.frombuffer(rec["data"], dtype=np_dt).reshape(rec["shape"]).copy()
    t = torch.from_numpy(arr)
    return t.view(torch.bfloat16) if dt == torch.bfloat16 else t


class TensorBatch(dict, Generic[DictType]):
    """Dictionary of equal-length tensors (first dimension = batch) plus ``metadata``."""

    metadata: Optional[Dict[str, Any]] = None

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._batch_size = None
        self._device = None
        self._check_consistency()

    def select(self, keys: List[str], metadata_keys: Optional[List[str]] = None) -> "TensorBatch[DictType]":
        new = self.__class__({k: self[k] for k in keys})
        new.metadata = self.metadata if metadata_keys is None else {k: self.metadata[k] for k in metadata_keys}
        return new

    def _check_consistency(self):
        keys = list(self.keys())
        if not keys:
            return
        self._batch_size = len(dict.__getitem__(self, keys[0]))
        for key in keys:
            value = dict.__getitem__(self, key)
            if value is None:
                continue
            if not isinstance(value, torch.Tensor):
                raise ValueError(f"Field {key} must be a tensor, got {type(value)}")
            self._device = value.device if self._device is None else self._device
            if len(value) != self._batch_size:
                raise ValueError(f"Batch size mismatch in {key}")
            if value.device != self._device:
                raise ValueError(f"Device mismatch in {key}. Expected {self._device}, got {value.device}")

    def __getitem__(self, index):
        if isinstance(index, slice):
            return self.slice(index.start, index.stop, index.step)
        if isinstance(index, int):
            return self.slice(index, index + 1)
        return super().__getitem__(index)

    def __setitem__(self, key: str, value: Optional[torch.Tensor]) -> None:
        if value is None:
            super().__setitem__(key, value)
            return
        if not isinstance(value, torch.Tensor):
            raise ValueError(f"Field {key} must be a tensor, got {type(value)}")
        if getattr(self, "_batch_size", None) is not None and len(value) != self._batch_size:
            raise ValueError(
                f"Batch size mismatch in {key}. Expected tensor to be of size {self._batch_size}, got {len(value)}.")
        super().__setitem__(key, value)
        if getattr(self, "_batch_size", None) is None:
            self._batch_size = len(value)

    def to(self, device: torch.device = None, dtype: torch.dtype = None, *, non_blocking: bool = False) -> "TensorBatch":
        dev = torch.device(device) if device is not None else None
        for key, value in list(self.items()):
            if value is None:
                continue
            if non_blocking and dev is not None and dev.type == "cuda" and value.device.type == "cpu":
                value = value.pin_memory()
            self[key] = value.to(dev, dtype, non_blocking=non_blocking)
        if dev is not None:
            self._device = dev if dev.index is not None or dev.type == "cpu" else self._device
            firsts = [v for v in self.values() if v is not None]
            if firsts:
                self._device = firsts[0].device
        return self

    def contiguous(self) -> "TensorBatch":
        for key, value in list(self.items()):
            if value is not None:
                self[key] = value.contiguous()
        return self

    @property
    def batch_size(self) -> int:
        return self._batch_size

    @property
    def device(self) -> torch.device:
        return self._device

    # ---- wire format ----------------------------------------------------------------
    def __getstate__(self):
        self.contiguous()
        if self._device is not None:
            assert self._device == torch.device("cpu"), "Tensors must be on CPU before serialization"
        return {
            "batch_dict": {k: (None if v is None else _tensor_record(v)) for k, v in self.items()},
            "batch_size": self._batch_size,
            "device": None if self._device is None else str(self._device),
            "metadata": self.metadata,
        }

    def __setstate__(self, state):
        for key, rec in state["batch_dict"].items():
            self[key] = None if rec is None else _tensor_from_record(rec)
        self._batch_size = state["batch_size"]
        self._device = None if state["device"] is None else torch.device(state["device"])
        self.metadata = state["metadata"]
        self._check_consistency()
        return self

    def to_bytes(self) -> bytes:
        """Header (JSON: keys, dtypes, shapes, byte lengths, JSON-able metadata) + raw tensor bytes."""
        recs, blobs = [], []
        for k, v in self.items():
            if v is None:
                recs.append({"key": k, "none": True})
                continue
            r = _tensor_record(v)
            blobs.append(r.pop("data"))
            r.update(key=k, nbytes=len(blobs[-1]))
            recs.append(r)
        header = json.dumps({"fields": recs, "batch_size": self._batch_size, "metadata": self.metadata}).encode()
        return _MAGIC + struct.pack("<Q", len(header)) + header + b"".join(blobs)

    @classmethod
    def from_bytes(cls, buf: bytes) -> "TensorBatch":
        if buf[: len(_MAGIC)] != _MAGIC:
            raise ValueError("not a TensorBatch byte stream")
        off = len(_MAGIC)
        (hlen,) = struct.unpack_from("<Q", buf, off)
        off += 8
        header = json.loads(buf[off:off + hlen].decode())
        off += hlen
        out = cls()
        for r in header["fields"]:
            if r.get("none"):
                out[r["key"]] = None
                continue
            n = r["nbytes"]
            out[r["key"]] = _tensor_from_record({"dtype": r["dtype"], "shape": r["shape"], "data": buf[off:off + n]})
            off += n
        out.metadata = header["metadata"]
        out._batch_size = header["batch_size"]
        return out

    # ---- reshaping ------------------------------------------------------------------
    def repeat(self, repeats: int):
        new = self.__class__({k: (None if v is None else v.repeat(repeats, *([1] * (v.dim() - 1))))
                              for k, v in self.items()})
        new.metadata = self.metadata
        return new

    def repeat_interleave(self, repeats: int):
        new = self.__class__({k: (None if v is None else v.repeat_interleave(repeats, dim=0)) for k, v in self.items()})
        new.metadata = self.metadata
        return new

    def chunk(self, chunk_size: int) -> List["TensorBatch[DictType]"]:
        return [self.slice(i, i + chunk_size) for i in range(0, self.batch_size, chunk_size)]

    def slice(self, start: int, end: int, step: int = 1) -> "TensorBatch[DictType]":
        sl = slice(start, end, step)
        new = self.__class__({k: (None if v is None else v[sl]) for k, v in self.items()})
        new.metadata = self.metadata
        return new

    def save(self, path: str):
        with open(path, "wb") as f:
            f.write(self.to_bytes())

    def load(self, path: str):
        with open(path, "rb") as f:
            return self.__class__.from_bytes(f.read())

    @classmethod
    def cat(cls, shards: List["TensorBatch[DictType]"]) -> "TensorBatch[DictType]":
        assert len(shards) > 0, "Cannot cat an empty list of shards"
        data = {k: (None if v is None else torch.cat([s[k] for s in shards])) for k, v in shards[0].items()}
        out = cls(data)
        out.metadata = shards[0].metadata
        return out

    def __len__(self) -> int:
        return self._batch_size

    def __eq__(self, other: Any) -> bool:
        if not isinstance(other, TensorBatch):
            return False
        if self.metadata != other.metadata or len(self) != len(other) or len(self.items()) != len(other.items()):
            return False
        for k, v in self.items():
            if k not in other:
                return False
            o = dict.__getitem__(other, k)
            if (v is None) != (o is None) or (v is not None and not torch.equal(v, o)):
                return False
        return True

    __hash__ = None

    def __str__(self) -> str:
        return (f"TensorBatch(batch_size={self.batch_size}, device={self.device}, metadata={self.metadata}), "
                f"items={self.items()}")

    __repr__ = __str__


class TrainingInputBatch(TensorBatch[Dict[str, torch.Tensor]]):
    """Training input data (keys of reference TrainingInput, training_batch.py:365-378)."""


class TrainingOutputBatch(TensorBatch[Dict[str, torch.Tensor]]):
    """Training output data."""
