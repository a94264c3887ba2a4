"""Ray-free mesh dispatch (skyrl_amd/dispatch.py) on a real 8-rank gloo group, mirroring the
reference's tests/cpu/distributed/test_dispatch.py: mesh dispatch + collect, dispatch from a
staged batch, pass-through, a None/non-None mix, and the registry.

Layout: dp=4 x sp=2 with tp fastest, then sp (mesh_rank), so the collection ranks (sp=0)
are the even global ranks 0, 2, 4, 6 for dp 0..3. The worker adds its global rank, as the
reference's RayActor.do_work does, so the expected vectors differ from the reference's only
through that layout."""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from skyrl_amd.dispatch import (ActorInfo, Dispatch, DispatchRegistry, MeshDispatch, PassThroughDispatch, collect,
                                mesh_rank, stage)
from skyrl_amd.training_batch import TrainingInputBatch

WORLD, DP, SP = 8, 4, 2


class Worker:
    def __init__(self, rank):
        self.rank = rank

    def do_work(self, data):
        data["a"] = data["a"] + self.rank
        return data

    def do_work_from_staged(self, data, start_idx, end_idx):
        data = data.slice(start_idx, end_idx)
        data["a"] = data["a"] + self.rank
        return data

    def dummy(self, a, b):
        return None


def _rank(rank, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    me = mesh_rank(rank, WORLD, DP, sp_size=SP)
    info = ActorInfo(Worker(rank), me)
    res = {}
    data = TrainingInputBatch({"a": torch.tensor([1, 2, 3, 4]), "m": torch.ones(4, 3, dtype=torch.bfloat16)})
    data.metadata = {"response_length": 3}
    out = MeshDispatch.dispatch(info, "do_work", data if rank == 0 else None)
    res["mesh"] = MeshDispatch.sync_collect(info, out)
    staged = stage(TrainingInputBatch({"a": torch.arange(16)}) if rank == 0 else None)
    out = MeshDispatch.dispatch_from_staged(info, "do_work_from_staged", staged, start_idx=4, end_idx=12)
    res["from_staged"] = MeshDispatch.sync_collect(info, out)
    res["pass"] = PassThroughDispatch.sync_collect(info, PassThroughDispatch.dispatch(info, "dummy", 1, 2))
    mixed = None if rank == 0 else info.handle.do_work(data)
    try:
        collect(me, mixed)
        res["mixed"] = "no error"
    except AssertionError:
        res["mixed"] = "assert"
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    out = tmp_path_factory.mktemp("dispatch")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(port, str(out)), nprocs=WORLD, join=True)
    return [torch.load(out / f"r{r}.pt", weights_only=False) for r in range(WORLD)]


def test_mesh_dispatch(results):
    got = results[0]["mesh"]
    assert torch.equal(got["a"], torch.tensor([1, 4, 7, 10]))  # + ranks 0, 2, 4, 6
    assert got["m"].dtype == torch.bfloat16 and got["m"].shape == (4, 3)
    assert all(r["mesh"] is None for r in results[1:])  # only dst holds the result


def test_dispatch_from_staged(results):
    # dp d gets [4 + 2d, 6 + 2d) and adds its collection rank 2d
    assert torch.equal(results[0]["from_staged"]["a"], torch.tensor([4, 5, 8, 9, 12, 13, 16, 17]))


def test_pass_through_dispatch(results):
    assert all(r["pass"] is None for r in results)


def test_mesh_dispatch_with_mixed(results):
    assert results[0]["mixed"] == "assert"


def test_mesh_rank_layout():
    ranks = [mesh_rank(r, 8, 2, sp_size=1, tp_size=2, pp_size=2) for r in range(8)]
    assert [(m.dp, m.pp, m.tp) for m in ranks[:4]] == [(0, 0, 0), (0, 0, 1), (0, 1, 0), (0, 1, 1)]
    assert [m.is_collection_dp_rank() for m in ranks] == [False, False, True, False] * 2
    with pytest.raises(ValueError):
        mesh_rank(0, 8, 3)


def test_single_process_dispatch_and_validation():
    me = mesh_rank(0, 1, 1)
    info = ActorInfo(Worker(5), me)
    out = MeshDispatch.dispatch(info, "do_work", TrainingInputBatch({"a": torch.tensor([1, 2])}))
    assert torch.equal(MeshDispatch.sync_collect(info, out)["a"], torch.tensor([6, 7]))
    with pytest.raises(ValueError):
        MeshDispatch.validate_dispatch_args({"a": 1})
    with pytest.raises(ValueError):
        MeshDispatch.validate_dispatch_args()
    assert MeshDispatch.validate_dispatch_args(data=TrainingInputBatch({"a": torch.zeros(2)}), x=1)[1] == {"x": 1}


def test_dispatch_registry():
    class CustomDispatch(Dispatch):
        @classmethod
        def dispatch(cls, actor_info, method, *args, **kwargs):
            return None

    try:
        DispatchRegistry.register("custom", CustomDispatch)
        assert DispatchRegistry.get("custom") is CustomDispatch
        assert DispatchRegistry.list_registered() == {"mesh": MeshDispatch, "pass_through": PassThroughDispatch,
                                                      "custom": CustomDispatch}
        with pytest.raises(KeyError):
            DispatchRegistry.get("nope")
    finally:
        DispatchRegistry._registry.pop("custom")
