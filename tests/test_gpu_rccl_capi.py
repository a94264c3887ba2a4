"""The C-ABI RCCL collectives (skyrl_comm_*, skyrl_amd/rccl.py) on the GPU: a one-rank
communicator (RCCL refuses two ranks on one device), so every collective's result is its input
-- the checks are that the calls run on the given stream, move the right byte counts for every
dtype and op, and validate their arguments; the 8-GPU run is the driver's."""

import pytest
import torch

from skyrl_amd import _ffi
from skyrl_amd.rccl import RcclComm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    torch.cuda.set_device(0)
    c = RcclComm(1, 0, RcclComm.unique_id())
    yield c
    c.close()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64, torch.int32, torch.uint8])
@pytest.mark.parametrize("op", ["sum", "max", "min", "avg"])
def test_allreduce_one_rank(comm, dev, dtype, op):
    if op == "avg" and dtype in (torch.int64, torch.int32, torch.uint8):
        pytest.skip("avg on integers")
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.rand(4099, device=dev, generator=g) * 100).to(dtype)
    out = torch.empty_like(x)
    comm.all_reduce(x, op, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, x)
    y = x.clone()
    comm.all_reduce(y, op)  # in place
    torch.cuda.synchronize()
    assert torch.equal(y, x)


def test_reduce_scatter_allgather_broadcast_one_rank(comm, dev):
    assert comm.size() == (1, 0)
    x = torch.randn(1 << 20, device=dev)
    rs = torch.empty_like(x)
    comm.reduce_scatter(rs, x)
    ag = torch.empty(x.numel(), dtype=torch.bfloat16, device=dev)
    xb = x.to(torch.bfloat16)
    comm.all_gather(ag, xb)
    bc = x.clone()
    comm.broadcast(bc, root=0)
    torch.cuda.synchronize()
    assert torch.equal(rs, x) and torch.equal(ag, xb) and torch.equal(bc, x)


def test_collective_on_a_side_stream(comm, dev):
    """Stream-ordered: the all-reduce runs on the stream it is given, after the work queued there."""
    s = torch.cuda.Stream(dev)
    x = torch.zeros(1 << 22, device=dev)
    with torch.cuda.stream(s):
        x.fill_(3.0)
        comm.all_reduce(x, "sum")
        x.mul_(2.0)
    s.synchronize()
    assert float(x.min()) == 6.0 and float(x.max()) == 6.0


def test_argument_errors(comm, dev):
    x = torch.zeros(8, device=dev)
    with pytest.raises(ValueError):
        comm.reduce_scatter(torch.zeros(3, device=dev), x)
    with pytest.raises(TypeError):
        comm.all_reduce(torch.zeros(8, dtype=torch.float16, device=dev))
    with pytest.raises(_ffi.SkyrlHipError, match="op must be"):
        comm.all_reduce(x, 7)


def test_from_group_under_torchrun(tmp_path):
    """RcclComm.from_group: rank 0's id travels over a torch (gloo) process group."""
    import os
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    code = ("import torch, torch.distributed as dist\n"
            "from skyrl_amd.rccl import RcclComm\n"
            "dist.init_process_group('gloo')\n"
            "torch.cuda.set_device(0)\n"
            "c = RcclComm.from_group()\n"
            "x = torch.arange(1000, dtype=torch.float32, device='cuda')\n"
            "y = c.all_reduce(x.clone(), 'max')\n"
            "torch.cuda.synchronize()\n"
            "assert torch.equal(x, y) and c.size() == (1, 0)\n"
            "c.close()\n"
            "dist.destroy_process_group()\n"
            "print('RCCL_FROM_GROUP_OK')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    script = tmp_path / "rccl_from_group.py"
    script.write_text(code)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(script)]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=180, env=env)
    assert p.returncode == 0 and "RCCL_FROM_GROUP_OK" in p.stdout, p.stderr[-3000:]
