"""Host side of the vocab-parallel lm_head logprob (skyrl_amd/lmhead.py): the per-token state
all-gather over a real 2-rank gloo group returns the ranks' states in rank order (the merge
kernel's contract), and a single process without a group is world 1."""

import os
import socket

import torch
import torch.multiprocessing as mp

from skyrl_amd.lmhead import _gather_states, _tp_world


def _rank(rank, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    T = 5
    state = torch.full((T * 16,), rank + 1, dtype=torch.uint8)  # raw bytes, as the device buffer
    states, n = _gather_states(state, T, dist.group.WORLD)
    torch.save({"n": n, "states": states}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_gather_states_rank_order(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(port, str(tmp_path)), nprocs=2, join=True)
    for r in (0, 1):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert got["n"] == 2 and got["states"].shape == (10, 4)
        raw = got["states"].contiguous().view(torch.uint8).view(2, 5 * 16)
        assert bool((raw[0] == 1).all()) and bool((raw[1] == 2).all())


def test_single_process_is_world_one():
    assert _tp_world(None) == 1
    st, n = _gather_states(torch.zeros(3 * 16, dtype=torch.uint8), 3, None)
    assert n == 1 and st.shape == (3, 4)
