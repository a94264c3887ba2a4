"""Separated placement on the GPU: the learner rank's GRPOTrainer feeds a rollout engine hosted
by another rank (scripts/rehearse_separated.py, 2 ranks on one GPU over gloo). The protocol
itself is covered on CPU by tests/test_remote_engine.py."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_separated_trainer_feeds_remote_engine():
    """After every synchronous step and after three FullyAsync steps (pause -> update ->
    resume with generation in flight) the remote engine's weights equal the learner's bf16
    weights bit for bit and its greedy tokens equal a colocated engine's
    (broadcast_strategy.py:98-191, vllm_worker.py:43-96, fully_async_trainer.py:415-419)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "scripts", "rehearse_separated.py")]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stderr[-3000:]
    res = json.loads(lines[-1])
    assert p.returncode == 0 and res["ok"], json.dumps(res)[:3000] + p.stderr[-2000:]
    assert len(res["sync"]) == 2 and res["fully_async"]["steps"] == 3
    print(json.dumps(res))
