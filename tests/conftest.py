import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (runs the HIP kernels)")


def load_golden(name: str) -> dict:
    """Golden vectors written by tools/gen_golden.py from the real reference (arrays only)."""
    out = {}
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        for k in z.files:
            v = z[k]
            if k.endswith("__bf16"):
                out[k[: -len("__bf16")]] = torch.from_numpy(v.astype(np.uint16).view(np.int16).copy()).view(torch.bfloat16)
            elif v.dtype.kind in "fiub":
                out[k] = torch.from_numpy(np.array(v))
            else:
                out[k] = v
    return out


@pytest.fixture
def golden():
    return load_golden


@pytest.fixture
def dev():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda:0")
