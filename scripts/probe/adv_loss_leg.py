"""Times bench.advantage_loss_leg alone (the graph-replayed GRPO + loss + backward leg) at the
batch size and 16x, for A/B runs of the loss kernels without the whole bench."""
import json
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda:0")
out = {"batch": bench.advantage_loss_leg(dev, 512, 1024, variants=True),
       "batch_x16": bench.advantage_loss_leg(dev, 16 * 512, 1024, reps=5)}
from skyrl_amd import _ffi  # noqa: E402

for nb in (8, 32, 64, 256, 1024):  # backward node grid cap (unit gradient: every block exits at once)
    _ffi.call("skyrl_tune", b"loss_bwd_blocks", nb)
    out[f"bwd_blocks{nb}"] = {k: v for k, v in bench.advantage_loss_leg(dev, 512, 1024).items()
                              if k in ("loss_bwd_us", "total_us")}
_ffi.call("skyrl_tune", b"loss_bwd_blocks", 256)
print(json.dumps(out))
