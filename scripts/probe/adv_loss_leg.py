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

for rpb in (1, 2):  # row chunks per fused GRPO+loss block
    _ffi.set_default_variant(grpo_loss_rpb=rpb)
    out[f"rpb{rpb}"] = {k: v for k, v in bench.advantage_loss_leg(dev, 512, 1024).items()
                        if k in ("grpo_loss_fused_us", "total_us")}
_ffi.set_default_variant(grpo_loss_rpb=1)
print(json.dumps(out))
