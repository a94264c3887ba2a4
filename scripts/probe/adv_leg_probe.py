"""A/B of the advantage+loss leg's finish launch (skyrl_variant "finish_mode", "loss_bwd_blocks"):
replays bench.advantage_loss_leg at the metric's batch for each setting, twice interleaved."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from skyrl_amd import _ffi  # noqa: E402

dev = torch.device("cuda", 0)
keys = ("loss_bwd_us", "grpo_loss_deferred_us", "finish_us", "total_us", "in_launch_fold_total_us")
out = {}
for rep in range(2):
    for mode in (0, 2, 3, 4):
        for blocks in (256,):
            _ffi.set_default_variant(finish_mode=mode)
            _ffi.set_default_variant(loss_bwd_blocks=blocks)
            r = bench.advantage_loss_leg(dev, 512, 1024)
            out.setdefault(f"mode{mode}_blocks{blocks}", []).append({k: r[k] for k in keys})
            print(f"mode {mode} blocks {blocks}:", {k: r[k] for k in keys}, flush=True)
_ffi.set_default_variant(finish_mode=0)
_ffi.set_default_variant(loss_bwd_blocks=256)
print(json.dumps(out))
