"""Where does a forced split cost time? Uniform 512 x 1280 contexts, nparts 1 vs 2 (and the ragged
512 x U[17,1536] mix at nparts 1 / 3 with a 512-token chunk), each config run 50 times so
rocprofv3 --kernel-trace --stats separates paged_decode_kernel from paged_decode_reduce_kernel.
Probe only."""
import json
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts/probe")
from attn_chunk_sweep import setup, time_it  # noqa: E402

from skyrl_amd.inference_engines import kernels  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    mode = sys.argv[1] if len(sys.argv) > 1 else "all"
    cfgs = {"u1": ((512, 1280, 1280), 1, kernels.MIN_PARTITION), "u2": ((512, 1280, 1280), 2, kernels.MIN_PARTITION),
            "r1": ((512, 17, 1536), 1, kernels.MIN_PARTITION), "r3": ((512, 17, 1536), 3, 512)}
    for name, (shape, np_, pm) in cfgs.items():
        if mode != "all" and name != mode:
            continue
        us, gbs, _ = time_it(dev, setup(dev, *shape), np_, pm, reps=50)
        print(json.dumps({"cfg": name, "nparts": np_, "part_min": pm, "us": round(us, 2), "GBps": round(gbs, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
