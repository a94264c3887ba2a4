"""Times bench.sampler_filtered_leg alone (the §8(d) top_k = 50 / top_p = 0.9 sampler variant,
one-pass kernel vs the two-kernel path) and prints its JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.sampler_filtered_leg(torch.device("cuda:0"), 512, 151936)))
