"""The bench's two lm_head legs alone (decode-side fused sampler at 512 rows, learner forward at
T = 8192): one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

dev = torch.device("cuda")
print(json.dumps({"rollout_lmhead_sample": bench.lmhead_sample_leg(dev, 512),
                  "learner_lmhead_fwd": bench.learner_lmhead_fwd_leg(dev)}))
