"""Run bench.py's graph-replayed advantage+loss leg alone (batch and 16x batch)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
print(json.dumps({"batch": bench.advantage_loss_leg(dev, 512, 1024),
                  "batch_x16": bench.advantage_loss_leg(dev, 8192, 1024, reps=5)}))
