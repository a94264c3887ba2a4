import json, torch, sys
sys.path.insert(0, '.')
import bench
print(json.dumps(bench.learner_lmhead_fwd_leg(torch.device('cuda'))))
