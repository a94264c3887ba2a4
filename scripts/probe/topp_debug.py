"""Debug: the V=4097 min_p=0.01 case of test_topp_fast_small_and_ragged_vocab, mismatching rows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import ops  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_gpu_sampler_topp_fast import _run  # noqa: E402

dev = torch.device("cuda:0")
for V in (4097, 1000, 517):
    g = torch.Generator().manual_seed(V)
    n = 40
    width = (V + 7) // 8 * 8 + 8
    base = (torch.randn(n, width, generator=g) * 2).to(torch.bfloat16)
    x = base.to(dev)[:, :V]
    ids = torch.arange(n, dtype=torch.int64)
    for p, mp in ((0.9, 0.0), (1.0, 0.05), (0.7, 0.01), (1.0, 0.01)):
        kw = dict(temperature=1.0, top_p=p, min_p=mp, seed=9, seq_ids=ids.to(dev), step=2)
        for chunked, helpers in ((False, 256), (True, 256), (True, 0)):
            tf, lf, ff = _run(x, True, chunked, helpers, **kw)
            ts, ls, fs = _run(x, False, **kw)
            bad = torch.nonzero(tf != ts).reshape(-1).tolist()
            print(V, p, mp, chunked, helpers, "mismatch rows", bad[:5], flush=True)
            for r in bad[:2]:
                xr = base[r, :V].float()
                print("   row", r, "fast", int(tf[r]), float(xr[tf[r]]), "slow", int(ts[r]), float(xr[ts[r]]), "max",
                      float(xr.max()), "ff", ff[r].tolist(), "fs", fs[r].tolist(), flush=True)
