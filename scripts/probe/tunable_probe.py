"""Does PyTorch TunableOp (runtime GEMM solution search over hipBLASLt/rocBLAS) speed up the
decode step's skinny GEMMs? Decode forward of the random Qwen2.5-1.5B-shaped decoder at
512 / 64 / 8 rows, eager and graph-replayed, with and without TunableOp."""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from engine_bench import decode_step_bench  # noqa: E402

if __name__ == "__main__":
    res = {"baseline": [decode_step_bench(n, c, 28) for n, c in ((512, 400), (64, 1024), (8, 512))]}
    print(json.dumps(res), file=sys.stderr, flush=True)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), "tunableop_results.csv"))
    res["tunable"] = [decode_step_bench(n, c, 28) for n, c in ((512, 400), (64, 1024), (8, 512))]
    print(json.dumps(res), flush=True)
