"""Decode-step kernel profile target: eager decode forwards of a random Qwen2.5-1.5B-shaped
decoder at (nseq, ctx) for rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from engine_bench import decode_step_bench  # noqa: E402

if __name__ == "__main__":
    nseq, ctx = (int(x) for x in (sys.argv[1:3] if len(sys.argv) > 2 else (512, 400)))
    print(decode_step_bench(nseq, ctx, 28, reps=20), flush=True)
