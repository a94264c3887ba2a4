"""The forward-only lm_head logprob pass (old / ref log-probs: lmhead.lmhead_logprobs_and_entropy
under no_grad) at T = 8192 tokens, H = 1536, V = 151,936, with a given V-chunk width, run
`--iters` times after one warm-up: profile it with rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE to see
whether the bf16 [T, chunk] logits chunks round-trip through HBM or stay in the caches (the
algorithmic bytes of the pass are W + H = 492 MB; logits through HBM would add 2 x 2.49 GB).
Prints one JSON line with the event-timed ms per pass."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from skyrl_amd import lmhead  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--H", type=int, default=1536)
    ap.add_argument("--V", type=int, default=151936)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    W = (torch.randn(a.V, a.H, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    h = torch.randn(a.T, a.H, device=dev, generator=g).to(torch.bfloat16)
    lab = torch.randint(0, a.V, (a.T,), device=dev, generator=g)

    def run():
        with torch.no_grad():
            return lmhead.lmhead_logprobs_and_entropy(h, W, lab, 1.0, True, a.chunk or None)

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    e1.synchronize()
    print(json.dumps({"T": a.T, "H": a.H, "V": a.V, "chunk": a.chunk or lmhead.default_chunk(a.T, a.V),
                      "ms_per_pass": round(e0.elapsed_time(e1) / a.iters, 4),
                      "algorithmic_bytes": a.V * a.H * 2 + a.T * a.H * 2 + a.T * 8,
                      "logits_bytes": a.T * a.V * 2}), flush=True)


if __name__ == "__main__":
    main()
