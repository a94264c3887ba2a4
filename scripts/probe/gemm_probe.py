"""hipBLASLt throughput on the lm_head shapes (logits = h @ W^T, W [V,H] bf16), whole-vocab and
V-chunked into one reused buffer, to size the fused lm_head logprob path. Prints one JSON line per case."""

import json
import sys

import torch


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda")
    H, V = 1536, 151936
    W = (torch.randn(V, H, device=dev) * 0.02).to(torch.bfloat16)
    for T in (4096, 8192, 16384):
        h = torch.randn(T, H, device=dev).to(torch.bfloat16)
        full = torch.empty(T, V, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: torch.mm(h, W.t(), out=full))
        fl = 2.0 * T * H * V
        print(json.dumps({"case": "full", "T": T, "ms": ms, "TFLOPs": fl / ms / 1e9}), flush=True)
        for vc in (4096, 8192, 16384, 32768):
            buf = torch.empty(T, vc, device=dev, dtype=torch.bfloat16)
            nch = (V + vc - 1) // vc

            def run():
                for c in range(nch):
                    lo, hi = c * vc, min(V, (c + 1) * vc)
                    torch.mm(h, W[lo:hi].t(), out=buf[:, : hi - lo])

            ms = timeit(run, 5)
            print(json.dumps({"case": "chunked", "T": T, "vc": vc, "ms": ms, "TFLOPs": fl / ms / 1e9}), flush=True)
        del full
    # backward-shaped GEMMs: dH = dZ @ W (K = V), dW = dZ^T @ h
    T = 8192
    h = torch.randn(T, H, device=dev).to(torch.bfloat16)
    dz = torch.randn(T, 16384, device=dev).to(torch.bfloat16)
    ms = timeit(lambda: torch.mm(dz, W[:16384]))
    print(json.dumps({"case": "dH_chunk", "T": T, "vc": 16384, "ms": ms, "TFLOPs": 2.0 * T * H * 16384 / ms / 1e9}))
    ms = timeit(lambda: torch.mm(dz.t(), h))
    print(json.dumps({"case": "dW_chunk", "T": T, "vc": 16384, "ms": ms, "TFLOPs": 2.0 * T * H * 16384 / ms / 1e9}))
    try:
        o = torch.mm(dz, W[:16384], out_dtype=torch.float32)
        print(json.dumps({"case": "out_dtype_f32", "ok": True, "dtype": str(o.dtype)}))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"case": "out_dtype_f32", "ok": False, "err": str(e)[:200]}))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
