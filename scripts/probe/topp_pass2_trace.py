"""Per-dispatch view of the top_p kernel's two launches (run under rocprofv3 --kernel-trace): the
R = 2 probe build of scripts/probe/topp_rbar_ab.py at [512, 151,936] bf16, T = 1, top_p = 0.95,
decode steps 0..19 three times each; prints the rows pass 1 left per step (one JSON line), so
the trace's sample_topp_pass2_kernel durations can be matched to 0 / 1 / 2 ... left rows."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
FILT = 1024 * 4


def main():
    import torch
    lib = ctypes.CDLL(os.path.join(HERE, f"libtprb_{sys.argv[1] if len(sys.argv) > 1 else 'r2'}.so"))
    dev = torch.device("cuda:0")
    N, V = 512, 151936
    logits = torch.empty((N, V), dtype=torch.bfloat16, device=dev).normal_(0, 3)
    ids = torch.arange(N, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    lib.skyrl_sample_workspace_bytes.restype = ctypes.c_size_t
    ws = torch.zeros(lib.skyrl_sample_workspace_bytes(N, V), dtype=torch.uint8, device=dev)
    tok = torch.empty(N, dtype=torch.int32, device=dev)
    lp = torch.empty(N, dtype=torch.float32, device=dev)
    left = []
    for t in range(20):
        for _ in range(3):
            rc = lib.skyrl_sample(ctypes.c_void_p(logits.data_ptr()), 1, ctypes.c_int64(V), N, V, ctypes.c_float(1.0),
                                  -1, ctypes.c_float(0.95), ctypes.c_float(0.0), ctypes.c_uint64(3),
                                  ctypes.c_void_p(ids.data_ptr()), ctypes.c_int64(t), ctypes.c_void_p(tok.data_ptr()),
                                  ctypes.c_void_p(lp.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                  ctypes.c_void_p(s.cuda_stream))
            assert rc == 0
        torch.cuda.synchronize()
        left.append(int((ws[FILT:FILT + 20 * N].view(torch.int32).view(N, 5)[:, 1] != 1).sum()))
    print(json.dumps({"rows_left_per_step": left}), flush=True)


if __name__ == "__main__":
    main()
