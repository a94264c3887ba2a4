"""lm_head logprob paths at the config-2 shape (H=1536, V=151936): fused (V-chunked GEMM + HIP
online softmax) vs unfused (whole-V GEMM -> bf16 logits -> HIP logprob kernel) vs the
reference's torch formulation. Forward-only (old/ref logprob passes) and forward+backward
(policy training pass). One JSON line per case."""

import argparse
import json

import torch

from skyrl_amd import lmhead, ops


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[4096, 8192])
    ap.add_argument("--H", type=int, default=1536)
    ap.add_argument("--V", type=int, default=151936)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--chunks", type=int, nargs="*", default=[0])
    args = ap.parse_args()
    dev = torch.device("cuda")
    H, V = args.H, args.V
    W = (torch.randn(V, H, device=dev) * 0.02).to(torch.bfloat16).requires_grad_(True)
    for T in args.T:
        h = torch.randn(T, H, device=dev).to(torch.bfloat16).requires_grad_(True)
        lab = torch.randint(0, V, (T,), device=dev)
        gl = torch.randn(T, device=dev)
        fl = 2.0 * T * H * V
        res = {"T": T, "H": H, "V": V, "gemm_tflop": fl / 1e12}

        def unfused_fwd():
            with torch.no_grad():
                z = torch.mm(h, W.t())
                return ops.logprobs_and_entropy(z, lab, 1.0)

        def torch_fwd():  # the reference formulation (torch_utils.py:136-145 _v2 + :59-111)
            with torch.no_grad():
                z = torch.mm(h, W.t()).float()
                lp = torch.log_softmax(z, -1)
                return lp.gather(-1, lab[:, None]), -(lp.exp() * lp).sum(-1)

        res["unfused_fwd_ms"] = timeit(unfused_fwd, args.iters)
        res["torch_fwd_ms"] = timeit(torch_fwd, args.iters)
        for c in args.chunks:
            def fused_fwd():
                with torch.no_grad():
                    return lmhead.lmhead_logprobs_and_entropy(h, W, lab, 1.0, True, c or None)
            res[f"fused_fwd_ms_c{c}"] = timeit(fused_fwd, args.iters)

            def fused_fb():
                lp, ent = lmhead.lmhead_logprobs_and_entropy(h, W, lab, 1.0, True, c or None)
                torch.autograd.backward([lp, ent], [gl, gl])
            res[f"fused_fwdbwd_ms_c{c}"] = timeit(fused_fb, max(2, args.iters // 2))
            h.grad = None
            W.grad = None

        def unfused_fb():
            z = torch.mm(h, W.t())
            lp, ent = ops.logprobs_and_entropy(z, lab, 1.0)
            torch.autograd.backward([lp, ent], [gl, gl])

        res["unfused_fwdbwd_ms"] = timeit(unfused_fb, max(2, args.iters // 2))
        h.grad = None
        W.grad = None

        # the training pass with the PPO loss included: (a) chunked lm_head logprob + HIP loss,
        # (b) whole-V GEMM + the fused policy pass (logprob + entropy + loss + dlogits in one
        # memory pass, split rows) + the dh / dW GEMMs
        from skyrl_amd import ppo_utils
        from skyrl_amd.config import AlgorithmConfig

        params = ppo_utils.ppo_params_from_config(AlgorithmConfig(use_entropy_loss=True), use_kl_loss=False,
                                                  use_entropy_loss=True, has_entropy=True)
        old = (-12 + torch.randn(1, T, device=dev))
        adv = torch.randn(1, T, device=dev)
        msk = torch.ones(1, T, device=dev)

        def chunked_loss_fb():
            lp, ent = lmhead.lmhead_logprobs_and_entropy(h, W, lab, 1.0, True, None)
            loss, _ = ops.ppo_loss(lp.view(1, T), old, adv, msk, params, entropy=ent.view(1, T))
            loss.backward()

        def policy_train_fb():
            z = torch.mm(h, W.t())
            loss, _, _, _ = ops.policy_train(z.view(1, T, V), lab.view(1, T), old, adv, msk, params)
            loss.backward()

        res["chunked_loss_fwdbwd_ms"] = timeit(chunked_loss_fb, max(2, args.iters // 2))
        h.grad = None
        W.grad = None
        res["policy_train_fwdbwd_ms"] = timeit(policy_train_fb, max(2, args.iters // 2))
        h.grad = None
        W.grad = None
        res["addmm_f32"] = lmhead._ADDMM_F32[0]
        res["fused_fwd_TFLOPs"] = fl / res[f"fused_fwd_ms_c{args.chunks[0]}"] / 1e9
        res["peak_mem_GB"] = torch.cuda.max_memory_allocated() / 1e9
        print(json.dumps(res), flush=True)
        torch.cuda.reset_peak_memory_stats()


if __name__ == "__main__":
    main()
