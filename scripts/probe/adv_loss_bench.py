"""Advantage + loss kernels at the north-star size (N=512, R=1024), for per-kernel durations
under `rocprofv3 --kernel-trace --stats` (the HIP-event view includes host launch gaps)."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from skyrl_amd import ops, ppo_utils  # noqa: E402
from skyrl_amd.config import AlgorithmConfig  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, R, G = 512, 1024, 8
    g = torch.Generator(device=dev).manual_seed(0)
    rew = torch.zeros(N, R, device=dev)
    lens = torch.randint(1, R + 1, (N,), device=dev, generator=g)
    rew[torch.arange(N, device=dev), lens - 1] = (torch.rand(N, device=dev, generator=g) < 0.3).float()
    mask = (torch.arange(R, device=dev)[None] < lens[:, None]).to(torch.int64)
    goff, grows, ng = ops.groups_from_index([str(i // G) for i in range(N)])
    lmask = mask.float()
    lp = -2 + 0.1 * torch.randn(N, R, device=dev, generator=g)
    old = lp + 0.05 * torch.randn(N, R, device=dev, generator=g)
    ref = lp + 0.05 * torch.randn(N, R, device=dev, generator=g)
    vals = torch.randn(N, R, device=dev, generator=g)
    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=False)
    iters = int(os.environ.get("ITERS", "200"))
    for _ in range(iters):
        adv = ops.grpo_advantage(rew, mask, None, None, ng)
        ops.grpo_advantage(rew, mask, goff, grows, ng)
        x = lp.requires_grad_(True)
        loss, m = ops.ppo_loss(x, old, adv, lmask, params, ref_log_probs=ref)
        (gx,) = torch.autograd.grad(loss, x)
        ops.gae_advantage_return(rew, vals, mask, 1.0, 0.95, check=False)
        ops.reward_kl_penalty(rew, lp.detach(), ref, lmask, "k3", 0.01)
    torch.cuda.synchronize()
    print("ok", float(loss), float(gx.abs().sum()))


if __name__ == "__main__":
    main()
