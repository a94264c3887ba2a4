"""a12/a14 HIP optimizer step vs the reference optimizer (torch AdamW + clip_grad_norm_, CPU fp32).

Reference: PolicyWorkerBase.optim_step (workers/worker.py:900-925) -> FSDPStrategy.optimizer_step
(distributed/fsdp_strategy.py:160-190) with optim.AdamW (:284-296) and clip (fsdp_utils.py:388-401).
Tolerance: fp32 vs the same algorithm in fp64, rtol 1e-5 on norms and parameters after several
steps; the bf16 rollout copy must equal
param.to(bfloat16) bit for bit.
"""

import math

import pytest
import torch

from skyrl_amd import comm, ops

pytestmark = pytest.mark.gpu


def _ref_steps(p0, grads, cfg, n_micro):
    # the reference algorithm run in float64: torch's fp32 CPU norm accumulates in fp32 (6e-5
    # relative error at 3M elements), the HIP sum of squares in fp64
    w = torch.nn.Parameter(p0.clone().double())
    opt = torch.optim.AdamW([w], lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay)
    norms = []
    for g in grads:
        w.grad = g.clone().double() * (1.0 / n_micro)  # optim_step scaling
        norm = torch.nn.utils.clip_grad_norm_([w], max_norm=cfg.max_grad_norm)
        norms.append(float(norm))
        if math.isfinite(float(norm)):
            opt.step()
        opt.zero_grad()
    return w.detach().float(), norms


@pytest.mark.parametrize("numel", [1, 4099, 3 * (1 << 20) + 5])
def test_adamw_matches_torch(dev, numel):
    torch.manual_seed(numel)
    cfg = comm.AdamWConfig(lr=1e-3, max_grad_norm=1.0)
    p0 = torch.randn(numel)
    grads = [torch.randn(numel) * s for s in (0.01, 5.0, 0.2)]  # clip inactive, active, inactive
    red = comm.GradReducer(numel, dev)
    opt = comm.ShardedAdamW(red, p0.to(dev), cfg)
    norms = []
    for g in grads:
        red.grad[:numel] = g.to(dev)
        norms.append(float(opt.step(n_micro=4)))
    ref, ref_norms = _ref_steps(p0, grads, cfg, 4)
    assert norms == pytest.approx(ref_norms, rel=1e-5)
    got = opt.param[:numel].cpu()
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-7), (got - ref).abs().max()
    assert torch.equal(opt.weights_bf16[:numel].cpu(), opt.param[:numel].cpu().to(torch.bfloat16))
    assert int(opt.step_count.item()) == 3
    assert float(red.grad.abs().max()) == 0.0  # zero_grad


def test_adamw_skips_non_finite_norm(dev):
    numel = 1000
    cfg = comm.AdamWConfig(lr=1e-2)
    p0 = torch.randn(numel)
    red = comm.GradReducer(numel, dev)
    opt = comm.ShardedAdamW(red, p0.to(dev), cfg)
    g = torch.randn(numel)
    g[7] = float("inf")
    red.grad[:numel] = g.to(dev)
    norm = float(opt.step())
    assert not math.isfinite(norm)
    assert torch.equal(opt.param[:numel].cpu(), p0)
    assert int(opt.step_count.item()) == 0
    red.grad[:numel] = torch.randn(numel, device=dev)
    opt.step()
    assert int(opt.step_count.item()) == 1
    assert not torch.equal(opt.param[:numel].cpu(), p0)


def test_sumsq_deterministic_and_exact(dev):
    torch.manual_seed(3)
    for n in (0, 3, 1 << 20, 50_000_001):
        x = torch.randn(n, device=dev)
        ws = torch.zeros(int(ops._ffi.query("skyrl_sumsq_workspace_bytes", n)), dtype=torch.uint8, device=dev)
        outs = []
        for _ in range(2):
            o = torch.zeros(1, device=dev)
            ops._ffi.call("skyrl_sumsq", ops._ptr(x), n, ops._ptr(o), ops._ptr(ws), ops._stream(dev))
            outs.append(float(o))
        assert outs[0] == outs[1]
        ref = float((x.double() ** 2).sum()) if n else 0.0
        assert outs[0] == pytest.approx(ref, rel=1e-6, abs=1e-30)


def test_cast_bf16_round_to_nearest_even(dev):
    x = torch.randn(10_001, device=dev) * 100
    x[:4] = torch.tensor([1.00390625, 1.01171875, float("nan"), -0.0], device=dev)  # ties, NaN, -0
    y = torch.empty(x.numel(), dtype=torch.bfloat16, device=dev)
    ops._ffi.call("skyrl_cast_bf16", ops._ptr(x), ops._ptr(y), x.numel(), ops._stream(dev))
    ref = x.cpu().to(torch.bfloat16)
    assert torch.equal(y.cpu().view(torch.int16)[3:], ref.view(torch.int16)[3:])
    assert torch.equal(y.cpu()[:2], ref[:2]) and torch.isnan(y[2].float())


def test_module_optimizer_skips_parameters_without_grad(dev):
    """ShardedModuleOptimizer (the trainer's "hip" optimizer) on a module with a parameter no
    backward reaches: like torch.optim.AdamW with a None grad, that parameter, its moments and
    its bf16 engine copy stay as they were, while the used ones match torch AdamW +
    clip_grad_norm_ (1e-6). Then the parameter is used and is updated with its OWN step count's
    bias correction (torch's per-parameter state["step"]), on the device (no host read)."""

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(64, 32)
            self.unused = torch.nn.Parameter(torch.randn(1000))
            self.b = torch.nn.Linear(16, 3)  # odd sizes: segments that do not start on a 16-B vector

        def forward(self, x, use=False):
            y = self.a(x).square().mean() + self.b(x[:, :16]).sum()
            return y + self.unused.sum() if use else y

    torch.manual_seed(0)
    m = M().to(dev)
    ref = M().to(dev)
    ref.load_state_dict(m.state_dict())
    cfg = comm.AdamWConfig(lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
    opt = comm.ShardedModuleOptimizer(m, cfg)
    topt = torch.optim.AdamW(ref.parameters(), lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay)
    u0 = m.unused.detach().clone()
    named_bf16 = dict(opt.named_bf16())
    ub0 = named_bf16["unused"].clone()
    for it in range(5):
        use = it in (2, 4)
        x = torch.randn(8, 64, device=dev)
        m(x, use).backward()
        opt.step(1)
        ref(x, use).backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), cfg.max_grad_norm)
        topt.step()
        topt.zero_grad(set_to_none=True)
        if it < 2:
            assert torch.equal(m.unused.detach(), u0)
            assert torch.equal(dict(opt.named_bf16())["unused"], ub0)  # the engine copy too (world 1)
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), atol=1e-6, rtol=1e-5, msg=f"{n} step {it}")
        for n, w in opt.named_bf16():
            assert torch.equal(w, dict(m.named_parameters())[n].detach().to(torch.bfloat16)), n
    assert not torch.equal(m.unused.detach(), u0)
    steps = opt.segments.param_step.tolist()
    assert steps[opt._index[id(m.unused)]] == 2 and max(steps) == 5  # per-parameter counts
