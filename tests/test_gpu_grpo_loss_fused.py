"""a4 + a7 in one launch (skyrl_grpo_ppo_loss_fwd): the GRPO advantage computed inside the
loss launch must give BIT-IDENTICAL advantages, loss, metrics and gradients to the two-call
path (skyrl_grpo_advantage, then skyrl_ppo_loss_fwd), whose parity with the reference-made
golden vectors and the oracle is pinned in test_gpu_parity.py; one case is also checked
against the oracle directly (advantages 1e-6, loss 1e-6 / 1e-5 rel, gradients 1e-4 rel).
Cases cover the one-launch kernel (XCD group map and plain map, every mask dtype, singleton
groups, two column chunks) and the two-launch fallback (R % 4 != 0, > 2048 row chunks).

Every case also runs the product forms: the pack kernel's GRPO scores instead of the reward
reads (``scores=``), and the fold deferred to the backward launch (``defer_fold=True``:
skyrl_ppo_loss_finish folds the per-block records and rescales); both bit-identical too."""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import ops, ppo_utils
from skyrl_amd.config import AlgorithmConfig

pytestmark = pytest.mark.gpu

CASES = [  # n, G, R, response-mask dtype, reduction, dual_clip, entropy loss, loss mask != response mask
    (512, 8, 1024, torch.int64, "token_mean", False, False, False),  # the bench's leg: XCD map
    (48, 4, 1024, torch.float32, "sequence_mean", True, True, True),  # 12 groups: plain map
    (64, 8, 2048, torch.uint8, "seq_mean_token_sum_norm", True, False, False),  # two chunks per row
    (40, 1, 1024, torch.int32, "token_mean", False, True, True),  # singleton groups
    (96, 16, 300, torch.int64, "token_mean", True, False, False),  # R % 4 != 0: ops composes the two calls
    (2560, 8, 1024, torch.int64, "token_mean", False, False, True),  # > 2048 chunks: two launches
]


def _inputs(n, R, G, mdt, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(0, R + 1, (n,), generator=g)
    rmask = (torch.arange(R)[None] < lens[:, None]).to(mdt)
    rew = torch.zeros(n, R)
    hit = lens > 0
    rew[torch.arange(n)[hit], lens[hit] - 1] = (torch.rand(int(hit.sum()), generator=g) < 0.4).float()
    rew += 0.01 * torch.randn(n, R, generator=g) * rmask.float()  # dense token rewards too
    lp = -2 + 0.1 * torch.randn(n, R, generator=g)
    old = lp + 0.1 * torch.randn(n, R, generator=g)  # ratios far enough from 1 to clip
    ref = lp + 0.05 * torch.randn(n, R, generator=g)
    ent = torch.rand(n, R, generator=g)
    return rew, rmask, lp, old, ref, ent


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}_G{c[1]}_R{c[2]}" for c in CASES])
def test_fused_matches_two_calls_bit_exact(dev, case):
    n, G, R, mdt, red, dual, use_ent, sep_mask = case
    rew, rmask, lp, old, ref, ent = _inputs(n, R, G, mdt, n * 7 + R)
    lmask = rmask.float()
    if sep_mask:  # multi-turn style: some response tokens carry no loss
        lmask = lmask * (torch.arange(R)[None] % 5 != 2).float()
    ng = n // G
    cfg = AlgorithmConfig(loss_reduction=red, max_seq_len=R, use_entropy_loss=use_ent, entropy_loss_coef=0.01,
                          policy_loss_type="dual_clip" if dual else "regular")
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=use_ent, has_entropy=True)
    d = {k: v.to(dev) for k, v in dict(rew=rew, rmask=rmask, lp=lp, old=old, ref=ref, ent=ent, lmask=lmask).items()}
    rows = d["lmask"].sum(-1)
    scores = torch.empty(n, device=dev)  # the GRPO kernel's own row sums (= pack's reward_row_sum)
    ops.grpo_advantage(d["rew"], d["rmask"], None, None, ng, scores_out=scores)
    runs = []
    # (fused, scores given, deferred fold, advantages output); the first is the two-call reference.
    # Without the advantages output the response mask is not read (loss_mask <= response_mask here)
    for fused, with_scores, defer, want_adv in ((False, False, False, True), (True, False, False, True),
                                                (True, True, True, True), (True, False, True, True),
                                                (False, True, True, True), (True, True, True, False)):
        x = d["lp"].clone().requires_grad_(True)
        en = d["ent"].clone().requires_grad_(use_ent)
        sc = scores if with_scores else None
        if fused:
            adv, loss, m = ops.grpo_ppo_loss(d["rew"], d["rmask"], ng, x, d["old"], d["lmask"], params, d["ref"], en,
                                             loss_mask_row_sum=rows, scores=sc, defer_fold=defer,
                                             want_advantages=want_adv, mask_within_response=not want_adv)
            if not want_adv:
                assert adv is None
                adv = runs[0][0]
        else:
            adv = ops.grpo_advantage(d["rew"], d["rmask"], None, None, ng, scores=sc)
            loss, m = ops.ppo_loss(x, d["old"], adv, d["lmask"], params, d["ref"], en, loss_mask_row_sum=rows,
                                   defer_fold=defer)
        (loss * 1.5).backward()
        runs.append((adv.cpu(), loss.detach().cpu(), m.cpu(), x.grad.cpu(), en.grad.cpu() if use_ent else None))
    a0, l0, m0, g0, e0 = runs[0]
    for k, (a1, l1, m1, g1, e1) in enumerate(runs[1:], 1):
        assert torch.equal(a0, a1), (k, "advantages differ from skyrl_grpo_advantage")
        assert torch.equal(l0, l1) and torch.equal(m0[:6], m1[:6]), (k, l0, l1, m0, m1)
        assert m1[6] == 0  # no fold timed out
        assert torch.equal(g0, g1), (k, "dL/dlogp differs from the two-call path")
        if use_ent:
            assert torch.equal(e0, e1), k
    assert float(m0[4]) > 0  # the clip branch ran


def test_fused_vs_oracle(dev):
    n, G, R = 512, 8, 1024
    rew, rmask, lp, old, ref, ent = _inputs(n, R, G, torch.int64, 99)
    mask = rmask.float()
    cfg = AlgorithmConfig(policy_loss_type="dual_clip")
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, has_entropy=True)
    x = lp.to(dev).requires_grad_(True)
    adv, loss, m = ops.grpo_ppo_loss(rew.to(dev), rmask.to(dev), n // G, x, old.to(dev), mask.to(dev), params,
                                     ref.to(dev), ent.to(dev), loss_mask_row_sum=mask.sum(-1).to(dev))
    loss.backward()
    uids = [str(i // G) for i in range(n)]
    eadv = cpu_ref.grpo_advantage(rew, rmask, uids)
    torch.testing.assert_close(adv.cpu(), eadv, atol=1e-6, rtol=1e-6)
    xc = lp.clone().requires_grad_(True)
    e, em = cpu_ref.policy_loss_assembly(xc, old, eadv, mask, ref, ent, dual_clip=True)
    e.backward()
    torch.testing.assert_close(loss.detach().cpu(), e.detach(), atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(m[4].cpu(), torch.as_tensor(em["clip_ratio"]).detach().float(), atol=1e-6, rtol=0)
    torch.testing.assert_close(x.grad.cpu(), xc.grad, atol=1e-9, rtol=1e-4)


def test_fused_graph_replay_and_errors(dev):
    """Replayed from a HIP graph the launch stays correct (the fold's epoch advances per
    launch); bad layouts raise through the C ABI."""
    n, G, R = 512, 8, 1024
    rew, rmask, lp, old, ref, ent = _inputs(n, R, G, torch.int64, 5)
    d = [t.to(dev) for t in (rew, rmask, lp, old, ref)]
    mask = d[1].float()
    rows = mask.sum(-1)
    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=False)
    adv0, loss0, m0 = ops.grpo_ppo_loss(d[0], d[1], n // G, d[2], d[3], mask, params, d[4], loss_mask_row_sum=rows)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        ops.grpo_ppo_loss(d[0], d[1], n // G, d[2], d[3], mask, params, d[4], loss_mask_row_sum=rows)
    torch.cuda.synchronize(dev)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        adv, loss, m = ops.grpo_ppo_loss(d[0], d[1], n // G, d[2], d[3], mask, params, d[4], loss_mask_row_sum=rows)
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(adv, adv0) and torch.equal(loss, loss0) and torch.equal(m[:7], m0[:7])
    del graph
    with pytest.raises(RuntimeError, match="n % num_groups"):
        ops.grpo_ppo_loss(d[0], d[1], 7, d[2], d[3], mask, params, d[4], loss_mask_row_sum=rows)


def test_deferred_fold_graph_replay_and_no_grad(dev):
    """The product leg as the bench replays it (C ABI, HIP graph): the deferred forward with the
    scores + skyrl_ppo_loss_finish, replayed several times, gives the eager in-launch-fold results
    bit for bit; a non-unit upstream gradient is applied by the finish launch; and a deferred call
    under no_grad folds at once (loss and metrics valid without a backward)."""
    import ctypes

    from skyrl_amd import _ffi
    from skyrl_amd.ops import _ptr

    n, G, R = 512, 8, 1024
    rew, rmask, lp, old, ref, ent = _inputs(n, R, G, torch.int64, 11)
    d = [t.to(dev) for t in (rew, rmask, lp, old, ref)]
    mask = d[1].float()
    rows = mask.sum(-1)
    scores = d[0].sum(-1)
    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=False)
    x = d[2].clone().requires_grad_(True)
    adv0, loss0, m0 = ops.grpo_ppo_loss(d[0], d[1], n // G, x, d[3], mask, params, d[4], loss_mask_row_sum=rows,
                                        scores=scores)
    (g0,) = torch.autograd.grad(loss0 * 0.25, x)
    adv, glp = torch.empty_like(d[2]), torch.empty_like(d[2])
    loss, met = torch.empty(1, device=dev), torch.empty(8, device=dev)
    gout = torch.full((1,), 0.25, device=dev)
    ws = torch.zeros(_ffi.query("skyrl_ppo_loss_workspace_bytes", n, R), dtype=torch.uint8, device=dev)

    def leg(s):
        _ffi.call("skyrl_grpo_ppo_loss_fwd", _ptr(d[0]), _ptr(scores), _ptr(d[1]), _ffi.I64, n // G, 1e-6, 1,
                  _ptr(d[2]), _ptr(d[3]), _ptr(mask), _ptr(d[4]), None, _ptr(rows), n, R, ctypes.byref(params),
                  _ptr(adv), _ptr(loss), _ptr(met), _ptr(glp), None, _ffi.LOSS_DEFER_FOLD, _ptr(ws), s)
        _ffi.call("skyrl_ppo_loss_finish", _ptr(gout), _ptr(glp), None, n, R, ctypes.byref(params), _ptr(loss),
                  _ptr(met), _ptr(ws), s)

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        leg(torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        leg(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(adv, adv0) and torch.equal(loss[0], loss0) and torch.equal(met[:7], m0[:7])
        assert torch.equal(glp, g0)
    del graph
    with torch.no_grad():
        adv1, loss1, m1 = ops.grpo_ppo_loss(d[0], d[1], n // G, d[2], d[3], mask, params, d[4],
                                            loss_mask_row_sum=rows, scores=scores, defer_fold=True)
        l2, m2 = ops.ppo_loss(d[2], d[3], adv0, mask, params, d[4], loss_mask_row_sum=rows, defer_fold=True)
    assert torch.equal(loss1, loss0) and torch.equal(m1[:7], m0[:7]) and torch.equal(adv1, adv0)
    assert torch.equal(l2, loss0) and torch.equal(m2[:7], m0[:7])
    ops.check_loss_metrics(torch.stack([m0, m1, m2]))
    bad = m0.clone()
    bad[6] = 1.0
    with pytest.raises(RuntimeError, match="timed out"):
        ops.check_loss_metrics(bad)


@pytest.mark.parametrize("rpb", [1, 2])
def test_rows_per_block_variants(dev, rpb):
    """Both block shapes of the one-launch kernel (skyrl_variant grpo_loss_rpb) give the two
    calls' outputs bit for bit."""
    from skyrl_amd import _ffi

    with _ffi.variant(grpo_loss_rpb=rpb):
        test_fused_matches_two_calls_bit_exact(dev, CASES[0])
        test_fused_matches_two_calls_bit_exact(dev, CASES[2])


@pytest.mark.parametrize("n", [4096, 777])
def test_deferred_fold_many_records_bit_identical(dev, n):
    """Many records (several passes of the fold) and a ragged count: the deferred fold gives the
    in-launch fold's loss and metrics bit for bit."""
    R = 1024
    g = torch.Generator().manual_seed(n)
    lp = (-2 + 0.1 * torch.randn(n, R, generator=g)).to(dev)
    old = lp + 0.05 * torch.randn(n, R, generator=g).to(dev)
    ref = lp + 0.05 * torch.randn(n, R, generator=g).to(dev)
    adv = torch.randn(n, R, generator=g).to(dev)
    mask = (torch.rand(n, R, generator=g) < 0.8).float().to(dev)
    rows = mask.sum(-1)
    params = ppo_utils.ppo_params_from_config(AlgorithmConfig(), use_kl_loss=True, has_entropy=False)
    l0, m0 = ops.ppo_loss(lp, old, adv, mask, params, ref, loss_mask_row_sum=rows)
    x = lp.clone().requires_grad_(True)
    l1, m1 = ops.ppo_loss(x, old, adv, mask, params, ref, loss_mask_row_sum=rows, defer_fold=True)
    l1.backward()
    assert torch.equal(l1.detach(), l0) and torch.equal(m1[:7], m0[:7])
