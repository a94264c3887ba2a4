"""Split-row fused training pass (policy_train_split_kernel: each row cut into pieces, one
workgroup each -- by default six of 256 threads for rows over 128 KB, four of 256 otherwise --
exchanging their softmax states through epoch-tagged granules in the workspace).

* a launch never reads the previous launch's granules: inputs B after inputs A on the same
  workspace give bit-for-bit what B gives on a fresh workspace (and again on replay);
* the pieces merge in one fixed order: every output is identical across repeated launches;
* rows at the metric's shape (V = 151,936, 16 x 128 tokens) against the resident kernel.
"""

import pytest
import torch

from skyrl_amd import ops, ppo_utils
from skyrl_amd.config import AlgorithmConfig

pytestmark = pytest.mark.gpu


def _inputs(seed, n, R, V, dev):
    g = torch.Generator().manual_seed(seed)
    logits = (torch.randn(n, R, V, generator=g) * 3).to(torch.bfloat16).to(dev)
    labels = torch.randint(0, V, (n, R), generator=g).to(dev)
    old = (-8 + torch.randn(n, R, generator=g)).to(dev)
    adv = torch.randn(n, R, generator=g).to(dev)
    mask = (torch.rand(n, R, generator=g) < 0.9).float().to(dev)
    ref = (-8 + torch.randn(n, R, generator=g)).to(dev)
    return logits, labels, old, adv, mask, ref


def _run(inp, params, temp=1.0):
    logits, labels, old, adv, mask, ref = inp
    x = logits.clone().requires_grad_(True)
    loss, m, lp, ent = ops.policy_train(x, labels, old, adv, mask, params, ref_log_probs=ref, temperature=temp)
    loss.backward()
    return loss.detach().clone(), m.clone(), lp.clone(), ent.clone(), x.grad.clone()


def _params():
    cfg = AlgorithmConfig(use_entropy_loss=True)
    return ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=True, has_entropy=True)


def _same(a, b):
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("V", [512, 151936])
@pytest.mark.parametrize("R", [40, 41])
@pytest.mark.parametrize("shape", [1, 2, 3, 4, 5])
def test_split_fresh_granules_every_launch(dev, V, R, shape):
    """Every built split shape (pieces x threads: 8 x 128, 4 x 256, 2 x 512, 5 x 256, 6 x 256;
    shapes whose pieces do not fit V fall back to the resident kernel); 120 and 123 rows."""
    params = _params()
    n = 3
    A, B = _inputs(1, n, R, V, dev), _inputs(2, n, R, V, dev)
    with ops.variant(train_split_shape=shape):
        ops.WORKSPACES._bufs.clear()
        ref_b = _run(B, params)  # B on a fresh workspace
        ops.WORKSPACES._bufs.clear()
        _run(A, params)
        got = _run(B, params)  # B after A on the same workspace
        _same(got, ref_b)
        _same(_run(B, params), ref_b)  # replay
    assert float(ref_b[1][6]) == 0.0
    if shape != 5:  # vs the default shape: another fp32 summation order only
        q = _run(B, params)
        for a, b in zip(ref_b[:4], q[:4]):
            torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(ref_b[4].float(), q[4].float(), atol=2e-6, rtol=1e-2)


@pytest.mark.parametrize("temp", [1.0, 0.6])
def test_split_matches_resident_at_metric_vocab(dev, temp):
    params = _params()
    inp = _inputs(3, 16, 128, 151936, dev)
    split = _run(inp, params, temp)
    with ops.variant(train_split=0):
        res = _run(inp, params, temp)
    for a, b in zip(split[:4], res[:4]):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(split[4].float(), res[4].float(), atol=2e-6, rtol=1e-2)
    # bf16 dlogits: at most a rounding apart, and nearly all bit-equal
    diff = (split[4] != res[4]).float().mean().item()
    assert diff < 0.01, diff
    assert float(split[1][6]) == 0.0


@pytest.mark.parametrize("V", [512, 151936, 50257])
@pytest.mark.parametrize("red", [0, 1, 2])
def test_ragged_matches_dense_on_padded_batch(dev, V, red):
    """skyrl_policy_train_ragged_fwd on the live tokens of a ragged batch == skyrl_policy_train_fwd
    on the padded batch (dead positions: loss mask 0, arbitrary logits): loss and metrics bit for
    bit under every loss reduction, logp / entropy at the live positions, and the live rows'
    dlogits; the dead positions of logp / entropy stay 0. GPT-2's odd V (the EDGE form): a packed
    row sits at another offset within 16 B than its padded row, so the pieces cut its span
    elsewhere: another fp32 summation order, compared at 1e-5 (dlogits within a bf16 rounding)."""
    n, R = 4, 24
    g = torch.Generator().manual_seed(V + red)
    lens = torch.tensor([24, 1, 13, 7])
    live = torch.arange(R)[None] < lens[:, None]
    logits = (torch.randn(n, R, V, generator=g) * 3).to(torch.bfloat16).to(dev)
    labels = torch.randint(0, V, (n, R), generator=g).to(dev)
    old = (-6 + torch.randn(n, R, generator=g)).to(dev)
    adv = torch.randn(n, R, generator=g).to(dev)
    ref = (-6 + torch.randn(n, R, generator=g)).to(dev)
    mask = (live & (torch.rand(n, R, generator=g) < 0.9)).float().to(dev)
    cfg = AlgorithmConfig(use_entropy_loss=True, policy_loss_type="dual_clip", loss_reduction=
                          ("token_mean", "sequence_mean", "seq_mean_token_sum_norm")[red], max_seq_len=R)
    params = ppo_utils.ppo_params_from_config(cfg, use_kl_loss=True, use_entropy_loss=True, has_entropy=True)
    x = logits.clone().requires_grad_(True)
    loss_d, m_d, lp_d, ent_d = ops.policy_train(x, labels, old, adv, mask, params, ref_log_probs=ref)
    loss_d.backward()
    lv = live.to(dev)
    z = logits[lv].contiguous().requires_grad_(True)
    pos = torch.nonzero(lv.reshape(-1)).reshape(-1).to(torch.int32)
    loss_r, m_r, lp_r, ent_r = ops.policy_train_ragged(z, labels[lv], pos, old, adv, mask, params, ref_log_probs=ref)
    loss_r.backward()
    assert not lp_r[~lv].any() and not ent_r[~lv].any()
    if V % 8:
        for a, b in ((loss_r, loss_d), (m_r[:7], m_d[:7]), (lp_r[lv], lp_d[lv]), (ent_r[lv], ent_d[lv])):
            torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(z.grad.float(), x.grad[lv].float(), atol=2e-6, rtol=1e-2)
        return
    assert torch.equal(loss_r, loss_d) and torch.equal(m_r[:7], m_d[:7])
    assert torch.equal(lp_r[lv], lp_d[lv]) and torch.equal(ent_r[lv], ent_d[lv])
    assert not lp_r[~lv].any() and not ent_r[~lv].any()
    assert torch.equal(z.grad, x.grad[lv])


@pytest.mark.parametrize("V", [1001, 8191, 50257, 100003])
@pytest.mark.parametrize("shape", [1, 2, 3])
def test_split_edge_rows_match_resident(dev, V, shape):
    """Rows with partial vectors (odd V on the model-wrapper slice [:, -R-1:-1], so each row sits
    at another offset within 16 B): the split kernel's EDGE form vs the resident EDGE kernel, and
    the dlogits of positions outside the slice stay exactly 0 (partial vectors write only their
    own row's slots)."""
    params = _params()
    n, S, R = 3, 21, 17
    g = torch.Generator().manual_seed(V + shape)
    logits = (torch.randn(n, S, V, generator=g) * 3).to(torch.bfloat16).to(dev)
    labels = torch.randint(0, V, (n, R), generator=g).to(dev)
    labels[0, 0], labels[1, 1], labels[2, 2] = 0, V - 1, V - 2  # labels in the partial vectors
    old = (-6 + torch.randn(n, R, generator=g)).to(dev)
    adv = torch.randn(n, R, generator=g).to(dev)
    mask = (torch.rand(n, R, generator=g) < 0.9).float().to(dev)
    ref = (-6 + torch.randn(n, R, generator=g)).to(dev)
    outs = []
    for split in (1, 0):
        with ops.variant(train_split_shape=shape, train_split=split):
            full = logits.clone().requires_grad_(True)
            loss, m, lp, ent = ops.policy_train(full[:, -R - 1:-1], labels, old, adv, mask, params, ref_log_probs=ref,
                                                temperature=0.8)
            loss.backward()
        outs.append((loss.detach(), m.clone(), lp, ent, full.grad))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(outs[0][4].float(), outs[1][4].float(), atol=2e-6, rtol=1e-2)
    assert float(outs[0][1][6]) == 0.0
    grad = outs[0][4]
    assert torch.count_nonzero(grad[:, :S - R - 1]) == 0 and torch.count_nonzero(grad[:, -1]) == 0
    live = grad[:, -R - 1:-1][mask.bool()]  # masked tokens have zero dlogits
    assert torch.count_nonzero(live) > 0.9 * live.numel()


def _recomputed(dev, n, R):
    """Header word 33 of the per-call workspace: partner states a piece computed itself."""
    ws = ops.WORKSPACES.get(dev, "policy_train", ops._ffi.query("skyrl_policy_train_workspace_bytes", n, R))
    return int(ws[132:136].view(torch.int32).item())


def test_partner_states_computed_in_place_give_the_same_bits(dev):
    """skyrl_variant train_split_wait = 0: a piece does not wait for any partner that has not
    published at its first poll and computes that partner's state from the partner's slice
    (the path a piece takes when its partners are not resident). The pieces' states are the
    same bits either way, so loss, metrics, logp, entropy and dlogits equal the default run's
    bit for bit, at the metric's V and an EDGE vocabulary (GPT-2's 50,257)."""
    params = _params()
    for V in (151936, 50257):  # (odd V: rows of a contiguous [n, R, V] tensor are not 16-B aligned)
        inp = _inputs(21, 4, 64, V, dev)
        base = _run(inp, params)
        n, R = inp[1].shape
        c0 = _recomputed(dev, n, R)
        with ops.variant(train_split_wait=0):
            forced = _run(inp, params)
        assert _recomputed(dev, n, R) > c0, V  # the in-place path ran
        for a, b in zip(base, forced):
            assert torch.equal(a, b), V


def occupy(*args):
    """tests/csrc/occupy.hip (a test hook library, not part of libskyrl_hip.so)."""
    import ctypes
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libskyrl_testhooks.so")
    fn = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL).skyrl_test_occupy
    fn.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    assert fn(*args) == 0


def test_split_pass_beside_a_kernel_holding_the_cus(dev):
    """the split pass on one stream while another stream's kernel holds every
    CU slot and releases them a few at a time (64 groups of workgroups ending 20 us apart), so the
    pieces of a row are dispatched far apart. No piece may wait on a partner's residency: no
    timeout flag, and the same bits as the uncontended run."""
    params = _params()
    inp = _inputs(5, 8, 256, 151936, dev)
    base = _run(inp, params)
    side = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(side):
        occupy(512, 1024, 100_000, 2_000, ops._stream(dev))
    out = _run(inp, params)  # current stream: runs beside the occupier
    torch.cuda.synchronize(dev)
    assert float(out[1][6]) == 0.0  # no split-exchange error
    for a, b in zip(base, out):
        assert torch.equal(a, b)
