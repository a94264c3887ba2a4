"""Edge cases on the HIP path, each against the oracle: empty / single-element / ragged inputs,
all-masked rows, tiny and odd vocabularies, unaligned strides, extreme values."""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import ops, ppo_utils

pytestmark = pytest.mark.gpu


def close(a, b, atol=1e-5, rtol=1e-5):
    torch.testing.assert_close(torch.as_tensor(a).detach().float().cpu(), torch.as_tensor(b).detach().float().cpu(),
                               atol=atol, rtol=rtol)


def test_sample_empty_batch_and_tiny_vocab(dev):
    tok, lp = ops.sample(torch.empty(0, 7, device=dev), seed=1)
    assert tok.numel() == 0 and lp.numel() == 0
    x = torch.tensor([[3.0], [-2.0]], device=dev)  # V = 1: the only token, logprob 0
    tok, lp = ops.sample(x, seed=1)
    assert tok.tolist() == [0, 0]
    close(lp, torch.zeros(2))
    tok, _ = ops.sample(x, temperature=0.0)
    assert tok.tolist() == [0, 0]


def test_sample_greedy_ties_lowest_index(dev):
    x = torch.zeros(3, 1000, device=dev)
    x[0, [7, 500]] = 5.0
    x[1, [999, 998]] = 2.0
    tok, _ = ops.sample(x, temperature=0.0)
    assert tok.tolist() == [7, 998, 0]


def test_grpo_singletons_and_zero_variance(dev):
    rew = torch.zeros(5, 4)
    rew[:, -1] = torch.tensor([1.0, 1.0, 0.5, 2.0, 0.0])
    mask = torch.ones(5, 4, dtype=torch.int64)
    uids = ["a", "a", "b", "c", "c"]  # a: zero variance, b: singleton, c: two values
    adv, _ = ppo_utils.compute_grpo_outcome_advantage(rew.to(dev), mask.to(dev), uids)
    close(adv, cpu_ref.grpo_advantage(rew, mask, uids), atol=1e-6)
    assert adv[0].abs().max() == 0 and adv[1].abs().max() == 0


def test_gae_single_column_and_error_paths(dev):
    r = torch.tensor([[1.0], [0.5], [0.0]])
    v = torch.tensor([[0.2], [0.1], [0.3]])
    m = torch.ones(3, 1)
    a, ret = ops.gae_advantage_return(r.to(dev), v.to(dev), m.to(dev), 1.0, 0.95)
    ea, eret = cpu_ref.gae(r, v, m, 1.0, 0.95)
    close(a, ea, atol=1e-5)
    close(ret, eret, atol=1e-6)
    with pytest.raises(ValueError, match="At least one element"):
        ops.gae_advantage_return(r.to(dev), v.to(dev), torch.zeros(3, 1, device=dev), 1.0, 0.95)


def test_ppo_loss_all_masked_rows(dev):
    g = torch.Generator().manual_seed(2)
    n, R = 4, 9
    lp = -1 + 0.1 * torch.randn(n, R, generator=g)
    old = lp + 0.05 * torch.randn(n, R, generator=g)
    adv = torch.randn(n, R, generator=g)
    mask = torch.ones(n, R)
    mask[1] = 0  # a fully masked row (pad row from pad_batch)
    for red in ("token_mean", "sequence_mean", "seq_mean_token_sum_norm"):
        params = ops.make_ppo_params(loss_reduction=red, max_seq_len=12)
        x = lp.to(dev).requires_grad_(True)
        loss, m = ops.ppo_loss(x, old.to(dev), adv.to(dev), mask.to(dev), params)
        loss.backward()
        xr = lp.clone().requires_grad_(True)
        el, _ = cpu_ref.ppo_policy_loss(xr, old, adv, mask=mask, reduction=red, max_seq_len=12)
        el.backward()
        close(loss, el, atol=1e-6)
        close(x.grad, xr.grad, atol=1e-7)
        assert float(x.grad[1].abs().max()) == 0.0


def test_logprob_tiny_odd_vocab_and_strided_labels(dev):
    g = torch.Generator().manual_seed(4)
    for V in (1, 3, 9, 17):
        logits = (torch.randn(2, 5, V, generator=g) * 4).to(torch.bfloat16)
        big = torch.randint(0, V, (2, 11), generator=g)
        labels = big[:, 1:11:2]  # non-unit label stride
        lp, ent = ops.logprobs_and_entropy(logits.to(dev), labels.to(dev))
        close(lp, cpu_ref.logprobs_from_logits(logits.float(), labels), atol=1e-5)
        close(ent, cpu_ref.entropy_from_logits(logits.float()), atol=1e-4)


def test_pack_empty_prompt_and_single_token_response(dev):
    from skyrl_amd import trainer_utils as tu

    go = {"prompt_token_ids": [[], [5, 6], [7]], "response_ids": [[1], [2, 3, 4], [9]],
          "rewards": [[0.0], [0.0, 0.0, 1.0], [0.5]], "loss_masks": [[1], [1, 0, 1], [1]],
          "rollout_logprobs": [[-0.1], [-0.2, -0.3, -0.4], [-0.5]]}
    b = tu.convert_to_training_input(go, ["0", "1", "2"], 99, dp_size=4, device=dev)
    ref = cpu_ref.pack(go["prompt_token_ids"], go["response_ids"], go["rewards"], go["loss_masks"],
                       go["rollout_logprobs"], 99, pad=1)
    for k, v in zip(("sequences", "attention_mask", "response_mask", "rewards", "loss_mask", "rollout_logprobs"), ref):
        assert torch.equal(b[k].cpu(), torch.from_numpy(v)), k


def test_reward_kl_zero_coef_is_identity(dev):
    g = torch.Generator().manual_seed(5)
    rew = torch.randn(3, 6, generator=g)
    lp = torch.randn(3, 6, generator=g)
    out, m = ops.reward_kl_penalty(rew.to(dev), lp.to(dev), (lp + 0.3).to(dev), torch.ones(3, 6, device=dev), "k3",
                                   0.0)
    close(out, rew, atol=0, rtol=0)
    assert float(m[0]) > 0  # the KL metric is still reported


@pytest.mark.parametrize("G,R,mdt", [(8, 1024, torch.int64), (1, 64, torch.float32), (16, 36, torch.bool),
                                     (5, 256, torch.int32)])
def test_grpo_contiguous_form_matches_csr_and_oracle(dev, G, R, mdt):
    """The index-free kernel (contiguous equal groups) is bit-identical to the CSR kernel."""
    g = torch.Generator().manual_seed(G * 100 + R)
    N = 6 * G
    rew = torch.zeros(N, R)
    lens = torch.randint(1, R + 1, (N,), generator=g)
    rew[torch.arange(N), lens - 1] = torch.randint(0, 3, (N,), generator=g).float()
    mask = (torch.arange(R)[None] < lens[:, None]).to(mdt)
    uids = [str(i // G) for i in range(N)]
    off, rows, ng = ops.groups_from_index(uids)
    assert ops.contiguous_group_size(off, rows, ng) == G
    a_csr = ops.grpo_advantage(rew.to(dev), mask.to(dev), off, rows, ng)
    a_fast = ops.grpo_advantage(rew.to(dev), mask.to(dev), None, None, ng)
    assert torch.equal(a_csr, a_fast)
    close(a_fast, cpu_ref.grpo_advantage(rew, mask.to(torch.int64), uids), atol=1e-6)
    # an unaligned view takes the CSR kernel through the same call
    big = torch.zeros(N * R + 1, device=dev)
    view = big[1:].view(N, R)
    view.copy_(rew.to(dev))
    assert torch.equal(ops.grpo_advantage(view, mask.to(dev), None, None, ng), a_csr)
