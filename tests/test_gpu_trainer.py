"""Trainer-level wrappers on the HIP path vs the reference's fixtures and the oracle.

convert_to_training_input (trainer.py:592-666 + pad_batch :872-907) from Python lists against
tests/golden/pack.npz (written by the reference's convert_prompts_responses_to_batch_tensors
and pad_batch); compute_advantages_and_returns (trainer.py:759-862) against the GRPO golden
plus the oracle's metric formulas; apply_reward_kl_penalty (trainer.py:981-1035) against the
reward-KL golden (its avg_kl/avg_kl_max include the reference test's 0.3143/0.1249 case).
"""

import pytest
import torch

from oracle import cpu_ref
from skyrl_amd import trainer_utils as tu
from skyrl_amd.config import AlgorithmConfig
from skyrl_amd.training_batch import TrainingInputBatch

pytestmark = pytest.mark.gpu


def _ragged(vals, off):
    v = vals.tolist()
    o = off.tolist()
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def test_convert_to_training_input_matches_golden(golden, dev):
    d = golden("pack")
    go = {
        "prompt_token_ids": _ragged(d["prompt_vals"], d["prompt_off"]),
        "response_ids": _ragged(d["response_vals"], d["response_off"]),
        "rewards": _ragged(d["reward_vals"], d["reward_off"]),
        "loss_masks": _ragged(d["loss_mask_vals"], d["loss_mask_off"]),
        "rollout_logprobs": _ragged(d["logprob_vals"], d["logprob_off"]),
    }
    N = len(go["response_ids"])
    pad = int(d["pad_size"])
    batch = tu.convert_to_training_input(go, [str(i) for i in range(N)], int(d["pad_token_id"]), dp_size=N + pad,
                                         device=dev)
    for k in ("sequences", "attention_mask", "response_mask", "rewards", "loss_mask", "rollout_logprobs"):
        assert torch.equal(batch[k].cpu(), d["p_" + k]), k
    assert batch.metadata["uids"] == [str(u) for u in d["p_uids"]]
    assert batch.metadata["pad_size"] == pad
    assert batch.metadata["response_length"] == d["p_response_mask"].shape[1]
    # no padding requested: the unpadded reference tensors
    b0 = tu.convert_to_training_input(go, [str(i) for i in range(N)], int(d["pad_token_id"]), dp_size=1, device=dev)
    assert torch.equal(b0["sequences"].cpu(), d["sequences"])


def test_compute_advantages_and_returns_metrics(golden, dev):
    d = golden("grpo_mixed")
    n = d["rewards"].shape[0]
    batch = TrainingInputBatch({"rewards": d["rewards"].to(dev), "response_mask": d["response_mask"].to(dev)})
    batch.metadata = {"uids": [str(u) for u in d["uids"]], "avg_response_length": 7.0, "pad_size": 2}
    cfg = AlgorithmConfig()
    out = tu.compute_advantages_and_returns(batch, cfg)
    assert torch.allclose(out["advantages"].cpu(), d["adv_norm1"], atol=1e-5)
    adv = d["adv_norm1"][: n - 2]
    m = d["response_mask"][: n - 2].bool()
    valid = torch.masked_select(adv, m)
    met = out.metadata["metrics"]
    assert met["avg_final_rewards"] == pytest.approx(float(d["rewards"].sum(-1)[: n - 2].mean()), abs=1e-6)
    assert met["avg_advantages"] == pytest.approx(float(valid.mean()), abs=1e-5)
    assert met["avg_advantages_abs"] == pytest.approx(float(valid.abs().mean()), abs=1e-5)
    assert met["avg_response_length"] == 7.0


def test_apply_reward_kl_penalty_matches_golden(golden, dev):
    d = golden("reward_kl")
    for kind in ("k1", "k3"):
        batch = TrainingInputBatch({k: d[k].to(dev) for k in ("rewards", "loss_mask", "action_log_probs",
                                                              "base_action_log_probs")})
        batch.metadata = {}
        cfg = AlgorithmConfig()
        cfg.kl_estimator_type = kind
        cfg.kl_loss_coef = float(d["kl_coef"])
        out = tu.apply_reward_kl_penalty(batch, cfg)
        assert torch.allclose(out["rewards"].cpu(), d[f"rewards_{kind}"], atol=1e-6)
        met = out.metadata["metrics"]
        assert met["avg_kl"] == pytest.approx(float(d[f"avg_kl_{kind}"]), abs=1e-6)
        assert met["avg_kl_max"] == pytest.approx(float(d[f"avg_kl_max_{kind}"]), abs=1e-6)
        assert met["kl_loss_coef"] == cfg.kl_loss_coef


def test_convert_large_ragged_batch_vs_oracle(dev):
    g = torch.Generator().manual_seed(5)
    N = 96
    plen = torch.randint(1, 300, (N,), generator=g).tolist()
    rlen = torch.randint(1, 700, (N,), generator=g).tolist()
    prompts = [torch.randint(0, 151936, (k,), generator=g).tolist() for k in plen]
    resps = [torch.randint(0, 151936, (k,), generator=g).tolist() for k in rlen]
    rewards = [[0.0] * (k - 1) + [float(i % 2)] for i, k in enumerate(rlen)]
    masks = [[1] * k for k in rlen]
    lps = [torch.randn(k, generator=g).tolist() for k in rlen]
    go = {"prompt_token_ids": prompts, "response_ids": resps, "rewards": rewards, "loss_masks": masks,
          "rollout_logprobs": lps}
    batch = tu.convert_to_training_input(go, [str(i // 8) for i in range(N)], 7, dp_size=5, device=dev)
    ref = cpu_ref.pack(prompts, resps, rewards, masks, lps, 7, pad=tu.pad_size_for(N, 5))
    for k, v in zip(("sequences", "attention_mask", "response_mask", "rewards", "loss_mask", "rollout_logprobs"), ref):
        assert torch.equal(batch[k].cpu(), torch.from_numpy(v)), k
