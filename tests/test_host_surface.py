"""a9–a11 host surface on CPU: TensorBatch container + wire format, pad_batch, data order,
mini-batch/DP slicing, metric reductions, generator-output post-processing.

Known answers are the reference's own test expectations (tests/cpu/test_train_batch.py,
tests/cpu/generators/test_skyrl_gym_generator.py:421-460, tests/cpu/test_trainer_utils.py:
660-690) and the committed pad_batch golden (tests/golden/pack.npz, written from the reference).
The data order is checked against torch's own DataLoader, which the reference's
build_dataloader wraps (utils/trainer_utils.py:661-699).
"""

import pickle

import numpy as np
import pytest
import torch

from skyrl_amd.training_batch import TensorBatch, TrainingInputBatch
from skyrl_amd import trainer_utils as tu


# --------------------------------------------------------------------------- a11 TensorBatch
def _batch(n=4):
    return TensorBatch({"sequences": torch.arange(n * 3).view(n, 3), "loss_mask": torch.ones(n, 3),
                        "logp": torch.randn(n, 3).to(torch.bfloat16), "values": None})


def test_tensor_batch_basics_and_validation():
    b = _batch()
    assert b.batch_size == 4 and len(b) == 4 and b.device == torch.device("cpu")
    with pytest.raises(ValueError, match="Batch size mismatch"):
        TensorBatch({"a": torch.zeros(3), "b": torch.zeros(2)})
    with pytest.raises(ValueError, match="must be a tensor"):
        TensorBatch({"a": [1, 2]})
    with pytest.raises(ValueError, match="Batch size mismatch in x"):
        b["x"] = torch.zeros(5)
    b["x"] = torch.zeros(4)
    assert "x" in b


def test_tensor_batch_reference_kats():
    d = TensorBatch(a=torch.tensor([1, 2, 3]), b=torch.tensor([4, 5, 6]))
    d.metadata = {"d": 1, "e": "test"}
    r = d.repeat(2)
    assert torch.equal(r["a"], torch.tensor([1, 2, 3, 1, 2, 3])) and r.metadata == {"d": 1, "e": "test"}
    ri = d.repeat_interleave(2)
    assert torch.equal(ri["b"], torch.tensor([4, 4, 5, 5, 6, 6]))
    assert torch.equal(d[:2]["a"], torch.tensor([1, 2]))
    assert torch.equal(d[1]["b"], torch.tensor([5]))


def test_tensor_batch_chunk_slice_cat_select():
    b = _batch(5)
    b.metadata = {"uids": list("abcde")}
    chunks = b.chunk(2)
    assert [len(c) for c in chunks] == [2, 2, 1]
    back = TensorBatch.cat(chunks)
    assert back == b
    s = b.select(["sequences"], ["uids"])
    assert list(s.keys()) == ["sequences"] and s.metadata == {"uids": list("abcde")}
    assert torch.equal(b.slice(1, 5, 2)["sequences"], b["sequences"][1:5:2])


def test_tensor_batch_wire_format_roundtrip():
    b = _batch()
    b.metadata = {"uids": ["0", "0", "1", "1"], "response_length": 3}
    raw = b.to_bytes()
    c = TensorBatch.from_bytes(raw)
    assert c == b
    assert c["logp"].dtype == torch.bfloat16 and c["values"] is None
    p = pickle.loads(pickle.dumps(b))
    assert p == b and p["logp"].dtype == torch.bfloat16
    with pytest.raises(ValueError, match="not a TensorBatch"):
        TensorBatch.from_bytes(b"garbage")


def test_tensor_batch_save_load(tmp_path):
    b = TrainingInputBatch({"rewards": torch.randn(3, 2)})
    b.metadata = {"k": 1}
    path = str(tmp_path / "b.bin")
    b.save(path)
    assert b.load(path) == b


# --------------------------------------------------------------------------- a9 pad_batch (golden)
def test_pad_batch_matches_reference_golden(golden):
    g = golden("pack")
    batch = TrainingInputBatch({k: g[k] for k in ("sequences", "attention_mask", "response_mask", "rewards",
                                                  "loss_mask", "rollout_logprobs")})
    n = batch.batch_size
    batch.metadata = {"uids": [str(i) for i in range(n)], "response_length": g["response_mask"].shape[1]}
    padded = tu.pad_batch(batch, dp_size=n + int(g["pad_size"]))
    assert padded.metadata["pad_size"] == int(g["pad_size"])
    for k in ("sequences", "attention_mask", "response_mask", "rewards", "loss_mask", "rollout_logprobs"):
        assert torch.equal(padded[k], g["p_" + k]), k
    assert padded.metadata["uids"] == [str(u) for u in g["p_uids"]]


def test_pad_batch_noop_and_is_last_step():
    b = TrainingInputBatch({"loss_mask": torch.ones(3, 2), "is_last_step": torch.tensor([True, False, True])})
    b.metadata = {"uids": ["a", "b", "c"]}
    assert tu.pad_batch(b, 3) is b and b.metadata["pad_size"] == 0
    p = tu.pad_batch(b, 4)
    assert p.batch_size == 4 and bool(p["is_last_step"][3]) and float(p["loss_mask"][3].sum()) == 0.0


def test_pad_batch_keeps_loss_mask_row_sums_consistent():
    """The pack kernel's loss_mask_row_sum (the fused loss's reduction scales) must follow the
    pads' zeroed loss mask: every row's sum equals its loss mask's sum after padding."""
    lm = torch.tensor([[1.0, 1.0, 0.0], [1.0, 0.0, 0.0], [1.0, 1.0, 1.0]])
    b = TrainingInputBatch({"loss_mask": lm, "loss_mask_row_sum": lm.sum(-1), "reward_row_sum": torch.ones(3)})
    b.metadata = {"uids": ["a", "b", "c"]}
    p = tu.pad_batch(b, 5)
    assert p.batch_size == 5
    assert torch.equal(p["loss_mask_row_sum"], p["loss_mask"].sum(-1))
    assert torch.equal(p["reward_row_sum"], torch.ones(5))  # rewards are cloned with their rows


def test_flatten_ragged():
    v, o = tu.flatten_ragged([[1, 2], [], [3]], np.int64)
    assert v.tolist() == [1, 2, 3] and o.tolist() == [0, 2, 2, 3]


# --------------------------------------------------------------------------- a10 order / slicing
def test_prompt_order_matches_torch_dataloader():
    n, bs, seed = 37, 8, 42
    g = torch.Generator()
    g.manual_seed(seed)
    dl = torch.utils.data.DataLoader(list(range(n)), batch_size=bs, shuffle=True, drop_last=True, generator=g,
                                     num_workers=0)
    order = tu.PromptOrder(n, bs, seed=seed)
    assert len(order) == len(dl)
    for _ in range(3):  # epochs
        assert order.epoch() == [b.tolist() for b in dl]


def test_remove_tail_and_slices():
    entries = list(range(10))
    assert tu.remove_tail_data(entries, lcm_dp_size=4, n_samples_per_prompt=2) == list(range(10))  # stride 2
    assert tu.remove_tail_data(entries, lcm_dp_size=8, n_samples_per_prompt=2) == list(range(8))
    assert tu.remove_tail_data(entries, lcm_dp_size=3, n_samples_per_prompt=1) == list(range(9))
    assert tu.remove_tail_data(entries, lcm_dp_size=8, n_samples_per_prompt=8) == entries
    assert tu.mini_batch_slices(10, 4) == [(0, 4), (4, 8)]
    assert tu.dp_slice(8, 16, 4, 2) == (12, 14)
    with pytest.raises(AssertionError, match="divisible"):
        tu.dp_slice(0, 6, 4, 0)


def test_reduce_metrics_and_batch_iterator():
    assert tu.reduce_metrics({"loss": [1.0, 3.0], "kl_max": [1, 5], "r_min": [2.0, -1.0]}) == \
        {"loss": 2.0, "kl_max": 5, "r_min": -1.0}
    b = TrainingInputBatch({"sequences": torch.zeros(5, 3), "response_mask": torch.ones(5, 2)})
    b.metadata = {"response_length": 2}
    it = tu.BatchIterator(b, 2)
    exps = list(it)
    assert len(it) == 3 and [e.sequences.shape[0] for e in exps] == [2, 2, 1]
    assert exps[0].num_actions == 2 and exps[0].action_mask is not None
    assert len(list(it)) == 3  # re-iterable, as the reference resets on StopIteration


# --------------------------------------------------------------------------- rewards / metrics
def test_get_metrics_reference_kats():
    go = {"rewards": [1.0, 2.0]}
    m = tu.get_metrics_from_generator_output(go, ["a", "b"])
    assert (m["avg_score"], m["pass_at_n"], m["mean_positive_reward"]) == (1.5, 1.0, 1.5)
    go["rewards"] = [[1.0, 0.0], [0.0, 1.0]]
    m = tu.get_metrics_from_generator_output(go, ["a", "b"])
    assert (m["avg_score"], m["pass_at_n"], m["mean_positive_reward"]) == (1.0, 0.5, 1.0)
    go["rewards"] = [-1.0, 2.0]
    m = tu.get_metrics_from_generator_output(go, ["a", "b"])
    assert (m["avg_score"], m["pass_at_n"], m["mean_positive_reward"]) == (0.5, 0.5, 1.0)
    go["rewards"] = [[1.0, -1.0], [-0.5, 0.5]]
    m = tu.get_metrics_from_generator_output(go, ["a", "b"])
    assert (m["avg_score"], m["pass_at_n"], m["mean_positive_reward"]) == (0.0, 0.5, 0.75)


def test_zero_variance_filter_reference_kats():
    assert tu.zero_variance_filter([1.0, 2.0, 3.0, 3.0, 5.0], ["uid1", "uid1", "uid2", "uid2", "uid3"]) == [0, 1, 4]
    assert tu.zero_variance_filter([1.0, 1.0, 2.0, 2.0], ["a", "a", "b", "b"]) == []
    assert tu.zero_variance_filter([1.0, 1.0, 1.0], ["x", "y", "z"]) == [0, 1, 2]


def test_postprocess_generator_output_last_token_reward_and_filter():
    go = {"response_ids": [[5, 6, 7], [8], [9, 9]], "rewards": [1.0, 1.0, 0.5],
          "loss_masks": [[1, 1, 1], [1], [1, 0]], "prompt_token_ids": [[1], [1], [2]]}
    out, metrics = tu.postprocess_generator_output(go, ["a", "a", "b"], 2, zero_variance_filter_enabled=True)
    assert out["rewards"] == [[0.0, 0.0, 1.0], [1.0], [0.0, 0.5]]
    assert out["loss_masks"] == [[0, 0, 0], [0], [1, 0]]  # group "a" has zero variance
    assert metrics["reward/avg_pass_at_2"] == 1.0
    tu.validate_generator_output(3, out)
    with pytest.raises(AssertionError, match="Mismatch"):
        tu.validate_generator_output(2, out)
