"""advantage_batch_normalize on the HIP kernels (skyrl_adv_norm_stats / _apply) against the
reference's normalize_advantages_dict (utils/ppo_utils.py:127-145, applied at trainer.py:275-276
and fully_async_trainer.py:514-515):

  * the reference-generated fixtures (tests/golden/advnorm.npz, tools/gen_golden.py) at 1e-6;
  * the oracle (oracle/cpu_ref.normalize_advantages) on the bench shape 512 x 1024 (int64 mask)
    and on ragged / unaligned / bool-mask inputs at 1e-6;
  * data parallel: 2 ranks on one GPU over gloo, each holding half of the rows of one batch,
    one all-reduce of the 5 fp64 sums: the concatenation equals the single-rank result (1e-6);
  * the trainer: GRPOTrainer.train_on with advantage_batch_normalize normalizes the advantages
    after compute_advantages_and_returns (so the plan-GRPO path is off) and trains on them.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import cpu_ref
from skyrl_amd import ops, ppo_utils

pytestmark = pytest.mark.gpu
TOL = dict(atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("case", ["grpo", "dense", "const"])
def test_golden(golden, dev, case):
    d = golden("advnorm")
    out = ops.normalize_advantages(d[f"{case}_in"].to(dev), d[f"{case}_mask"].to(dev))
    torch.testing.assert_close(out.cpu(), d[f"{case}_out"], **TOL)


def test_dict_form_keeps_returns(golden, dev):
    d = golden("advnorm")
    adv = d["grpo_in"].to(dev)
    data = {"advantages": adv, "returns": adv, "response_mask": d["grpo_mask"].to(dev)}
    ppo_utils.normalize_advantages_dict(data)
    torch.testing.assert_close(data["advantages"].cpu(), d["grpo_out"], **TOL)
    assert data["returns"] is adv and torch.equal(adv.cpu(), d["grpo_in"])  # a new tensor, as the reference


@pytest.mark.parametrize("shape,mdt,offset", [((512, 1024), torch.int64, 0), ((33, 77), torch.float32, 1),
                                              ((7, 1000), torch.bool, 0), ((1, 3), torch.int32, 0),
                                              ((300, 129), torch.uint8, 3)])
def test_oracle(dev, shape, mdt, offset):
    g = torch.Generator().manual_seed(sum(shape))
    n = shape[0] * shape[1]
    base = torch.randn(n + offset, generator=g) * 1.3 + 0.4
    a = base[offset:].view(shape)  # offset > 0: an unaligned view (the scalar path)
    m = (torch.rand(shape, generator=g) < 0.7).to(mdt)
    exp = cpu_ref.normalize_advantages(a, m.float())
    out = ops.normalize_advantages(base.to(dev)[offset:].view(shape), m.to(dev))
    torch.testing.assert_close(out.cpu(), exp, atol=2e-6, rtol=2e-6)


def test_empty_mask_is_nan_like_the_reference(dev):
    a = torch.randn(4, 8)
    m = torch.zeros(4, 8)
    exp = cpu_ref.normalize_advantages(a, m)  # 0 / 0 -> nan
    out = ops.normalize_advantages(a.to(dev), m.to(dev)).cpu()
    assert torch.isnan(exp).all() and torch.isnan(out).all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_case(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        g = torch.Generator().manual_seed(7)
        a = torch.randn(64, 200, generator=g) * 0.5 + 1.0
        m = (torch.rand(64, 200, generator=g) < 0.6).to(torch.int64)
        rows = 64 // world
        mine = ops.normalize_advantages(a[rank * rows:(rank + 1) * rows].to(dev), m[rank * rows:(rank + 1) * rows].to(dev),
                                        group=dist.group.WORLD)
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        if rank == 0:
            whole = ops.normalize_advantages(a.to(dev), m.to(dev))
            q.put((float((torch.cat(parts) - whole).abs().max()),
                   float((torch.cat(parts).cpu() - cpu_ref.normalize_advantages(a, m.float())).abs().max())))
    finally:
        dist.destroy_process_group()


def test_data_parallel_two_ranks_equal_single_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_dp_case, args=(2, _free_port(), q), nprocs=2, join=True)
    d_single, d_oracle = q.get(timeout=5)
    assert d_single < 1e-6 and d_oracle < 2e-6, (d_single, d_oracle)


def test_trainer_applies_it_after_the_advantages(dev, monkeypatch):
    """GRPOTrainer.train_on with advantage_batch_normalize: the plan-GRPO path is off, the
    advantages the policy step trains on are normalize_advantages_dict's output of the GRPO
    advantages (checked against the oracle on the same input)."""
    import copy

    from transformers import AutoModelForCausalLM, Qwen2Config

    from skyrl_amd import trainer as trainer_mod
    from skyrl_amd.config import AlgorithmConfig
    from skyrl_amd.trainer import GRPOTrainer, TrainerConfig

    cfg = Qwen2Config(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=1,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=128,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(dev)
    g = torch.Generator().manual_seed(3)
    gen = {"prompt_token_ids": [], "response_ids": [], "rewards": [], "rollout_logprobs": [], "loss_masks": [],
           "stop_reasons": []}
    for i in range(4):
        p = torch.randint(2, 512, (5,), generator=g).tolist()
        for _ in range(4):
            r = torch.randint(2, 512, (int(torch.randint(1, 9, (1,), generator=g)),), generator=g).tolist()
            gen["prompt_token_ids"].append(p)
            gen["response_ids"].append(r)
            gen["rewards"].append(float(torch.rand(1, generator=g) < 0.5))
            gen["rollout_logprobs"].append([-2.0] * len(r))
            gen["loss_masks"].append([1] * len(r))
            gen["stop_reasons"].append("length")
    seen = {}
    orig = ppo_utils.normalize_advantages_dict

    def spy(data, group=None):
        seen["in"] = data["advantages"].clone()
        seen["mask"] = data["response_mask"].clone()
        out = orig(data, group=group)
        seen["out"] = out["advantages"].clone()
        return out

    monkeypatch.setattr(trainer_mod.ppo_utils, "normalize_advantages_dict", spy)
    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=4, micro_train_batch_size_per_gpu=8,
                         micro_forward_batch_size_per_gpu=16, lr=1e-3,
                         algorithm=AlgorithmConfig(use_kl_loss=False, advantage_batch_normalize=True))
    tr = GRPOTrainer(tcfg, policy, None, None, pad_token_id=0)
    m = tr.train_on(copy.deepcopy(gen))
    assert "in" in seen and all(torch.isfinite(torch.tensor(v)) for v in m.values())
    exp = cpu_ref.normalize_advantages(seen["in"].cpu(), seen["mask"].cpu().float())
    torch.testing.assert_close(seen["out"].cpu(), exp, atol=2e-6, rtol=2e-6)
    assert abs(float(seen["out"].mean())) < 1e-5  # the unmasked mean is removed
