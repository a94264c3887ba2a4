"""Separated placement on the GPU (config 4's learner / rollout split, at 1 + 1 ranks): rank 0
runs GRPOTrainer (HIP sharded optimizer) whose rollout client is a RemoteEngine, rank 1 hosts
the AMDInferenceEngine under serve_engine. Generation requests go over the gloo control
channel, weights by broadcast from the learner (ShardedBroadcastWeightSender ->
ShardedBroadcastWeightReceiver: init_weight_update_communicator / update_named_weights), as
broadcast_strategy.py:98-191 and vllm_worker.py:43-96 do with NCCL. Both ranks share ONE GPU
(RCCL refuses two ranks on one device; gloo carries the broadcast, the 8-GPU node uses RCCL).

Checked after every synchronous step: the remote engine's weights equal the learner's bf16
weights bit for bit, and its greedy tokens equal those of a colocated engine loaded with the
same weights. Then FullyAsyncGRPOTrainer drives the same remote engine: generation runs ahead
under the staleness budget and each step pauses (aborting what is in flight), updates the
weights and resumes (fully_async_trainer.py:415-419); the same weight check follows.
Prints one JSON line from rank 0.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/rehearse_separated.py
"""

import asyncio
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from skyrl_amd.config import AlgorithmConfig  # noqa: E402
from skyrl_amd.inference_engines.client import InferenceEngineClient  # noqa: E402
from skyrl_amd.inference_engines.engine import AMDInferenceEngine  # noqa: E402
from skyrl_amd.inference_engines.model import PagedDecoder  # noqa: E402
from skyrl_amd.inference_engines.remote import RemoteEngine, serve_engine  # noqa: E402


def build_policy(dev):
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)  # the same initial policy on both ranks
    return cfg, AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(dev)


def make_engine(cfg, named, dev, seed):
    em = PagedDecoder(cfg, dev, seed=None, max_model_len=256)
    em.load_weights(named)
    return AMDInferenceEngine(em, num_blocks=256, max_num_seqs=32, seed=seed)


def reward(p, r, e):
    return sum(t < 64 for t in r) / max(len(r), 1)


def main():
    from skyrl_amd.fully_async import FullyAsyncGRPOTrainer
    from skyrl_amd.trainer import GRPOTrainer, TrainerConfig

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    assert dist.get_world_size() == 2
    req, rep, wg = (dist.new_group([0, 1], backend="gloo") for _ in range(3))
    learners = dist.new_group([0], backend="gloo")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg, policy = build_policy(dev)
    init = [(n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters()]
    if rank == 1:  # the rollout rank
        del policy
        engine = make_engine(cfg, init, dev, seed=7)
        serve_engine(engine, 0, req, rep, wg)
        dist.destroy_process_group()
        return

    remote = RemoteEngine(1, req, rep, wg, weight_src_ranks=[0])
    client = InferenceEngineClient([remote], abort_grace_seconds=0.05)
    asyncio.run(client.init_weight_update_communicator(None))
    local = make_engine(cfg, init, dev, seed=7)  # colocated twin for the greedy check
    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=4, micro_train_batch_size_per_gpu=8,
                         micro_forward_batch_size_per_gpu=16, lr=3e-3, weight_decay=0.0,
                         sampling_params={"max_tokens": 12, "min_tokens": 1, "ignore_eos": True},
                         algorithm=AlgorithmConfig(use_kl_loss=False))
    trainer = GRPOTrainer(tcfg, policy, client, reward, pad_token_id=0, dp_group=learners)
    aborted = {"n": 0}
    gen0 = remote.generate

    async def counting_generate(batch):
        out = await gen0(batch)
        aborted["n"] += sum(r == "abort" for r in out["stop_reasons"])
        return out

    remote.generate = counting_generate
    g = torch.Generator().manual_seed(10)
    prompts = [torch.randint(2, 512, (6,), generator=g).tolist() for _ in range(4)]
    probe = [torch.randint(2, 512, (5,), generator=g).tolist() for _ in range(6)]

    def check(tag):
        remote_w = asyncio.run(remote.named_weights())
        mine = dict(trainer.optim.named_bf16())
        missing = [n for n in mine if n not in remote_w]
        bit_exact = all(torch.equal(remote_w[n].view(torch.int16), t.detach().cpu().view(torch.int16))
                        for n, t in mine.items() if n in remote_w)
        asyncio.run(local.update_named_weights({"names": list(mine), "tensors": list(mine.values())}))
        sp = {"max_tokens": 16, "temperature": 0.0, "ignore_eos": True}
        a = asyncio.run(remote.generate({"prompt_token_ids": probe, "sampling_params": sp}))
        b = asyncio.run(local.generate({"prompt_token_ids": probe, "sampling_params": sp}))
        return {"step": tag, "weights_bit_exact": bit_exact and len(missing) <= 1, "missing": missing,
                "greedy_equal_colocated": a["response_ids"] == b["response_ids"]}

    out = {"sync": [], "fully_async": None}
    for step in range(2):
        m = trainer.step(prompts)
        rec = check(f"sync{step}")
        rec.update(reward=round(m["avg_final_rewards"], 4), final_loss=m["final_loss"])
        out["sync"].append(rec)

    def prompt_iter():
        h = torch.Generator().manual_seed(99)
        while True:
            yield torch.randint(2, 512, (6,), generator=h).tolist(), None

    tcfg.sampling_params = {"max_tokens": 48, "min_tokens": 1, "ignore_eos": True}
    fa = FullyAsyncGRPOTrainer(trainer, client, mini_batch_groups=2, max_staleness_steps=2, num_generation_workers=4)
    hist = asyncio.run(fa.train(prompt_iter(), num_steps=3))
    rec = check("fully_async")
    rec.update(steps=len(hist), staleness_max=max(h["async/staleness_max"] for h in hist),
               aborted_then_retried=aborted["n"],
               final_loss=[h.get("final_loss") for h in hist], keys=sorted(hist[-1]),
               finite=all(torch.isfinite(torch.tensor(float(v))).item() for h in hist for v in h.values()
                          if isinstance(v, (int, float))))
    out["fully_async"] = rec
    asyncio.run(client.teardown())
    ok = all(r["weights_bit_exact"] and r["greedy_equal_colocated"] for r in out["sync"] + [rec]) and rec["finite"] \
        and rec["steps"] == 3
    out["ok"] = bool(ok)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    try:
        main()
    except BaseException:
        import traceback

        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "ok": False, "error": traceback.format_exc()}),
              flush=True)
        raise
