"""GRPOTrainer with the HIP optimizer path (comm.ShardedModuleOptimizer: flat fp32 master,
bucket reduce-scatters fired from the backward hooks, one HIP clip + AdamW pass writing the
engine's bf16 weights, fp32 + bf16 all-gathers) against single-process torch AdamW + clip on the
rank-mean gradient (fsdp_strategy.py:155-191, worker.py:902-924): at every optimizer step of
the trainer the local gradient sum is read from the flat buffer, all-reduced and scaled by
1/(world * n_micro), clipped with torch.nn.utils.clip_grad_norm_ and applied by
torch.optim.AdamW to a reference copy of the parameters. Each rank trains on its own fixed
generator outputs. Checked at every optimizer step:

  * the trainer's parameters equal the reference's (1e-6) and its grad norm equals
    clip_grad_norm_'s (rel 1e-5),
  * all ranks hold identical parameters (after each train_on),
  * after the weight sync the engine's bf16 weights equal the learner's fp32 parameters cast
    to bf16, bit for bit.

World size 1 (plain python) or 2 ranks on ONE GPU over gloo (RCCL refuses two ranks on one
device; the 8-GPU RCCL run issues the same calls). Prints one JSON line from rank 0.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        scripts/rehearse_trainer_optim.py
"""

import asyncio
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from skyrl_amd.config import AlgorithmConfig  # noqa: E402
from skyrl_amd.inference_engines.engine import AMDInferenceEngine  # noqa: E402
from skyrl_amd.inference_engines.model import PagedDecoder  # noqa: E402
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig  # noqa: E402


def fixed_generation(step, rank, n_prompts=4, G=4, vocab=512):
    """A deterministic stand-in for the rollout: ragged responses, rewards, rollout logprobs."""
    g = torch.Generator().manual_seed(1000 * step + 17 * rank)
    prompts, resp, rew, lps = [], [], [], []
    for i in range(n_prompts):
        p = torch.randint(2, vocab, (int(torch.randint(3, 9, (1,), generator=g)),), generator=g).tolist()
        for _ in range(G):
            r = torch.randint(2, vocab, (int(torch.randint(1, 13, (1,), generator=g)),), generator=g).tolist()
            prompts.append(p)
            resp.append(r)
            rew.append(float(torch.rand(1, generator=g) < 0.5))
            lps.append((-2.0 + 0.1 * torch.randn(len(r), generator=g)).tolist())
    return {"prompt_token_ids": prompts, "response_ids": resp, "rewards": rew, "rollout_logprobs": lps,
            "loss_masks": [[1] * len(r) for r in resp], "stop_reasons": ["length"] * len(resp)}


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    # REHEARSE_BACKEND=nccl with SKYRL_FORCE_COLLECTIVES=1 under a one-rank torchrun: every
    # exchange of the trainer runs as a one-rank RCCL collective on the comm stream
    backend = os.environ.get("REHEARSE_BACKEND", "gloo")
    dist_on = world > 1 or os.environ.get("SKYRL_FORCE_COLLECTIVES", "0") == "1"
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    rank = dist.get_rank() if dist_on else 0
    group = dist.group.WORLD if dist_on else None
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)  # same initial policy on every rank
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(dev)
    ref_policy = copy.deepcopy(policy)
    em = PagedDecoder(cfg, dev, seed=None, max_model_len=256)
    em.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(em, num_blocks=64, max_num_seqs=8, seed=7)

    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=2, micro_train_batch_size_per_gpu=4,
                         micro_forward_batch_size_per_gpu=16, lr=3e-3, weight_decay=0.01, max_grad_norm=0.5,
                         optimizer="hip", algorithm=AlgorithmConfig(use_kl_loss=False, use_entropy_loss=True,
                                                                    entropy_loss_coef=0.01))
    # 2 prompts x 4 samples per mini-batch: 2 optimizer steps per train_on, 2 micro-batches each
    hip = GRPOTrainer(tcfg, policy, engine, None, pad_token_id=0, dp_group=group)
    opt = hip.optim
    ref = [p.detach().clone().requires_grad_(True) for _, p in opt.named]
    ref_opt = torch.optim.AdamW(ref, lr=tcfg.lr, betas=tuple(tcfg.betas), eps=1e-8, weight_decay=tcfg.weight_decay)
    checks = []
    orig_step = opt.step

    def checked_step(n_micro=1, lr=None):
        local = opt.reducer.grad[: opt.reducer.layout.numel].clone()  # this rank's gradient sum
        if dist_on:
            dist.all_reduce(local, op=dist.ReduceOp.SUM, group=group)
        mean = local / (world * n_micro)
        for (_, p), o, r in zip(opt.named, opt.offsets, ref):
            r.grad = mean[o:o + p.numel()].view_as(r).clone()
        ref_norm = float(torch.nn.utils.clip_grad_norm_(ref, tcfg.max_grad_norm))
        ref_opt.step()
        gn = orig_step(n_micro, lr)
        hip_norm = float(gn)
        diff = max(float((p.detach() - r.detach()).abs().max()) for (_, p), r in zip(opt.named, ref))
        checks.append({"param_max_diff": diff, "grad_norm": hip_norm, "grad_norm_ref": ref_norm,
                       "grad_norm_rel": abs(hip_norm - ref_norm) / max(ref_norm, 1e-12)})
        return gn

    opt.step = checked_step
    # REHEARSE_DELAY_GATHER=1 (one-rank RCCL): the comm stream sleeps before each in-flight
    # re-assembly of the master, and every read of the policy's weights by the trainer's passes
    # (base_model forward, the lm_head weight) checks on the reading stream that the weights it
    # sees are the optimizer's updated shard: a pass that did not wait for the gather reads the
    # previous step's weights (2 mini-batches per train_on)
    weight_reads = {"checked": 0, "stale": 0}
    if os.environ.get("REHEARSE_DELAY_GATHER") == "1" and opt.collective and world == 1:
        orig_gather = opt._gather_full

        def delayed_gather(sync):
            with torch.cuda.stream(opt.reducer.stream):
                torch.cuda._sleep(100_000_000)  # ~40 ms of spinning before the all-gather
            return orig_gather(sync)

        opt._gather_full = delayed_gather

        def check_weights(*_):
            n = opt.reducer.layout.numel  # one rank: the shard is the whole master in flat order
            weight_reads["checked"] += 1
            if not torch.equal(opt.full[:n], opt.opt.param[:n]):  # (syncs the reading stream only)
                weight_reads["stale"] += 1

        policy.base_model.register_forward_pre_hook(check_weights)
        orig_emb = policy.get_output_embeddings

        def checked_emb():
            check_weights()
            return orig_emb()

        policy.get_output_embeddings = checked_emb
    init = torch.cat([p.detach().reshape(-1) for p in policy.parameters()]).clone()
    out = []
    ok_all = True
    for step in range(3):
        gen = fixed_generation(step, rank)
        m = hip.train_on(copy.deepcopy(gen))
        a = torch.cat([p.detach().reshape(-1) for p in policy.parameters()])
        same = torch.tensor([1.0], device=dev)
        if world > 1:
            a0 = a.clone()
            dist.broadcast(a0, 0)
            same = torch.tensor([1.0 if torch.equal(a0, a) else 0.0], device=dev)
            dist.all_reduce(same, op=dist.ReduceOp.MIN)
        hip._sync_weights()  # engine <- the optimizer's bf16 copy (views, no cast)
        eng = dict(em.hf_named_tensors())
        pairs = [(eng[n], p) for n, p in policy.named_parameters() if n in eng]
        bit_exact = len(pairs) >= len(list(policy.parameters())) - 1 and all(
            torch.equal(e, p.detach().to(torch.bfloat16)) for e, p in pairs)
        rec = {"step": step, "moved_from_init": float((a - init).abs().max()), "optimizer_steps": checks[-2:],
               "ranks_identical": bool(same.item() == 1.0), "engine_bf16_bit_exact": bit_exact,
               "final_loss": m["final_loss"], "grad_norm": m["grad_norm"]}
        ok = (rec["moved_from_init"] > 1e-4 and rec["ranks_identical"] and bit_exact
              and all(c["param_max_diff"] < 1e-6 and c["grad_norm_rel"] < 1e-5 for c in checks[-2:]))
        ok_all = ok_all and ok
        out.append(rec)
    ok_all = ok_all and weight_reads["stale"] == 0
    if rank == 0:
        print(json.dumps({"world": world, "backend": dist.get_backend() if dist_on else None,
                          "collective_path": bool(opt.collective),
                          "reduce_scatters_from_backward": opt.launched_during_backward,
                          "weight_reads": weight_reads, "ok": ok_all, "steps": out}), flush=True)
    if dist_on:
        dist.destroy_process_group()
    if not ok_all:
        sys.exit(1)


if __name__ == "__main__":
    asyncio.set_event_loop(asyncio.new_event_loop())
    main()
