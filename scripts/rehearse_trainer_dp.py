"""Data-parallel GRPOTrainer rehearsal: 2 ranks on ONE GPU over gloo (RCCL refuses two ranks on
one device; the 8-GPU RCCL run uses the same calls). Every rank runs its own engine and
learner on its own prompts; gradients are mean-reduced (comm.allreduce_grads) before the
clip/AdamW. The DP invariant checked: after every step all ranks hold bit-identical policy
weights, although their rollouts differ. Prints one JSON line from rank 0.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        scripts/rehearse_trainer_dp.py
"""

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


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)  # same initial policy on every rank
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(dev)
    em = PagedDecoder(cfg, dev, seed=None, max_model_len=256)
    em.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(em, num_blocks=256, max_num_seqs=32, seed=100 + rank)
    tcfg = TrainerConfig(n_samples_per_prompt=4, policy_mini_batch_size=4, micro_train_batch_size_per_gpu=8,
                         micro_forward_batch_size_per_gpu=16, lr=3e-3, weight_decay=0.0,
                         sampling_params={"max_tokens": 10, "min_tokens": 1, "ignore_eos": True},
                         algorithm=AlgorithmConfig(use_kl_loss=False))
    trainer = GRPOTrainer(tcfg, policy, engine, lambda p, r, e: sum(t < 64 for t in r) / len(r), pad_token_id=0,
                          dp_group=dist.group.WORLD)
    g = torch.Generator().manual_seed(10 + rank)  # different prompts per rank
    prompts = [torch.randint(2, 512, (6,), generator=g).tolist() for _ in range(4)]
    out = []
    for step in range(3):
        m = trainer.step(prompts)
        flat = torch.cat([p.detach().reshape(-1) for p in policy.parameters()])
        mine = flat.clone()
        dist.broadcast(flat, 0)
        same = bool(torch.equal(mine, flat))
        ok = torch.tensor([1.0 if same else 0.0], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        out.append({"step": step, "weights_identical_across_ranks": bool(ok.item() == 1.0),
                    "reward": round(m["avg_final_rewards"], 4), "logprobs_diff_mean": round(m["logprobs_diff_mean"], 5)})
    if rank == 0:
        print(json.dumps({"world": world, "steps": out}), flush=True)
    dist.destroy_process_group()
    if not all(o["weights_identical_across_ranks"] for o in out):
        sys.exit(1)


if __name__ == "__main__":
    main()
