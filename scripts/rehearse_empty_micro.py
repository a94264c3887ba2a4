"""A fused-pass micro-batch with no response token on ONE data-parallel rank (ADVICE r04,
VERDICT r05 item 5). GRPOTrainer._fused_policy_pass back-propagates a zero loss through the
same forward for such a micro-batch, so its backward still reaches every parameter and the
HIP optimizer's per-bucket reduce-scatters fire from the backward hooks in the same order on
every rank (the reference's micro-batch loop, workers/worker.py:731-900, runs the same
forward/backward whatever the mask). The valid generator output check rejects empty
responses, so the micro-batch is made empty after packing: its attention mask over the
response and its loss mask are zeroed on rank 1 only.

Checked: the zero-token micro-batch's loss is exactly 0; both ranks launch the same bucket
sequence during the last micro-batch's backward (the same count, the same bucket order); after
the optimizer step both ranks hold bit-identical weights; the step moved them.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        scripts/rehearse_empty_micro.py
2 ranks on ONE GPU over gloo (RCCL refuses two ranks on one device). Prints one JSON line.
"""

import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rehearse_trainer_optim import fixed_generation  # noqa: E402
from skyrl_amd import comm, ops, trainer_utils  # noqa: E402
from skyrl_amd.config import AlgorithmConfig  # noqa: E402
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    group = dist.group.WORLD
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=256,
                      tie_word_embeddings=True, eos_token_id=1)
    torch.manual_seed(0)  # the same initial policy on every rank
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(dev)
    G = 4
    tcfg = TrainerConfig(n_samples_per_prompt=G, policy_mini_batch_size=2, micro_train_batch_size_per_gpu=4,
                         micro_forward_batch_size_per_gpu=8, lr=3e-3, optimizer="hip",
                         algorithm=AlgorithmConfig(use_kl_loss=False, use_entropy_loss=True, entropy_loss_coef=0.01))
    # 256 KB gradient buckets (the trainer's default would hold this model in one): ~20 bucket
    # reduce-scatters, so their order is what the check compares
    comm.ShardedModuleOptimizer.__init__.__defaults__ = (None, 256 << 10)
    tr = GRPOTrainer(tcfg, policy, None, None, pad_token_id=0, dp_group=group)
    assert tr._fused_pass_ok() and len(tr.optim.reducer.layout.buckets) > 4
    gen = fixed_generation(0, rank, n_prompts=2, G=G)  # 8 rows: one mini-batch of 2 micro-batches
    uids = [str(i // G) for i in range(len(gen["response_ids"]))]
    gen, _ = trainer_utils.postprocess_generator_output(copy.deepcopy(gen), uids, G)
    data = trainer_utils.convert_to_training_input(gen, uids, 0, dp_size=1, device=dev)
    data["action_log_probs"] = tr._fwd_logprobs(policy, data)
    data = trainer_utils.compute_advantages_and_returns(data, tcfg.algorithm)
    R = data["response_mask"].shape[1]
    mb = tcfg.micro_train_batch_size_per_gpu
    if rank == 1:  # micro-batch 1 (rows 4..7) without a single response token
        data["attention_mask"][mb:, -R:] = 0
        data["loss_mask"][mb:] = 0
        if data.get("loss_mask_row_sum") is not None:
            data["loss_mask_row_sum"][mb:] = 0
    n = len(data["sequences"])
    launched = []
    orig_launch = tr.optim.reducer.launch

    def rec_launch(buckets=None):
        launched.append(list(buckets) if buckets is not None else None)
        return orig_launch(buckets)

    tr.optim.reducer.launch = rec_launch
    init = torch.cat([p.detach().reshape(-1) for p in policy.parameters()]).clone()
    step = ops.PolicyTrainStep(data["action_log_probs"], data["advantages"], data["loss_mask"], tr.loss_params, mb,
                               temperature=tcfg.temperature)
    losses = []
    policy.train()
    for k, i in enumerate(range(0, n, mb)):
        j = min(i + mb, n)
        loss = tr._fused_policy_pass(step, k, data, i, j, R)
        if j == n:
            launched.clear()
            tr.optim.arm()
        loss.backward()
        losses.append(float(loss.detach()) if loss.dim() == 0 else None)
    during_backward = tr.optim.launched_during_backward
    allm = step.fold()[1].cpu()
    ops.check_loss_metrics(allm)
    tr.optim.step(n // mb)
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in policy.parameters()])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    same = torch.tensor([1.0 if torch.equal(ref, flat) else 0.0], device=dev)
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    seqs = [None] * world
    dist.all_gather_object(seqs, {"launched": launched, "during_backward": during_backward,
                                  "empty_loss": losses[-1] if rank == 1 else None})
    res = {
        "world": world,
        "launch_sequences_equal": all(s["launched"] == seqs[0]["launched"] for s in seqs),
        "launched_during_backward": [s["during_backward"] for s in seqs],
        "empty_micro_loss": seqs[1]["empty_loss"],
        "weights_identical_across_ranks": bool(same.item() == 1.0),
        "moved_from_init": float((flat - init).abs().max()),
        "buckets": len(tr.optim.reducer.layout.buckets),
    }
    res["ok"] = (res["launch_sequences_equal"] and len(set(res["launched_during_backward"])) == 1
                 and res["launched_during_backward"][0] == res["buckets"] and res["empty_micro_loss"] == 0.0
                 and res["weights_identical_across_ranks"] and res["moved_from_init"] > 0)
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    if not res["ok"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
