"""Real-model GRPO step on one MI355X at the headline configuration (BASELINE configs[1]):
Qwen2.5-1.5B-shaped policy (random init: no checkpoint download), 64 prompts x G=8 = 512
trajectories, prompts uniform [16, 512] tokens, responses uniform [1, 1024] tokens (SURVEY
§8(d); ignore_eos with a per-trajectory max_tokens), colocated actor/ref, one optimizer step.

The learner is a HF transformers Qwen2 under autocast(bf16) with gradient checkpointing (the
reference's default); rollout is AMDInferenceEngine; every §8 kernel is the HIP path. Prints
one JSON line: samples/s and the per-phase seconds of each timed step.
"""

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from skyrl_amd.config import AlgorithmConfig  # noqa: E402
from skyrl_amd.inference_engines.engine import AMDInferenceEngine  # noqa: E402
from skyrl_amd.inference_engines.model import PagedDecoder  # noqa: E402
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig  # noqa: E402

DEV = torch.device("cuda:0")


def log(msg):
    print(f"[e2e {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--max-response", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=28)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--micro", type=int, default=16)
    ap.add_argument("--tunable", action="store_true", help="TunableOp GEMM search in the rollout engine")
    ap.add_argument("--no-packing", action="store_true", help="padded learner batches (no sample packing)")
    ap.add_argument("--no-grad-ckpt", action="store_true",
                    help="keep the activations instead of recomputing them (288 GB of HBM affords it)")
    args = ap.parse_args()
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(vocab_size=151936, hidden_size=1536, intermediate_size=8960, num_hidden_layers=args.layers,
                      num_attention_heads=12, num_key_value_heads=2, max_position_embeddings=32768,
                      rope_theta=1000000.0, rms_norm_eps=1e-6, tie_word_embeddings=True, eos_token_id=151645)
    torch.manual_seed(0)
    t0 = time.time()
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    if not args.no_grad_ckpt:  # the reference's default (ppo_base_config.yaml gradient_checkpointing: true)
        policy.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
    policy.config.use_cache = False
    ref = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    ref.load_state_dict(policy.state_dict())
    engine_model = PagedDecoder(cfg, DEV, seed=None, max_model_len=512 + args.max_response + 16)
    engine_model.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(engine_model, num_blocks=None, max_num_seqs=args.prompts * args.group,
                                kv_cache_fraction=0.15, seed=0,
                                tunable_gemm=os.path.join(os.environ.get("TMPDIR", "/tmp"), "skyrl_tunableop.csv")
                                if args.tunable else None)
    log(f"models ready in {time.time() - t0:.1f}s; kv blocks {engine.num_blocks}")
    tcfg = TrainerConfig(n_samples_per_prompt=args.group, policy_mini_batch_size=args.prompts,
                         micro_train_batch_size_per_gpu=args.micro, micro_forward_batch_size_per_gpu=args.micro,
                         lr=1e-6, sampling_params={"min_tokens": 1, "ignore_eos": True},
                         use_sample_packing=not args.no_packing,
                         algorithm=AlgorithmConfig(use_kl_loss=True))
    g = torch.Generator().manual_seed(1234)
    N = args.prompts * args.group
    resp_len = torch.randint(1, args.max_response + 1, (N,), generator=g).tolist()
    prompts = [torch.randint(0, cfg.vocab_size, (int(torch.randint(16, 513, (1,), generator=g)),),
                             generator=g).tolist() for _ in range(args.prompts)]

    trainer = GRPOTrainer(tcfg, policy, engine, lambda p, r, e: float(len(r) % 2), pad_token_id=0, ref=ref)

    async def generate(ps):  # per-trajectory max_tokens (SURVEY §8(d) response lengths)
        ids = [p for p in ps for _ in range(args.group)]
        sp = {"temperature": 1.0, "min_tokens": 1, "ignore_eos": True, "logprobs": 0}
        outs = await asyncio.gather(*[engine.generate({"prompt_token_ids": [p],
                                                       "sampling_params": dict(sp, max_tokens=m)})
                                      for p, m in zip(ids, resp_len)])
        rids = [o["response_ids"][0] for o in outs]
        return {"prompt_token_ids": ids, "response_ids": rids, "stop_reasons": [o["stop_reasons"][0] for o in outs],
                "rollout_logprobs": [o["response_logprobs"][0] for o in outs],
                "loss_masks": [[1] * len(r) for r in rids]}

    trainer._generate = generate
    mark = trainer._mark

    def logged_mark(phase):  # progress line per phase (a long silent phase looks hung to gpurun)
        mark(phase)
        log(f"  {phase}: {trainer.timings[phase]:.2f}s")

    trainer._mark = logged_mark
    steps = []
    for k in range(args.warmup + args.steps):
        t = time.perf_counter()
        m = trainer.step(prompts)
        dt = time.perf_counter() - t
        rec = {"seconds": round(dt, 3), "phases": {k2: round(v, 3) for k2, v in trainer.timings.items()},
               "final_loss": round(m["final_loss"], 6), "logprobs_diff_mean": round(m["logprobs_diff_mean"], 5),
               "engine": {k2: round(v, 4) for k2, v in engine.core.stats.items()}}
        engine.core.stats.clear()
        log(f"step {k}: {json.dumps(rec)}")
        if k >= args.warmup:
            steps.append(rec)
    sec = sum(s["seconds"] for s in steps) / len(steps)
    print(json.dumps({"metric": "trained samples/sec (rollout+update), real-model GRPO step", "value": round(N / sec, 3),
                      "unit": "samples/s", "seconds_per_step": round(sec, 3), "trajectories": N,
                      "config": {"model": "Qwen2.5-1.5B (random init)", "layers": args.layers, "prompts": args.prompts,
                                 "group": args.group, "prompt_len": "U[16,512]",
                                 "response_len": f"U[1,{args.max_response}]", "micro_batch": args.micro,
                                 "gradient_checkpointing": not args.no_grad_ckpt, "sample_packing": tcfg.use_sample_packing,
                                 "learner": "HF transformers fp32 master, autocast bf16"},
                      "generated_tokens": sum(resp_len), "steps": steps}), flush=True)


if __name__ == "__main__":
    main()
