"""Debug: GPT-2 rollout logprobs (HFGenerateEngine) vs learner recomputation."""
import asyncio
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from transformers import AutoModelForCausalLM, GPT2Config  # noqa: E402

from skyrl_amd.inference_engines.hf_engine import HFGenerateEngine  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
cfg = GPT2Config()
policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(dev)
rollout = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(dev)
rollout.load_state_dict(policy.state_dict())
eng = HFGenerateEngine(rollout, pad_token_id=0, seed=5)
g = torch.Generator().manual_seed(1)
prompts = [torch.randint(1, 50256, (int(torch.randint(8, 33, (1,), generator=g)),), generator=g).tolist()
           for _ in range(4)]
out = asyncio.run(eng.generate({"prompt_token_ids": prompts, "sampling_params": {"max_tokens": 8, "logprobs": 0}}))
for i, (p, r, lp) in enumerate(zip(prompts, out["response_ids"], out["response_logprobs"])):
    s = torch.tensor(p + r, device=dev)[None]
    with torch.no_grad():
        lb = torch.log_softmax(rollout(s).logits.float(), -1)[0]
        l32 = torch.log_softmax(policy(s).logits.float(), -1)[0]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lac = torch.log_softmax(policy(s).logits.float(), -1)[0]
    idx = torch.arange(len(r), device=dev) + len(p) - 1
    rt = torch.tensor(r, device=dev)
    eng_lp = torch.tensor(lp, device=dev)
    print(i, "eng-vs-bf16full", (eng_lp - lb[idx, rt]).abs().max().item(),
          "bf16-vs-fp32", (lb[idx, rt] - l32[idx, rt]).abs().max().item(),
          "ac-vs-fp32", (lac[idx, rt] - l32[idx, rt]).abs().max().item(), "lp", eng_lp[:3].tolist(),
          "fp32", l32[idx, rt][:3].tolist())
