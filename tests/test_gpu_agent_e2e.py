"""§8(f)4 on the GPU: the multi-turn SkyRL-SQL agent loop driving the MI355X engine, inside the
GRPO trainer (config 5 shape, tiny model). Parity of the loop itself is pinned on CPU against
the reference generator (tests/test_agent_loop.py); here the properties are end to end:
  * stop strings end engine turns (vLLM semantics) and the env sees the text;
  * observation tokens are masked out of the loss and carry rollout logprob 0.0, generated
    tokens keep the engine's logprobs, which agree with the learner's recomputation;
  * rewards come from the SQL env (in {-1, 0, 1}), the trainer steps without error.
"""

import asyncio

import pytest
import torch

import agent_fixtures as af
from skyrl_amd.config import AlgorithmConfig, SamplingParams
from skyrl_amd.generators import GeneratorConfig, SkyRLGymGenerator
from skyrl_amd.inference_engines.engine import AMDInferenceEngine
from skyrl_amd.inference_engines.model import PagedDecoder
from skyrl_amd.trainer import GRPOTrainer, TrainerConfig

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_sql_agent_loop_through_engine_and_trainer(tmp_path):
    from transformers import AutoModelForCausalLM, Qwen2Config

    tok = af.make_tokenizer()
    root = af.make_sql_root(str(tmp_path))
    cfg = Qwen2Config(vocab_size=128, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=1024,
                      tie_word_embeddings=True, eos_token_id=tok.eos_token_id)
    torch.manual_seed(0)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    with torch.no_grad():  # make "</sql>" likely so that some turns end on the stop string
        for ch in "</sql>":
            policy.model.embed_tokens.weight[tok.convert_tokens_to_ids(ch)] += 0.5
    em = PagedDecoder(cfg, DEV, seed=None, max_model_len=1024)
    em.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(em, num_blocks=512, max_num_seqs=16, seed=1, tokenizer=tok)
    gcfg = GeneratorConfig(max_turns=3, max_input_length=600,
                           sampling_params=SamplingParams(max_generate_length=24, logprobs=0,
                                                          stop=["</sql>", "</solution>"]))
    generator = SkyRLGymGenerator(gcfg, {"text2sql": {"db_path": root}}, engine, tok)
    prompts, _, extras, _ = af.scenario(True)
    prompts, extras = prompts[:4], extras[:4]

    # the loop alone: masks and logprobs of observation tokens
    from skyrl_amd.generators.skyrl_gym_generator import get_vllm_sampling_params

    out = asyncio.run(generator.generate({"prompts": prompts, "env_classes": ["text2sql"] * 4, "env_extras": extras,
                                          "sampling_params": get_vllm_sampling_params(gcfg.sampling_params)}))
    turns_with_obs = 0
    for ids, mask, lps, rew in zip(out["response_ids"], out["loss_masks"], out["rollout_logprobs"], out["rewards"]):
        assert len(ids) == len(mask) == len(lps) == len(rew)
        obs = [i for i, m in enumerate(mask) if m == 0]
        if obs:
            turns_with_obs += 1
            assert "<observation>" in tok.decode([ids[i] for i in obs])
            assert all(lps[i] == 0.0 for i in obs)
        assert all(lp < 0 for lp, m in zip(lps, mask) if m == 1)
        assert sum(rew) in (-1.0, 0.0, 1.0)
    assert turns_with_obs >= 1

    ref = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    ref.load_state_dict(policy.state_dict())
    tcfg = TrainerConfig(n_samples_per_prompt=2, policy_mini_batch_size=4, micro_train_batch_size_per_gpu=8,
                         micro_forward_batch_size_per_gpu=8, lr=1e-4, algorithm=AlgorithmConfig(use_kl_loss=True))
    trainer = GRPOTrainer(tcfg, policy, engine, None, pad_token_id=tok.pad_token_id, ref=ref, generator=generator,
                          env_class="text2sql")
    for _ in range(2):
        m = trainer.step(prompts, extras)
        assert m["logprobs_diff_mean"] < 0.03
        assert torch.isfinite(torch.tensor(m["final_loss"]))
