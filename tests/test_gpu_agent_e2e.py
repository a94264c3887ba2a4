"""§8(f)4 on the GPU: the multi-turn SkyRL-SQL agent loop driving the MI355X engine, inside the
GRPO trainer (config 5 shape: 8-turn rollouts, tiny model). Parity of the loop itself is pinned on CPU against
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
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=2048,
                      tie_word_embeddings=True, eos_token_id=tok.eos_token_id)
    torch.manual_seed(0)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    with torch.no_grad():  # make "</sql>" likely so that some turns end on the stop string
        for ch in "</sql>":
            policy.model.embed_tokens.weight[tok.convert_tokens_to_ids(ch)] += 0.5
    em = PagedDecoder(cfg, DEV, seed=None, max_model_len=2048)
    em.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(em, num_blocks=512, max_num_seqs=16, seed=1, tokenizer=tok)
    gcfg = GeneratorConfig(max_turns=8, max_input_length=1600,
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
    n_obs_blocks = [sum(1 for a, b in zip([1] + m[:-1], m) if a == 1 and b == 0) for m in out["loss_masks"]]
    assert max(n_obs_blocks) >= 4  # multi-turn: up to 8 turns per trajectory

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


def test_step_wise_trajectories_through_engine_and_trainer(tmp_path):
    """Step-wise training (one sample per turn) end to end: the generator flattens turns with
    is_last_step / trajectory ids, and the trainer's advantages give every step of a trajectory
    its last step's GRPO advantage (trainer.py:777-808) -- checked against the oracle on the
    same batch -- before the policy update."""
    from transformers import AutoModelForCausalLM, Qwen2Config

    from oracle import cpu_ref
    from skyrl_amd import trainer_utils
    from skyrl_amd.generators import TrajectoryID
    from skyrl_amd.generators.skyrl_gym_generator import get_vllm_sampling_params

    tok = af.make_tokenizer()
    root = af.make_sql_root(str(tmp_path))
    cfg = Qwen2Config(vocab_size=128, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=2048,
                      tie_word_embeddings=True, eos_token_id=tok.eos_token_id)
    torch.manual_seed(1)
    policy = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).to(DEV)
    with torch.no_grad():
        for ch in "</sql>":
            policy.model.embed_tokens.weight[tok.convert_tokens_to_ids(ch)] += 0.5
    em = PagedDecoder(cfg, DEV, seed=None, max_model_len=2048)
    em.load_weights((n, p.detach().to(torch.bfloat16)) for n, p in policy.named_parameters())
    engine = AMDInferenceEngine(em, num_blocks=512, max_num_seqs=16, seed=3, tokenizer=tok)
    gcfg = GeneratorConfig(max_turns=4, max_input_length=1600, step_wise_trajectories=True,
                           sampling_params=SamplingParams(max_generate_length=24, logprobs=0,
                                                          stop=["</sql>", "</solution>"]))
    generator = SkyRLGymGenerator(gcfg, {"text2sql": {"db_path": root}}, engine, tok)
    prompts, _, extras, _ = af.scenario(True)
    prompts, extras = prompts[:4], extras[:4]
    G = 2
    gen = asyncio.run(generator.generate({
        "sampling_params": get_vllm_sampling_params(gcfg.sampling_params),
        "prompts": [p for p in prompts for _ in range(G)], "env_classes": ["text2sql"] * (G * 4),
        "env_extras": [dict(e) for e in extras for _ in range(G)],
        "trajectory_ids": [TrajectoryID(f"p{i}", j) for i in range(4) for j in range(G)]}))
    last = gen["is_last_step"]
    assert sum(last) == G * 4 and len(last) > G * 4  # some trajectories have several turns
    for ids, mask, rew in zip(gen["response_ids"], gen["loss_masks"], gen["rewards"]):
        assert len(ids) == len(mask) == len(rew)
    # the trainer's advantage path vs the oracle on the same packed batch
    uids = [t.instance_id for t in gen["trajectory_ids"]]
    g2, _ = trainer_utils.postprocess_generator_output(dict(gen), uids, G, step_wise=True)
    data = trainer_utils.convert_to_training_input(g2, uids, tok.pad_token_id, device=DEV, step_wise=True)
    data = trainer_utils.compute_advantages_and_returns(data, AlgorithmConfig())
    rew, rmask = data["rewards"].cpu(), data["response_mask"].cpu()
    ls = data["is_last_step"].cpu().bool()
    exp_last = cpu_ref.grpo_advantage(rew[ls], rmask[ls], [u for u, f in zip(uids, ls.tolist()) if f])
    traj = torch.cat([torch.zeros(1, dtype=torch.int64), ls[:-1].long()]).cumsum(0)
    torch.testing.assert_close(data["advantages"].cpu(), exp_last[traj], atol=1e-5, rtol=1e-5)
    # and one trainer step on step-wise samples
    ref = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).to(DEV).eval()
    ref.load_state_dict(policy.state_dict())
    tcfg = TrainerConfig(n_samples_per_prompt=G, policy_mini_batch_size=4, micro_train_batch_size_per_gpu=8,
                         micro_forward_batch_size_per_gpu=8, lr=1e-4, algorithm=AlgorithmConfig(use_kl_loss=True))
    trainer = GRPOTrainer(tcfg, policy, engine, None, pad_token_id=tok.pad_token_id, ref=ref, generator=generator,
                          env_class="text2sql")
    m = trainer.step(prompts, extras)
    assert torch.isfinite(torch.tensor(m["final_loss"]))
