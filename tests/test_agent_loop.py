"""§8(f)4 multi-turn agent loop vs the REAL reference generator (CPU).

tests/golden/agent_loop.json was written by tools/gen_golden_agent.py, which ran the
reference SkyRLGymGenerator with skyrl_gym's SQL and GSM8K environments on the scripted
scenario of tests/agent_fixtures.py. Here the same scenario runs through skyrl_amd's
generator and environments; every GeneratorOutput field must be identical (token ids, loss
masks, per-token rewards, stop reasons, rollout logprobs), as must every prompt the engine saw.
"""

import asyncio
import json
import os

import pytest

import agent_fixtures as af
from skyrl_amd.config import SamplingParams
from skyrl_amd.envs import gsm8k, make
from skyrl_amd.envs.sql import compute_score_single, verify_format_and_extract
from skyrl_amd.generators import GeneratorConfig, SkyRLGymGenerator, TrajectoryID

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "agent_loop.json")


def load():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("case", range(4))
def test_agent_loop_matches_reference(case):
    g = load()
    exp = g["cases"][case]
    af.make_sql_root(g["db_root"])
    tok = af.make_tokenizer()
    cfg = GeneratorConfig(max_turns=3, max_input_length=g["max_input_length"],
                          use_conversation_multi_turn=exp["multi_turn"],
                          zero_reward_on_non_stop=exp["zero_reward_and_overlong"],
                          apply_overlong_filtering=exp["zero_reward_and_overlong"],
                          sampling_params=SamplingParams(max_generate_length=64, logprobs=0,
                                                         stop=["</sql>", "</solution>"]))
    client = af.ScriptedClient(tok)
    gen = SkyRLGymGenerator(cfg, {"text2sql": {"db_path": g["db_root"]}}, client, tok)
    prompts, classes, extras, tids = af.scenario(exp["multi_turn"])
    out = asyncio.run(gen.generate({"prompts": prompts, "env_classes": classes, "env_extras": extras,
                                    "sampling_params": None,
                                    "trajectory_ids": [TrajectoryID(a, b) for a, b in tids]}))
    for key in ("prompt_token_ids", "response_ids", "rewards", "loss_masks", "stop_reasons", "rollout_logprobs"):
        assert out[key] == exp[key], key
    assert sorted(client.prompts) == [(s, p) for s, p in exp["engine_prompts"]]
    for k, v in exp["rollout_metrics"].items():
        assert out["rollout_metrics"][k] == pytest.approx(v, abs=1e-9), k


def test_sql_reward_format_rules(tmp_path):
    root = af.make_sql_root(str(tmp_path))
    db = os.path.join(root, "spider", "database", "people", "people.sqlite")
    gold = "SELECT age FROM person WHERE name = 'bob'"
    ok = "<think>x</think><solution>SELECT age FROM person WHERE id = 2</solution>"
    assert compute_score_single(ok, gold, db) == 1.0
    assert compute_score_single(ok.replace("id = 2", "id = 1"), gold, db) == 0.0
    assert compute_score_single("<solution>SELECT 27</solution>", gold, db) == -1.0  # no <think>
    assert compute_score_single(ok + "<solution>x</solution>", gold, db) == -1.0  # two solutions
    assert compute_score_single("<think>a</think><solution><sql>x</sql></solution>", gold, db) == -1.0
    # every </observation> must be followed by a <think>
    bad = "<think>a</think><observation>r</observation> oops <solution>SELECT 27</solution>"
    assert not verify_format_and_extract(bad)[0]
    assert compute_score_single("<think>a</think><solution>NOT SQL</solution>", gold, db) == 0.0


def test_gsm8k_strict_extraction():
    assert gsm8k.extract_solution("so #### 1,234") == "1234"
    assert gsm8k.compute_score("#### 42", "42") == 1.0
    assert gsm8k.compute_score("42", "42") == 0
    env = make("gsm8k", extras={"reward_spec": {"ground_truth": "7"}})
    out = env.step("#### 7")
    assert out["done"] and out["reward"] == 1.0 and out["observations"] == []


def test_sql_env_turns_and_validation(tmp_path):
    root = af.make_sql_root(str(tmp_path))
    env = make("text2sql", env_config={"db_path": root},
               extras={"db_id": "people", "data": "spider", "max_turns": 2,
                       "reward_spec": {"ground_truth": "SELECT 1"}})
    o = env.step("<think>q</think><sql>SELECT name FROM person WHERE id = 3</sql>")
    assert not o["done"] and "carol" in o["observations"][0]["content"]
    assert "1 turns left" in o["observations"][0]["content"]
    with pytest.raises(AssertionError):
        env.step("<sql>SELECT 1</sql> trailing text")
    with pytest.raises(FileNotFoundError):
        make("text2sql", env_config={"db_path": root},
             extras={"db_id": "missing", "data": "spider", "reward_spec": {"ground_truth": "x"}})


MODES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "agent_loop_modes.json")


@pytest.mark.parametrize("name", sorted(af.MODE_CASES))
def test_generator_modes_match_reference(name):
    """Re-tokenized chat history (custom chat templates, incl. the single-assistant-message chat
    with a custom template), step-wise trajectories and the batched single-call mode against the
    reference generator's outputs on the same scripted scenario (tests/golden/agent_loop_modes.json)."""
    with open(MODES) as f:
        g = json.load(f)
    exp = g["cases"][name]
    over, with_lp, subset = af.MODE_CASES[name]
    af.make_sql_root(g["db_root"])
    tok = af.make_tokenizer()
    cfg = GeneratorConfig(max_turns=3, max_input_length=g["max_input_length"],
                          sampling_params=SamplingParams(max_generate_length=64, logprobs=0 if with_lp else None,
                                                         stop=["</sql>", "</solution>"]), **over)
    client = af.ScriptedClient(tok, logprobs=with_lp)
    gen = SkyRLGymGenerator(cfg, {"text2sql": {"db_path": g["db_root"]}}, client, tok)
    prompts, classes, extras, tids = af.scenario_subset(cfg.use_conversation_multi_turn, subset)
    out = asyncio.run(gen.generate({"prompts": prompts, "env_classes": classes, "env_extras": extras,
                                    "sampling_params": None,
                                    "trajectory_ids": [TrajectoryID(a, b) for a, b in tids]}))
    for key in ("prompt_token_ids", "response_ids", "rewards", "loss_masks", "stop_reasons", "rollout_logprobs",
                "is_last_step"):
        assert out.get(key) == exp[key], key
    assert ("trajectory_ids" in out) == exp["has_trajectory_keys"]
    got_tids = [t.to_string() for t in out["trajectory_ids"]] if out.get("trajectory_ids") is not None else None
    assert got_tids == exp["trajectory_ids"]
    assert sorted(client.prompts) == [tuple(x) for x in exp["engine_prompts"]]
    for k, v in exp["rollout_metrics"].items():
        assert out["rollout_metrics"][k] == pytest.approx(v, abs=1e-9), k


def test_generator_mode_validation():
    tok = af.make_tokenizer()
    sp = SamplingParams(max_generate_length=8)
    with pytest.raises(ValueError, match="batched"):
        SkyRLGymGenerator(GeneratorConfig(step_wise_trajectories=True, batched=True, sampling_params=sp), {}, None, tok)
    with pytest.raises(ValueError, match="custom chat template"):
        SkyRLGymGenerator(GeneratorConfig(step_wise_trajectories=True, sampling_params=sp,
                                          chat_template={"source": "name", "name_or_path": "qwen3_with_thinking"}),
                          {}, None, tok)
    with pytest.raises(ValueError, match="use_conversation_multi_turn"):
        SkyRLGymGenerator(GeneratorConfig(step_wise_trajectories=True, use_conversation_multi_turn=False,
                                          sampling_params=sp), {}, None, tok)
    with pytest.raises(ValueError, match="not found"):
        SkyRLGymGenerator(GeneratorConfig(chat_template={"source": "name", "name_or_path": "nope"},
                                          sampling_params=sp), {}, None, tok)
