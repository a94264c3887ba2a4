"""Golden vectors for the multi-turn agent loop (§8(f)4) from the REAL reference generator.

Runs skyrl_train.generators.skyrl_gym_generator.SkyRLGymGenerator (imported read-only from
/root/reference behind the gen_golden.py shim; bytecode writing off) with skyrl_gym's own SQL
and GSM8K environments on the scripted scenario of tests/agent_fixtures.py, for
use_conversation_multi_turn in {True, False} and with/without zero_reward_on_non_stop +
apply_overlong_filtering. Writes tests/golden/agent_loop.json: the GeneratorOutput fields and
every prompt the engine was sent. Build container only.

    PYTHONDONTWRITEBYTECODE=1 python -B tools/gen_golden_agent.py
"""

import asyncio
import json
import os
import sys

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import agent_fixtures as af  # noqa: E402
from gen_golden import install_shim  # noqa: E402

DB_ROOT = "/tmp/skyrl_agent_golden_db"
MAX_INPUT = 600
CASES = [(mt, flags) for mt in (True, False) for flags in (False, True)]


def main():
    install_shim()
    from skyrl_train.config.config import GeneratorConfig, SamplingParams, SkyRLGymConfig, Text2SQLEnvConfig
    from skyrl_train.generators.base import TrajectoryID
    from skyrl_train.generators.skyrl_gym_generator import SkyRLGymGenerator

    af.make_sql_root(DB_ROOT)
    out = {"db_root": DB_ROOT, "max_input_length": MAX_INPUT, "cases": []}
    for multi_turn, flags in CASES:
        tok = af.make_tokenizer()
        cfg = GeneratorConfig(max_turns=3, max_input_length=MAX_INPUT, use_conversation_multi_turn=multi_turn,
                              zero_reward_on_non_stop=flags, apply_overlong_filtering=flags,
                              sampling_params=SamplingParams(max_generate_length=64, logprobs=0,
                                                             stop=["</sql>", "</solution>"]))
        env_cfg = SkyRLGymConfig(max_env_workers=0, text2sql=Text2SQLEnvConfig(db_path=DB_ROOT))
        client = af.ScriptedClient(tok)
        gen = SkyRLGymGenerator(cfg, env_cfg, client, tok, model_name="scripted")
        prompts, classes, extras, tids = af.scenario(multi_turn)
        res = asyncio.run(gen.generate({"prompts": prompts, "env_classes": classes, "env_extras": extras,
                                        "sampling_params": None,
                                        "trajectory_ids": [TrajectoryID(a, b) for a, b in tids]}, disable_tqdm=True))
        out["cases"].append({
            "multi_turn": multi_turn, "zero_reward_and_overlong": flags,
            "prompt_token_ids": res["prompt_token_ids"], "response_ids": res["response_ids"],
            "rewards": res["rewards"], "loss_masks": res["loss_masks"], "stop_reasons": res["stop_reasons"],
            "rollout_logprobs": res["rollout_logprobs"],
            "rollout_metrics": {k: float(v) for k, v in res["rollout_metrics"].items()},
            "engine_prompts": sorted(client.prompts),
        })
    path = os.path.join(ROOT, "tests", "golden", "agent_loop.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print(f"wrote {path}")

    # the other generator modes: re-tokenized chat history (custom chat templates), step-wise
    # trajectories, the batched single-call mode (tests/agent_fixtures.py MODE_CASES)
    from skyrl_train.config.config import ChatTemplateConfig

    modes = {"db_root": DB_ROOT, "max_input_length": MAX_INPUT, "cases": {}}
    for name, (over, with_lp, subset) in af.MODE_CASES.items():
        tok = af.make_tokenizer()
        over = dict(over)
        if "chat_template" in over:
            over["chat_template"] = ChatTemplateConfig(**over["chat_template"])
        cfg = GeneratorConfig(max_turns=3, max_input_length=MAX_INPUT,
                              sampling_params=SamplingParams(max_generate_length=64, logprobs=0 if with_lp else None,
                                                             stop=["</sql>", "</solution>"]), **over)
        env_cfg = SkyRLGymConfig(max_env_workers=0, text2sql=Text2SQLEnvConfig(db_path=DB_ROOT))
        client = af.ScriptedClient(tok, logprobs=with_lp)
        gen = SkyRLGymGenerator(cfg, env_cfg, client, tok, model_name="scripted")
        prompts, classes, extras, tids = af.scenario_subset(cfg.use_conversation_multi_turn, subset)
        res = asyncio.run(gen.generate({"prompts": prompts, "env_classes": classes, "env_extras": extras,
                                        "sampling_params": None,
                                        "trajectory_ids": [TrajectoryID(a, b) for a, b in tids]}, disable_tqdm=True))
        rec = {k: res.get(k) for k in ("prompt_token_ids", "response_ids", "rewards", "loss_masks", "stop_reasons",
                                      "rollout_logprobs", "is_last_step")}
        rec["trajectory_ids"] = ([t.to_string() for t in res["trajectory_ids"]]
                                 if res.get("trajectory_ids") is not None else None)
        rec["has_trajectory_keys"] = "trajectory_ids" in res
        rec["rollout_metrics"] = {k: float(v) for k, v in res["rollout_metrics"].items()}
        rec["engine_prompts"] = sorted(client.prompts)
        modes["cases"][name] = rec
    path = os.path.join(ROOT, "tests", "golden", "agent_loop_modes.json")
    with open(path, "w") as f:
        json.dump(modes, f)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
