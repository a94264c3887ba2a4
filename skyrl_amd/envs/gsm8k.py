"""Single-turn GSM8K environment: reward 1 when the strict `#### <number>` answer equals the
ground truth (skyrl_gym/envs/gsm8k/env.py, utils.py:17-63; method "strict", format score 0)."""

from __future__ import annotations

import re
from typing import Any, Dict, Optional

from .base import BaseTextEnv, BaseTextEnvStepOutput, register

_ANSWER = re.compile(r"#### (\-?[0-9\.\,]+)")


def extract_solution(text: str) -> Optional[str]:
    m = _ANSWER.search(text)
    if m is None:
        return None
    return m.group(1).replace(",", "").replace("$", "")


def compute_score(text: str, ground_truth: str, format_score: float = 0.0, score: float = 1.0) -> float:
    ans = extract_solution(text)
    if ans is None:
        return 0
    return score if ans == ground_truth else format_score


class GSM8kEnv(BaseTextEnv):
    def __init__(self, env_config: Any = None, extras: Dict[str, Any] = None):
        super().__init__()
        extras = extras or {}
        if "ground_truth" not in extras.get("reward_spec", {}):
            raise ValueError("gsm8k needs extras['reward_spec']['ground_truth']")
        self.ground_truth = extras["reward_spec"]["ground_truth"]

    def step(self, action: str) -> BaseTextEnvStepOutput:
        return BaseTextEnvStepOutput(observations=[], reward=compute_score(action, self.ground_truth), done=True,
                                     metadata={})


register("gsm8k", GSM8kEnv)
