"""Text-in/text-out environment base and registry.

Mirrors skyrl-gym's BaseTextEnv (skyrl_gym/envs/base_text_env.py:17-100: turns, max_turns,
tool groups, init/step/close/get_metrics) and skyrl_gym.make/register (envs/registration.py),
which SkyRLGymGenerator.agent_loop drives (generators/skyrl_gym_generator.py:226-228).
"""

from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple, TypedDict

ConversationType = List[Dict[str, str]]


class BaseTextEnvStepOutput(TypedDict, total=False):
    observations: ConversationType
    reward: float
    done: bool
    metadata: Dict[str, Any]
    postprocessed_action: Optional[str]


class BaseTextEnv:
    def __init__(self):
        self.turns = 0
        self.max_turns = 1

    def init(self, prompt: ConversationType) -> Tuple[ConversationType, Dict[str, Any]]:
        """The first prompt given to the model (and optional metadata)."""
        return prompt, {}

    def step(self, action: str) -> BaseTextEnvStepOutput:
        raise NotImplementedError

    def close(self) -> None:
        pass

    def get_metrics(self) -> Dict[str, Any]:
        return {}


_REGISTRY: Dict[str, Callable[..., BaseTextEnv]] = {}


def register(name: str, factory: Callable[..., BaseTextEnv]) -> None:
    if name in _REGISTRY:
        raise ValueError(f"environment {name!r} already registered")
    _REGISTRY[name] = factory


def make(name: str, env_config: Any = None, extras: Optional[Dict[str, Any]] = None) -> BaseTextEnv:
    if name not in _REGISTRY:
        raise ValueError(f"unknown environment {name!r}; registered: {sorted(_REGISTRY)}")
    return _REGISTRY[name](env_config=env_config, extras=dict(extras or {}))
