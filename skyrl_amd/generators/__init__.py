"""§8(f)4: the multi-turn generator (SkyRLGymGenerator surface, token-in/token-out)."""

from .skyrl_gym_generator import GeneratorConfig, SkyRLGymGenerator, TrajectoryID  # noqa: F401
