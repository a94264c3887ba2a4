"""§8(f)4: text environments for the multi-turn agent loop (skyrl-gym surface: BaseTextEnv,
make/register) with the SkyRL-SQL and GSM8K rewards."""

from .base import BaseTextEnv, BaseTextEnvStepOutput, make, register  # noqa: F401
from . import gsm8k, sql  # noqa: F401  (registers "gsm8k" and "text2sql")
