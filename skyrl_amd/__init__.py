"""skyrl_amd — MI355X-native (gfx950) hot path of the skyrl-train GRPO/PPO actor-learner loop.

Hand-written HIP kernels behind a C ABI (include/skyrl_hip.h, built into
skyrl_amd/lib/libskyrl_hip.so), driven from Python modules that keep the reference's plugin
surface: ppo_utils (registries, estimators, losses), torch_utils (logprobs/entropy),
preprocess (experience pack), sampler (rollout sampling), worker (loss assembly), comm
(RCCL gradient all-reduce / weight broadcast).
"""

__version__ = "0.1.0"


def native_library_path() -> str:
    from . import _ffi

    return _ffi.LIB_PATH


def require_native():
    """Load the HIP library (raises ImportError if it was not built)."""
    from . import _ffi

    return _ffi.load()
