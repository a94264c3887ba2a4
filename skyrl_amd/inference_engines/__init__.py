"""§8(f)2: the rollout decode loop around the HIP sampler — a paged-KV continuous-batching
engine behind the reference's InferenceEngineInterface (skyrl_train/inference_engines/)."""

from .base import InferenceEngineInput, InferenceEngineInterface, InferenceEngineOutput  # noqa: F401
from .engine import AMDInferenceEngine, BlockAllocator, EngineCore, RequestParams  # noqa: F401
