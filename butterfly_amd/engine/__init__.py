"""Inference engine: paged KV cache, continuous batching, sampling, hipGraph decode."""
from .batch import ForwardBatch  # noqa: F401
from .sampler import Sampler, SamplingParams  # noqa: F401
