"""butterfly_amd — MI355X-native distributed transformer inference.

Capabilities of TensorHusker/Butterfly (partition transformer layers / heads across devices,
minimise communication, distributed inference engine, scheduling, API, monitoring) built
MI355X-first: hand-written HIP/CDNA4 kernels on MFMA, RCCL over xGMI, hipGraph decode.

Public API:
    ModelConfig, EngineConfig, ParallelConfig     configuration
    partition(...) -> PartitionPlan               the partitioning API
    LLM(...).generate(prompts, SamplingParams)    inference
    ckpt.save / ckpt.load_into / ckpt.reshard     checkpoint format
"""
__version__ = "0.1.0"

from .config import EngineConfig, ModelConfig, ParallelConfig  # noqa: F401,E402
from .engine.sampler import SamplingParams  # noqa: F401,E402
from .partition import Hardware, PartitionPlan, partition  # noqa: F401,E402


def __getattr__(name):  # lazy: importing the engine pulls in the kernels / runtime
    if name in ("LLM", "RequestOutput"):
        from . import api

        return getattr(api, name)
    raise AttributeError(name)
