"""Model families: Llama-3 (8B/70B), Mixtral 8x7B (MoE), GPT-2 — one shard-aware decoder."""
from .shard import LocalDims, Shard, local_dims  # noqa: F401
from .transformer import LogicalParam, TransformerLM  # noqa: F401


class LlamaForCausalLM(TransformerLM):
    """Llama-3 family (GQA, RoPE theta 5e5, RMSNorm, SwiGLU)."""


class MixtralForCausalLM(TransformerLM):
    """Mixtral (Llama attention + top-2 of 8 SwiGLU experts, dense-dispatch MoE)."""


class GPT2LMHeadModel(TransformerLM):
    """GPT-2 (learned positions, LayerNorm, GELU MLP with biases, tied embeddings)."""


_ARCH = {"llama": LlamaForCausalLM, "mixtral": MixtralForCausalLM, "gpt2": GPT2LMHeadModel}


def build_model(cfg, shard=None, device="cpu", dtype=None, comm=None):
    import torch

    cls = _ARCH[cfg.arch]
    return cls(cfg, shard or Shard(), device=device, dtype=dtype or torch.bfloat16, comm=comm)
