"""Configuration: model presets, parallel layout, engine settings, feature flags.

Precedence: explicit arguments / CLI > BFLY_* environment > YAML/JSON file >
preset. The reference only states "Use feature flags for incompatible changes during
transition" (/root/reference/CLAUDE.md:81); the flag registry lives in utils/flags.py.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Optional


@dataclass
class ModelConfig:
    name: str
    arch: str                       # "llama" | "gpt2" | "mixtral"
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    max_position: int = 8192
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    norm_eps: float = 1e-5
    norm: str = "rms"               # "rms" | "layer"
    act: str = "silu"               # "silu" (SwiGLU) | "gelu" (plain MLP)
    pos_emb: str = "rope"           # "rope" | "learned"
    bias: bool = False              # linear biases (GPT-2)
    tie_embeddings: bool = False
    num_experts: int = 0            # > 0: MoE FFN
    experts_per_token: int = 0
    init_std: float = 0.02

    # ---- derived quantities ------------------------------------------------------------
    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def padded_vocab(self, multiple: int = 256) -> int:
        return (self.vocab_size + multiple - 1) // multiple * multiple

    def layer_params(self) -> int:
        h, f = self.hidden_size, self.intermediate_size
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        mlp = (3 if self.act == "silu" else 2) * h * f
        if self.is_moe:
            mlp = mlp * self.num_experts + h * self.num_experts
        norms = 2 * h * (2 if self.norm == "layer" else 1)
        b = 0
        if self.bias:
            b = self.q_size + 2 * self.kv_size + h + f + h
        return attn + mlp + norms + b

    def param_count(self) -> int:
        emb = self.vocab_size * self.hidden_size
        head = 0 if self.tie_embeddings else emb
        pos = self.max_position * self.hidden_size if self.pos_emb == "learned" else 0
        final = self.hidden_size * (2 if self.norm == "layer" else 1)
        return emb + head + pos + final + self.num_layers * self.layer_params()

    def active_params_per_token(self) -> int:
        if not self.is_moe:
            return self.param_count()
        h, f = self.hidden_size, self.intermediate_size
        dense_mlp = 3 * h * f
        per_layer = self.layer_params() - dense_mlp * self.num_experts + dense_mlp * self.experts_per_token
        return self.param_count() - self.num_layers * (self.layer_params() - per_layer)

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    # ---- (de)serialisation -------------------------------------------------------------
    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def from_preset(cls, name: str, **overrides) -> "ModelConfig":
        if name not in PRESETS:
            raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
        d = dict(PRESETS[name])
        d.update(overrides)
        return cls(name=name, **d)

    @classmethod
    def from_hf(cls, hf: dict, name: str = "hf") -> "ModelConfig":
        """Map a HuggingFace config.json (Llama / Mistral / Mixtral / GPT-2) to ModelConfig."""
        mt = hf.get("model_type", "llama")
        if mt == "gpt2":
            h = hf["n_embd"]
            return cls(name=name, arch="gpt2", vocab_size=hf["vocab_size"], hidden_size=h,
                       intermediate_size=hf.get("n_inner") or 4 * h, num_layers=hf["n_layer"],
                       num_heads=hf["n_head"], num_kv_heads=hf["n_head"], head_dim=h // hf["n_head"],
                       max_position=hf["n_positions"], norm="layer", act="gelu", pos_emb="learned",
                       bias=True, tie_embeddings=True, norm_eps=hf.get("layer_norm_epsilon", 1e-5))
        h = hf["hidden_size"]
        nh = hf["num_attention_heads"]
        arch = "mixtral" if mt == "mixtral" else "llama"
        # rope: older configs carry rope_theta / rope_scaling at top level, newer ones a
        # "rope_parameters" dict; llama3-style frequency scaling is normalised to our keys
        rp = dict(hf.get("rope_parameters") or {})
        theta = rp.get("rope_theta", hf.get("rope_theta", 10000.0))
        scaling = hf.get("rope_scaling") or (rp if rp.get("rope_type", "default") != "default" else None)
        if scaling:
            kind = scaling.get("rope_type", scaling.get("type"))
            scaling = {"type": kind, **{k: v for k, v in scaling.items() if k not in ("rope_type", "type", "rope_theta")}}
        return cls(name=name, arch=arch, vocab_size=hf["vocab_size"], hidden_size=h,
                   intermediate_size=hf["intermediate_size"], num_layers=hf["num_hidden_layers"],
                   num_heads=nh, num_kv_heads=hf.get("num_key_value_heads", nh),
                   head_dim=hf.get("head_dim", h // nh),
                   max_position=hf.get("max_position_embeddings", 8192),
                   rope_theta=theta, rope_scaling=scaling,
                   norm_eps=hf.get("rms_norm_eps", 1e-5),
                   tie_embeddings=hf.get("tie_word_embeddings", False),
                   num_experts=hf.get("num_local_experts", 0),
                   experts_per_token=hf.get("num_experts_per_tok", 0))


PRESETS: dict[str, dict[str, Any]] = {
    # Public architecture hyper-parameters (weights are random-init; no checkpoints here).
    "gpt2-small": dict(arch="gpt2", vocab_size=50257, hidden_size=768, intermediate_size=3072,
                       num_layers=12, num_heads=12, num_kv_heads=12, head_dim=64, max_position=1024,
                       norm="layer", act="gelu", pos_emb="learned", bias=True, tie_embeddings=True),
    "llama3-8b": dict(arch="llama", vocab_size=128256, hidden_size=4096, intermediate_size=14336,
                      num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128, max_position=8192,
                      rope_theta=500000.0),
    "llama3-70b": dict(arch="llama", vocab_size=128256, hidden_size=8192, intermediate_size=28672,
                       num_layers=80, num_heads=64, num_kv_heads=8, head_dim=128, max_position=8192,
                       rope_theta=500000.0),
    "llama3.1-70b": dict(arch="llama", vocab_size=128256, hidden_size=8192, intermediate_size=28672,
                         num_layers=80, num_heads=64, num_kv_heads=8, head_dim=128,
                         max_position=131072, rope_theta=500000.0,
                         rope_scaling={"type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                       "high_freq_factor": 4.0,
                                       "original_max_position_embeddings": 8192}),
    "mixtral-8x7b": dict(arch="mixtral", vocab_size=32000, hidden_size=4096, intermediate_size=14336,
                         num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128,
                         max_position=32768, rope_theta=1e6, num_experts=8, experts_per_token=2),
    # Small configs for tests (same code paths, GPU-kernel-compatible dims).
    "llama-tiny": dict(arch="llama", vocab_size=1024, hidden_size=256, intermediate_size=512,
                       num_layers=2, num_heads=4, num_kv_heads=2, head_dim=128, max_position=2048,
                       rope_theta=10000.0, init_std=0.05),
    "llama-small": dict(arch="llama", vocab_size=4096, hidden_size=1024, intermediate_size=2048,
                        num_layers=4, num_heads=8, num_kv_heads=2, head_dim=128, max_position=4096,
                        rope_theta=500000.0, init_std=0.05),
    "gpt2-tiny": dict(arch="gpt2", vocab_size=512, hidden_size=128, intermediate_size=512,
                      num_layers=2, num_heads=2, num_kv_heads=2, head_dim=64, max_position=256,
                      norm="layer", act="gelu", pos_emb="learned", bias=True, tie_embeddings=True,
                      init_std=0.05),
    "mixtral-tiny": dict(arch="mixtral", vocab_size=1024, hidden_size=256, intermediate_size=512,
                         num_layers=2, num_heads=4, num_kv_heads=2, head_dim=128, max_position=2048,
                         rope_theta=1e6, num_experts=4, experts_per_token=2, init_std=0.05),
}


@dataclass
class ParallelConfig:
    tp: int = 1
    pp: int = 1
    ep: int = 1
    dp: int = 1
    # layer ranges per pipeline stage ([start, end) pairs); None = balanced split
    stage_layers: Optional[list] = None

    @property
    def world_size(self) -> int:
        # EP reuses the DP x TP ranks of a stage (DP-attention + expert-parallel FFN)
        return self.tp * self.pp * self.dp

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ParallelConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})


@dataclass
class EngineConfig:
    max_batch: int = 64               # max concurrent sequences per DP replica
    max_seq_len: int = 4096           # prompt + generated tokens per sequence
    max_prefill_tokens: int = 8192    # per engine step
    block_size: int = 32              # tokens per KV page (decode kernel is specialised to 32)
    kv_cache_tokens: Optional[int] = None   # explicit KV capacity; None = size from free HBM
    hbm_utilization: float = 0.92     # fraction of device memory the engine may use
    use_graphs: bool = True           # hipGraph-captured decode steps
    graph_batch_sizes: list = field(default_factory=lambda: [1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192, 256])
    seed: int = 0
    dtype: str = "bf16"
    custom_allreduce: bool = True     # one-shot IPC all-reduce for small TP messages
    # chunked prefill mixed into decode steps (pp == 1, no EP): every step decodes all running
    # sequences and fills the rest of max_prefill_tokens with prompt chunks
    mixed_prefill: bool = True
    # automatic prefix caching (with mixed_prefill): full prompt pages are registered under a
    # hash of their token prefix and reused by later requests that start with the same tokens
    prefix_caching: bool = True
    # KV-cache element type: "auto" (= the model dtype, bf16 on GPU) or "fp8" (e4m3, unscaled,
    # |x| <= 448): half the KV bytes per token, so twice the cached tokens and half the KV
    # traffic of a decode step; attention math stays bf16 (csrc/include/bfly_kv.h)
    kv_cache_dtype: str = "auto"
    # context-parallel prefill across data-parallel replicas (pp == 1, no EP): a prompt of at
    # least this many tokens is prefilled by ALL dp replicas together (ring or Ulysses
    # attention, parallel/context_parallel.py), its K/V collected in the cache of the replica
    # that then decodes it. 0 = off. Replicas step in lockstep while it is on.
    cp_prefill_min_tokens: int = 0
    # overlapped decode for single-stage layouts (pp == 1, no EP; the serving default): the
    # asynchronous pipeline of engine/pipeline.py with one group, so the host schedules step
    # k+1 (inputs gathered on the device from step k's sampled ids) while step k still runs, and
    # token values reach the host one step late. Mixed chunked prefill and prefix caching run
    # inside it (a plan's decode rows and prompt chunks travel together). Off (synchronous
    # steps) with context-parallel prefill, whose replicas step in lockstep.
    async_decode: bool = True
    cp_attention: str = "ring"        # "ring" | "ulysses"
    # request-state snapshots (engine/state.py): every `snapshot_every` steps one rank per DP
    # replica writes <snapshot_dir>/replica-<dp>.json; LLM(..., resume=dir) replays it
    snapshot_dir: Optional[str] = None
    snapshot_every: int = 0


def load_config_file(path: str | Path) -> dict:
    p = Path(path)
    text = p.read_text()
    if p.suffix in (".yaml", ".yml"):
        import yaml

        return yaml.safe_load(text)
    return json.loads(text)
