"""Model IR: the per-layer op list the partitioner prices and the scheduler reasons about
(the reference's "divide transformer layers/attention heads",
/root/reference/CLAUDE.md:21).

`build_ir(cfg, tp, ep)` describes what ONE rank of a (tp, ep) shard executes per layer: each
op carries its kind, the GEMM shape it runs (M is the token count, filled in at pricing time),
the parameters it reads and the collective it issues. The same list drives
  * partition/costmodel.py — time = sum over ops of max(FLOPs / rate, bytes / bandwidth),
  * memory accounting — parameter bytes per layer / per stage,
  * tools that print per-op FLOPs and bytes for a plan (`python -m butterfly_amd info`).
The transformer forward (models/transformer.py) executes exactly these ops in this order, so
the IR and the kernels stay in one-to-one correspondence (see `OP_KERNELS`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

from ..config import ModelConfig


@dataclass(frozen=True)
class OpSpec:
    name: str
    kind: str                      # gemm | attn | norm | rope | act | route | collective | embed
    n: int = 0                     # gemm: output columns (local)
    k: int = 0                     # gemm: reduction dim (local)
    m_scale: int = 1               # gemm rows = tokens * m_scale (routed MoE: top-k slots per token)
    groups: int = 1                # grouped gemm: the rows split over `groups` weight matrices
    params: tuple = ()             # (logical name, local shape) read by this op
    collective: Optional[str] = None   # all_reduce | all_gather | reduce_scatter
    group: Optional[str] = None        # tp | ep
    width: int = 0                 # activation row width moved / normalised (elements)

    @property
    def param_elems(self) -> int:
        total = 0
        for _, shape in self.params:
            n = 1
            for d in shape:
                n *= d
            total += n
        return total

    def flops(self, tokens: int) -> float:
        if self.kind == "gemm":
            return 2.0 * tokens * self.m_scale * self.n * self.k     # groups share the rows
        return 0.0

    def act_bytes(self, tokens: int, dtype_bytes: int = 2) -> float:
        """Activation bytes read + written (weights excluded)."""
        if self.kind == "gemm":
            return dtype_bytes * tokens * self.m_scale * (self.n + self.k)
        return 2.0 * dtype_bytes * tokens * self.width


@dataclass
class LayerSpec:
    index: int
    ops: list = field(default_factory=list)

    @property
    def param_elems(self) -> int:
        return sum(o.param_elems for o in self.ops)

    def op(self, name: str) -> OpSpec:
        for o in self.ops:
            if o.name == name:
                return o
        raise KeyError(name)


@dataclass
class ModelIR:
    cfg: ModelConfig
    tp: int
    ep: int
    embed: list
    layers: list
    head: list

    @property
    def param_elems(self) -> int:
        return (sum(o.param_elems for o in self.embed) + sum(l.param_elems for l in self.layers)
                + sum(o.param_elems for o in self.head))


# kernel(s) each op kind runs on the GPU (for docs / traces)
OP_KERNELS = {
    "embed": "embed_kernel", "norm": "rmsnorm_kernel | layernorm_kernel (fused residual add)",
    "gemm": "gemm_tile_kernel | gemm_skinny_kernel (+ split-K reduce)",
    "rope": "rope_kv_kernel (fused KV-cache append) | kv_append_kernel",
    "attn": "attn_decode_kernel + attn_decode_combine_kernel | attn_prefill_kernel",
    "act": "gemm SiLU epilogue | gelu_kernel", "route": "moe_route_kernel + moe_gate_scale_kernel",
    "collective": "allreduce_kernel (one-shot IPC, fused add+norm) | RCCL",
}


def build_ir(cfg: ModelConfig, tp: int = 1, ep: int = 1) -> ModelIR:
    """Per-rank op lists for a (tp, ep) shard of `cfg` (all layers; a pipeline stage is a slice)."""
    h, D = cfg.hidden_size, cfg.head_dim
    hq = cfg.num_heads // tp
    hkv = max(1, cfg.num_kv_heads // tp)
    vocab_l = -(-cfg.vocab_size // (128 * tp)) * 128          # padded vocab shard
    norm_params = lambda nm: ((nm + ".weight", (h,)),) + (((nm + ".bias", (h,)),) if cfg.norm == "layer" else ())  # noqa: E731
    embed = [OpSpec("embed", "embed", params=(("embed_tokens.weight", (vocab_l, h)),), width=h)]
    if tp > 1:
        embed.append(OpSpec("embed_allreduce", "collective", collective="all_reduce", group="tp", width=h))
    if cfg.pos_emb == "learned":
        embed.append(OpSpec("pos_embed", "embed", params=(("pos_embed.weight", (cfg.max_position, h)),), width=h))
    layers = []
    for i in range(cfg.num_layers):
        L = f"layers.{i}."
        ops = [OpSpec("input_norm", "norm", params=norm_params(L + "input_norm"), width=h)]
        qkv_n = (hq + 2 * hkv) * D
        ops.append(OpSpec("qkv", "gemm", n=qkv_n, k=h,
                          params=((L + "attn.qkv_proj.weight", (qkv_n, h)),)
                          + (((L + "attn.qkv_proj.bias", (qkv_n,)),) if cfg.bias else ())))
        if cfg.pos_emb == "rope":
            ops.append(OpSpec("rope_kv", "rope", width=(hq + 2 * hkv) * D))
        ops.append(OpSpec("attention", "attn", width=hq * D))
        ops.append(OpSpec("o", "gemm", n=h, k=hq * D,
                          params=((L + "attn.o_proj.weight", (h, hq * D)),)
                          + (((L + "attn.o_proj.bias", (h,)),) if cfg.bias else ())))
        if tp > 1:
            ops.append(OpSpec("attn_allreduce", "collective", collective="all_reduce", group="tp", width=h))
        ops.append(OpSpec("post_norm", "norm", params=norm_params(L + "post_norm"), width=h))
        if cfg.is_moe:
            e_l = cfg.num_experts // ep
            f = cfg.intermediate_size // (tp if ep == 1 else 1)
            ops.append(OpSpec("router", "route", params=((L + "moe.router.weight", (cfg.num_experts, h)),), width=h))
            if ep > 1:
                # fixed-capacity all-to-all dispatch; each rank then runs its experts on the
                # rows routed to them only (on average tokens x top_k rows over e_l experts)
                kt = cfg.experts_per_token
                ops.append(OpSpec("ep_dispatch", "collective", collective="all_to_all", group="ep", width=h))
                ops.append(OpSpec("experts_gate_up", "gemm", n=2 * f, k=h, m_scale=kt, groups=e_l,
                                  params=((L + "moe.experts.gate_up", (e_l, 2 * f, h)),)))
                ops.append(OpSpec("experts_down", "gemm", n=h, k=f, m_scale=kt, groups=e_l,
                                  params=((L + "moe.experts.down", (e_l, h, f)),)))
                ops.append(OpSpec("ep_combine", "collective", collective="all_to_all", group="ep", width=h))
            else:
                # decode without EP: every local expert on every row (dense, fixed shape)
                ops.append(OpSpec("experts_gate_up", "gemm", n=2 * f * e_l, k=h,
                                  params=((L + "moe.experts.gate_up", (e_l, 2 * f, h)),)))
                ops.append(OpSpec("experts_down", "gemm", n=h, k=f * e_l,
                                  params=((L + "moe.experts.down", (e_l, h, f)),)))
            if ep > 1:
                pass
            elif tp > 1:
                ops.append(OpSpec("mlp_allreduce", "collective", collective="all_reduce", group="tp", width=h))
        else:
            f = cfg.intermediate_size // tp
            if cfg.act == "silu":
                ops.append(OpSpec("gate_up", "gemm", n=2 * f, k=h,
                                  params=((L + "mlp.gate_up_proj.weight", (2 * f, h)),)))
            else:
                ops.append(OpSpec("fc", "gemm", n=f, k=h, params=((L + "mlp.fc.weight", (f, h)),)
                                  + (((L + "mlp.fc.bias", (f,)),) if cfg.bias else ())))
                ops.append(OpSpec("gelu", "act", width=f))
            ops.append(OpSpec("down", "gemm", n=h, k=f, params=((L + "mlp.down_proj.weight", (h, f)),)
                              + (((L + "mlp.down_proj.bias", (h,)),) if cfg.bias else ())))
            if tp > 1:
                ops.append(OpSpec("mlp_allreduce", "collective", collective="all_reduce", group="tp", width=h))
        layers.append(LayerSpec(i, ops))
    head = [OpSpec("final_norm", "norm", params=norm_params("final_norm"), width=h)]
    head.append(OpSpec("lm_head", "gemm", n=vocab_l, k=h,
                       params=() if cfg.tie_embeddings else (("lm_head.weight", (vocab_l, h)),)))
    return ModelIR(cfg, tp, ep, embed, layers, head)
