"""Analytic cost model for partition search.

Every op is priced max(FLOPs / sustained MFMA rate, bytes / sustained HBM rate) plus a
kernel-boundary overhead; collectives are priced against xGMI:
  * TP all-reduce of S bytes over t ranks: ring (RCCL) moves 2(t-1)/t * S over ONE link per
    rank (per-link bound on a point-to-point mesh); small messages pay a fixed latency
    (the one-shot IPC kernel's when enabled).
  * PP boundary: one link, S bytes, plus a hop latency.
Memory per rank = local weights + KV for the rank's sequences + activation workspace;
it must fit the usable HBM (288 GB per MI355X).
"""
from __future__ import annotations

from dataclasses import dataclass

from ..config import ModelConfig
from .hw import MI355X, Hardware


@dataclass
class LayerCost:
    seconds: float
    weight_bytes: float
    comm_bytes: float


class CostModel:
    def __init__(self, cfg: ModelConfig, hw: Hardware = MI355X, oneshot_allreduce: bool = True):
        self.cfg = cfg
        self.hw = hw
        self.oneshot = oneshot_allreduce

    # ---- primitives ------------------------------------------------------------------------
    def gemm(self, M: int, N: int, K: int) -> float:
        hw = self.hw
        flops = 2.0 * M * N * K
        byts = 2.0 * (N * K + M * K + M * N)
        return max(flops / hw.bf16_flops_eff, byts / hw.hbm_bw_eff) + hw.kernel_overhead_s

    def allreduce(self, nbytes: float, n: int) -> float:
        if n <= 1:
            return 0.0
        hw = self.hw
        if self.oneshot and nbytes <= 512 * 1024:
            # one-shot: every rank reads the n-1 peer buffers over n-1 distinct links at once
            return hw.oneshot_ar_latency_s + nbytes / hw.xgmi_link_bw
        return hw.collective_latency_s + 2.0 * (n - 1) / n * nbytes / hw.xgmi_link_bw

    def p2p(self, nbytes: float) -> float:
        return self.hw.p2p_latency_s + nbytes / self.hw.xgmi_link_bw

    # ---- model pieces ------------------------------------------------------------------------
    def layer_weight_bytes(self, tp: int, ep: int = 1) -> float:
        c = self.cfg
        h, D = c.hidden_size, c.head_dim
        hkv_l = max(1, c.num_kv_heads // tp)
        attn = (c.num_heads // tp + 2 * hkv_l) * D * h + (c.num_heads // tp) * D * h
        mlp_cols = c.intermediate_size // (tp if ep == 1 else 1)
        mlp = (3 if c.act == "silu" else 2) * h * mlp_cols
        if c.is_moe:
            mlp *= c.num_experts // ep
            mlp += c.num_experts * h
        return 2.0 * (attn + mlp)

    def layer_time(self, tokens: int, tp: int, ctx: int, decode: bool, seqs: int = 0,
                   ep: int = 1) -> LayerCost:
        """One transformer layer on `tokens` tokens (decode: one per sequence, each attending
        to `ctx` cached tokens; prefill: `seqs` causal sequences of tokens/seqs each)."""
        c = self.cfg
        h, D = c.hidden_size, c.head_dim
        hq_l = c.num_heads // tp
        hkv_l = max(1, c.num_kv_heads // tp)
        t = 0.0
        t += self.gemm(tokens, (hq_l + 2 * hkv_l) * D, h)                # QKV
        t += self.gemm(tokens, h, hq_l * D)                               # O
        if c.is_moe:
            e_l = c.num_experts // ep
            f = c.intermediate_size // (tp if ep == 1 else 1)
            tt = tokens * ep
            t += self.gemm(tt, 2 * f * e_l, h) + self.gemm(tt, h, f * e_l)
        else:
            f = c.intermediate_size // tp
            n_up = 2 * f if c.act == "silu" else f
            t += self.gemm(tokens, n_up, h) + self.gemm(tokens, h, f)
        if decode:
            kv_bytes = 2.0 * tokens * ctx * hkv_l * D * 2
            flops = 4.0 * tokens * ctx * hq_l * D
            t += max(kv_bytes / self.hw.hbm_bw_eff, flops / self.hw.bf16_flops_eff) + self.hw.kernel_overhead_s
        else:
            L = tokens / max(seqs, 1)
            flops = 2.0 * tokens * L * hq_l * D   # causal: half of 4*T*L*H*D
            t += flops / (0.6 * self.hw.bf16_flops_eff) + self.hw.kernel_overhead_s
        t += 6 * self.hw.kernel_overhead_s                                 # norms, rope, act
        ar_bytes = 2.0 * tokens * h
        comm = 0.0
        if tp > 1:
            comm = 2 * self.allreduce(ar_bytes, tp)
        if c.is_moe and ep > 1:
            comm += 2 * (self.hw.collective_latency_s + (ep - 1) / ep * ar_bytes * ep / self.hw.xgmi_link_bw)
        return LayerCost(t + comm, self.layer_weight_bytes(tp, ep), ar_bytes * 2 * (tp > 1))

    def embed_head_time(self, tokens: int, logits_rows: int, tp: int) -> tuple[float, float]:
        c = self.cfg
        v_l = c.vocab_size / tp
        first = 2.0 * tokens * c.hidden_size / self.hw.hbm_bw_eff + self.hw.kernel_overhead_s
        if tp > 1:
            first += self.allreduce(2.0 * tokens * c.hidden_size, tp)
        last = self.gemm(logits_rows, int(v_l), c.hidden_size) + 3 * self.hw.kernel_overhead_s
        return first, last

    def embed_head_bytes(self, tp: int) -> tuple[float, float]:
        c = self.cfg
        emb = 2.0 * c.vocab_size * c.hidden_size / tp
        head = 0.0 if c.tie_embeddings else emb
        return emb, head
