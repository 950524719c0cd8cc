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

import json
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

from ..config import ModelConfig
from ..models.ir import OpSpec, build_ir
from .hw import MI355X, Hardware


@dataclass
class LayerCost:
    seconds: float
    weight_bytes: float
    comm_bytes: float


_CALIB = Path(__file__).resolve().parent / "calibration" / "mi355x_gemm.json"
_M_BUCKETS = (1, 16, 32, 64, 128, 256, 512)


def _load_gemm_calibration() -> dict:
    try:
        d = json.loads(_CALIB.read_text())
    except (OSError, ValueError):
        return {}
    out = {}
    for key, us in d.get("gemm", {}).items():
        n, k, m = (int(v) for v in key.split("x"))
        out[(n, k, m)] = us * 1e-6
    return out


class CostModel:
    """GEMM times come from the measured MI355X table (partition/calibration, produced by
    tools/gemm_tune.sh) when the shape is known, otherwise from max(FLOPs / eff(M), bytes /
    bandwidth) with an M-dependent MFMA efficiency fitted to the same measurements."""
    _calib: Optional[dict] = None

    def __init__(self, cfg: ModelConfig, hw: Hardware = MI355X, oneshot_allreduce: bool = True):
        self.cfg = cfg
        self.hw = hw
        self.oneshot = oneshot_allreduce
        if CostModel._calib is None:
            CostModel._calib = _load_gemm_calibration()
        self._irs: dict = {}
        self._cur_ep = 1

    # ---- primitives ------------------------------------------------------------------------
    def gemm(self, M: int, N: int, K: int) -> float:
        hw = self.hw
        bucket = next((b for b in _M_BUCKETS if b >= M), None)
        if bucket is not None and (N, K, bucket) in self._calib:
            return self._calib[(N, K, bucket)] + hw.kernel_overhead_s
        flops = 2.0 * M * N * K
        byts = 2.0 * (N * K + M * K + M * N)
        eff = hw.bf16_flops_eff * M / (M + 110.0)     # fit: 0.66 PF @128 ... 1.27 PF @8192
        return max(flops / eff, byts / hw.hbm_bw_eff) + hw.kernel_overhead_s

    def allreduce(self, nbytes: float, n: int) -> float:
        if n <= 1:
            return 0.0
        hw = self.hw
        if self.oneshot and nbytes <= hw.oneshot_ar_max_bytes:
            # one-shot: every rank reads the n-1 peer buffers over n-1 distinct links at once
            return hw.oneshot_ar_latency_s + nbytes / hw.xgmi_link_bw
        return hw.collective_latency_s + 2.0 * (n - 1) / n * nbytes / hw.xgmi_link_bw

    def p2p(self, nbytes: float) -> float:
        return self.hw.p2p_latency_s + nbytes / self.hw.xgmi_link_bw

    # ---- model pieces (priced from the model IR: models/ir.py) ---------------------------------
    def _ir(self, tp: int, ep: int):
        key = (tp, ep)
        if key not in self._irs:
            self._irs[key] = build_ir(self.cfg, tp, ep)
        return self._irs[key]

    def layer_weight_bytes(self, tp: int, ep: int = 1) -> float:
        return 2.0 * self._ir(tp, ep).layers[0].param_elems

    def op_time(self, op: OpSpec, tokens: int, ctx: int, decode: bool, seqs: int, tp: int) -> float:
        """Seconds for one IR op on one rank (collectives priced against xGMI)."""
        hw, c = self.hw, self.cfg
        if op.kind == "gemm":
            return self.gemm(tokens * op.m_scale, op.n, op.k)
        if op.kind == "attn":
            D = c.head_dim
            hq_l = c.num_heads // tp
            hkv_l = max(1, c.num_kv_heads // tp)
            if decode:
                kv_bytes = 2.0 * tokens * ctx * hkv_l * D * 2
                flops = 4.0 * tokens * ctx * hq_l * D
                return max(kv_bytes / hw.hbm_bw_eff, flops / hw.bf16_flops_eff) + hw.kernel_overhead_s
            L = tokens / max(seqs, 1)
            flops = 2.0 * tokens * L * hq_l * D   # causal: half of 4*T*L*H*D
            return flops / (0.6 * hw.bf16_flops_eff) + hw.kernel_overhead_s
        if op.kind == "collective":
            nbytes = 2.0 * tokens * op.width
            if op.collective == "all_reduce":
                return self.allreduce(nbytes, tp)
            g = tp if op.group == "tp" else max(2, self._cur_ep)
            return hw.collective_latency_s + (g - 1) * nbytes / hw.xgmi_link_bw
        # memory-bound elementwise / norm / rope / routing ops
        byts = op.act_bytes(tokens) + 2.0 * op.param_elems
        return byts / hw.hbm_bw_eff + hw.kernel_overhead_s

    def layer_time(self, tokens: int, tp: int, ctx: int, decode: bool, seqs: int = 0,
                   ep: int = 1) -> LayerCost:
        """One transformer layer on `tokens` tokens (decode: one per sequence, each attending
        to `ctx` cached tokens; prefill: `seqs` causal sequences of tokens/seqs each)."""
        self._cur_ep = ep
        layer = self._ir(tp, ep).layers[0]
        t = comm = 0.0
        comm_bytes = 0.0
        for op in layer.ops:
            dt = self.op_time(op, tokens, ctx, decode, seqs, tp)
            if op.kind == "collective":
                comm += dt
                comm_bytes += 2.0 * tokens * op.width
            else:
                t += dt
        return LayerCost(t + comm, 2.0 * layer.param_elems, comm_bytes)

    def embed_head_time(self, tokens: int, logits_rows: int, tp: int) -> tuple[float, float]:
        ir = self._ir(tp, 1)
        first = sum(self.op_time(o, tokens, 0, True, 1, tp) for o in ir.embed)
        last = sum(self.op_time(o, logits_rows, 0, True, 1, tp) for o in ir.head) + 2 * self.hw.kernel_overhead_s
        return first, last

    def embed_head_bytes(self, tp: int) -> tuple[float, float]:
        ir = self._ir(tp, 1)
        emb = 2.0 * sum(o.param_elems for o in ir.embed)
        head = 2.0 * sum(o.param_elems for o in ir.head if o.kind == "gemm")
        return emb, head
