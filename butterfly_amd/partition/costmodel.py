"""Analytic cost model for partition search.

Every op is priced max(FLOPs / sustained MFMA rate, bytes / sustained HBM rate) plus a
kernel-boundary overhead; collectives are priced against xGMI, from the measured table of
parallel/probe.py when the Hardware carries one (log-log interpolation over message size,
the fastest available implementation), else analytically:
  * IPC one-shot all-reduce of S bytes over t ranks: every rank pulls S from each peer, each
    over its own link: latency + S / link rate;
  * IPC two-shot (t >= 4): reduce-scatter + all-gather, 2S/t per link, two rendezvous;
  * RCCL: latency + 2(t-1)/t * S / bus bandwidth;
  * PP boundary: one link, S bytes, plus a hop latency.
Memory per rank = local weights + KV for the rank's sequences + activation workspace;
it must fit the usable HBM (288 GB per MI355X).
"""
from __future__ import annotations

import json
import math
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


def interp_loglog(pts: list, x: float) -> float:
    """Piecewise log-log interpolation of measured (bytes, seconds) points; linear in bytes
    beyond the largest point (bandwidth-bound), flat below the smallest (latency-bound)."""
    pts = sorted((float(a), float(b)) for a, b in pts)
    if x <= pts[0][0]:
        return pts[0][1]
    if x >= pts[-1][0]:
        if len(pts) == 1:
            return pts[0][1] * x / pts[0][0]
        (x0, y0), (x1, y1) = pts[-2], pts[-1]
        slope = (y1 - y0) / (x1 - x0) if x1 > x0 else 0.0
        return y1 + max(slope, 0.0) * (x - x1)
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if x0 <= x <= x1:
            if x0 <= 0 or y0 <= 0 or y1 <= 0:
                return y0 + (y1 - y0) * (x - x0) / (x1 - x0)
            f = math.log(x / x0) / math.log(x1 / x0)
            return math.exp(math.log(y0) + f * (math.log(y1) - math.log(y0)))
    return pts[-1][1]


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
        """Seconds for one all-reduce of `nbytes` over `n` ranks, with the implementation the
        runtime picks (parallel/comm.py): the IPC kernel for messages up to its buffer (two-shot
        from twoshot_ar_min_bytes on, groups of 4 / 8), RCCL otherwise."""
        if n <= 1:
            return 0.0
        hw = self.hw
        ipc_max, two_min = hw.oneshot_ar_max_bytes, hw.twoshot_ar_min_bytes
        pol = ((hw.comm or {}).get("policy") or {})
        pol = pol.get(n) or pol.get(str(n))
        if pol:       # measured crossovers (parallel/probe.py ar_policy), as the runtime uses them
            ipc_max, two_min = pol["ipc_max"], pol["twoshot_min"]
        ipc = self.oneshot and nbytes <= ipc_max and n in (2, 4, 8)
        two = ipc and n >= 4 and nbytes >= two_min
        impl = ("twoshot" if two else "oneshot") if ipc else "rccl"
        tab = (hw.comm or {}).get("all_reduce") or {}
        per_n = tab.get(impl) or {}
        pts = per_n.get(n) or per_n.get(str(n))
        if pts:
            return interp_loglog(pts, nbytes)
        link = hw.xgmi_link_eff_bw
        if two:
            return 2 * hw.oneshot_ar_latency_s + 2.0 * nbytes / (n * link)
        if ipc:
            # one-shot: every rank reads the n-1 peer buffers over n-1 distinct links at once
            return hw.oneshot_ar_latency_s + nbytes / link
        bus = min(hw.rccl_bus_bw, (n - 1) * link)
        return hw.collective_latency_s + 2.0 * (n - 1) / n * nbytes / bus

    def all_to_all(self, nbytes: float, n: int) -> float:
        """Equal-split all-to-all of `nbytes` per rank over `n` ranks: every peer block on its
        own xGMI link (measured table from the probe when available)."""
        if n <= 1:
            return 0.0
        tab = (self.hw.comm or {}).get("all_to_all") or {}
        pts = tab.get(n) or tab.get(str(n))
        if pts:
            return interp_loglog(pts, nbytes)
        return self.hw.collective_latency_s + nbytes / n / self.hw.xgmi_link_eff_bw

    def p2p(self, nbytes: float) -> float:
        pts = (self.hw.comm or {}).get("p2p")
        if pts:
            return interp_loglog(pts, nbytes)
        return self.hw.p2p_latency_s + nbytes / self.hw.xgmi_link_eff_bw

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
            if op.groups > 1:     # one grouped launch: each group streams its own weights
                per = self.gemm(max(1, tokens * op.m_scale // op.groups), op.n, op.k) - hw.kernel_overhead_s
                return op.groups * per + hw.kernel_overhead_s
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
            if op.collective == "all_to_all":
                return self.all_to_all(nbytes * g, g)     # `tokens` rows reserved per destination
            return hw.collective_latency_s + (g - 1) * nbytes / hw.xgmi_link_eff_bw
        # memory-bound elementwise / norm / rope / routing ops
        byts = op.act_bytes(tokens) + 2.0 * op.param_elems
        return byts / hw.hbm_bw_eff + hw.kernel_overhead_s

    def layer_time(self, tokens: int, tp: int, ctx: int, decode: bool, seqs: int = 0,
                   ep: int = 1, index: int = 0) -> LayerCost:
        """Layer `index` on `tokens` tokens (decode: one per sequence, each attending to `ctx`
        cached tokens; prefill: `seqs` causal sequences of tokens/seqs each)."""
        self._cur_ep = ep
        layer = self._ir(tp, ep).layers[index]
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

    def layer_costs(self, tokens: int, tp: int, ctx: int, decode: bool, seqs: int = 0,
                    ep: int = 1) -> list:
        """Every layer priced from its own IR spec (identical layers are priced once)."""
        memo: dict = {}
        out = []
        for layer in self._ir(tp, ep).layers:
            key = tuple((o.kind, o.n, o.k, o.m_scale, o.collective, o.group, o.width, o.param_elems)
                        for o in layer.ops)
            if key not in memo:
                memo[key] = self.layer_time(tokens, tp, ctx, decode, seqs, ep, layer.index)
            out.append(memo[key])
        return out

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
