"""Hardware model of one MI355X node (the partitioner's view).

Numbers: HBM and MFMA from /opt/skills/guides/MI355X_MICROARCH.md (chip table: 288 GB HBM3E,
6.29 TB/s measured copy bandwidth, ~2.5 PF dense bf16 spec); xGMI from the task brief
(7 links x ~153 GB/s per GPU, point-to-point full mesh on an 8-GPU node). "eff" fields are
what our kernels sustain (measured on one MI355X). The communication fields are NOT measured
on this hardware — one GPU per test box — they are conservative defaults (the per-direction
sustained link rate is taken as ~0.45 of the nominal figure, which may count both directions).
On a real node the benchmark replaces them by a measured table: `parallel/probe.py` times
RCCL and IPC all-reduces, send/recv and all-to-all at start-up and `with_comm_table` attaches
it; the cost model then interpolates measurements instead of using these constants.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, replace
from pathlib import Path
from typing import Optional


@dataclass(frozen=True)
class Hardware:
    name: str = "MI355X"
    gpus_per_node: int = 8
    hbm_bytes: float = 288e9
    hbm_bw: float = 6.29e12            # measured copy bandwidth
    hbm_bw_eff: float = 5.7e12          # sustained by weight-streaming GEMMs / paged attention (measured)
    bf16_flops: float = 2.5e15          # dense spec
    bf16_flops_eff: float = 1.3e15      # large-M asymptote of our 256x256 MFMA GEMM (measured 1.27 PF @8192)
    xgmi_links: int = 7                 # per GPU, full mesh within a node
    xgmi_link_bw: float = 153e9         # nominal per link (task brief)
    xgmi_link_eff_bw: float = 69e9      # assumed sustained per link per direction (default only)
    rccl_bus_bw: float = 300e9          # assumed RCCL all-reduce bus bandwidth, 8 ranks (default only)
    kernel_overhead_s: float = 1.5e-6   # dependent kernel boundary inside a graph (measured)
    collective_latency_s: float = 12e-6  # small-message RCCL all-reduce (default only)
    p2p_latency_s: float = 8e-6         # RCCL send/recv hop (default only)
    oneshot_ar_latency_s: float = 5e-6  # IPC all-reduce rendezvous (default only)
    oneshot_ar_max_bytes: float = 8 << 20  # larger all-reduces go to RCCL (BFLY_CUSTOM_AR_MAX_BYTES)
    twoshot_ar_min_bytes: float = 512 << 10  # BFLY_CUSTOM_AR_2SHOT_BYTES
    usable_hbm_fraction: float = 0.92
    comm: Optional[dict] = None         # measured table from parallel/probe.py (or a calibration file)

    def to_dict(self) -> dict:
        return asdict(self)

    def with_comm_table(self, table: Optional[dict]) -> "Hardware":
        """This hardware with measured collective times (parallel/probe.py format)."""
        return replace(self, comm=table) if table else self

    @classmethod
    def from_calibration(cls, path: str | Path, base: "Hardware" = None) -> "Hardware":
        base = base or cls()
        d = json.loads(Path(path).read_text())
        known = {k: v for k, v in d.items() if k in asdict(base)}
        return replace(base, **known)


MI355X = Hardware()
