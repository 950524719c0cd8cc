"""Hardware model of one MI355X node (the partitioner's view).

Numbers: HBM and MFMA from /opt/skills/guides/MI355X_MICROARCH.md (chip table: 288 GB HBM3E,
6.29 TB/s measured copy bandwidth, ~2.5 PF dense bf16 spec); xGMI from the task brief
(7 links x ~153 GB/s per GPU, point-to-point full mesh on an 8-GPU node). "eff" fields are
what our kernels sustain and are meant to be overwritten by a calibration file written by
the benchmark (`Hardware.from_calibration`).
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, replace
from pathlib import Path


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
    xgmi_link_bw: float = 153e9         # bytes/s per link per direction
    kernel_overhead_s: float = 1.5e-6   # dependent kernel boundary inside a graph
    collective_latency_s: float = 12e-6  # small-message RCCL all-reduce
    p2p_latency_s: float = 8e-6         # RCCL send/recv hop
    oneshot_ar_latency_s: float = 5e-6  # one-shot IPC all-reduce (small messages)
    oneshot_ar_max_bytes: float = 8 << 20  # larger all-reduces go to RCCL (BFLY_CUSTOM_AR_MAX_BYTES)
    usable_hbm_fraction: float = 0.92

    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_calibration(cls, path: str | Path, base: "Hardware" = None) -> "Hardware":
        base = base or cls()
        d = json.loads(Path(path).read_text())
        known = {k: v for k, v in d.items() if k in asdict(base)}
        return replace(base, **known)


MI355X = Hardware()
