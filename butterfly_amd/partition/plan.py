"""PartitionPlan — the partitioning API's output and on-disk format.

The reference names a partitioning capability ("Algorithms to intelligently divide
transformer layers/attention heads", /root/reference/CLAUDE.md:21) but defines no format, so
this one is ours (frozen, versioned):

{
  "format": "butterfly-plan", "version": 1,
  "model": {...ModelConfig...},
  "n_gpus": 8, "dp": 1, "tp": 2, "pp": 4, "ep": 1,
  "stages": [[0, 20], [20, 40], [40, 60], [60, 80]],     # layer range per pipeline stage
  "placement": [0, 1, ..., 7],                          # mesh rank -> GPU index
  "kv_budget_bytes": [...], "weight_bytes": [...],      # per mesh rank
  "objective": "throughput", "estimate": {...},          # cost-model predictions
  "link_bytes_per_token": {"0-1": ..., ...}              # xGMI traffic per generated token
}
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Optional

from ..config import ModelConfig
from ..models.shard import Shard, local_dims
from ..parallel.mesh import Mesh

FORMAT = "butterfly-plan"
VERSION = 1


@dataclass
class ShardSpec:
    kind: str                 # "replicate" | "split" | "expert"
    dim: Optional[int] = None
    parts: int = 1
    index: int = 0


@dataclass
class PartitionPlan:
    model: ModelConfig
    n_gpus: int
    dp: int = 1
    tp: int = 1
    pp: int = 1
    ep: int = 1
    stages: list = field(default_factory=list)
    placement: list = field(default_factory=list)
    objective: str = "throughput"
    kv_budget_bytes: list = field(default_factory=list)
    weight_bytes: list = field(default_factory=list)
    estimate: dict = field(default_factory=dict)
    link_bytes_per_token: dict = field(default_factory=dict)

    # ---- derived ---------------------------------------------------------------------------
    @property
    def mesh(self) -> Mesh:
        return Mesh(dp=self.dp, pp=self.pp, tp=self.tp, ep=self.ep)

    @property
    def name(self) -> str:
        parts = [f"{k}{v}" for k, v in (("dp", self.dp), ("tp", self.tp), ("pp", self.pp), ("ep", self.ep)) if v > 1]
        return "x".join(parts) or "single"

    def shard(self, rank: int) -> Shard:
        c = self.mesh.coord(rank)
        a, b = self.stages[c.pp]
        return Shard(tp_rank=c.tp, tp_size=self.tp, layer_start=a, layer_end=b,
                     ep_rank=c.dp if self.ep > 1 else 0, ep_size=self.ep)

    def shard_spec(self, logical_name: str, rank: int = 0) -> ShardSpec:
        """How a logical parameter is split across the mesh (for tools / checkpoints)."""
        s = self.shard(rank)
        if ".experts." in logical_name:
            e = int(logical_name.split(".experts.")[1].split(".")[0])
            return ShardSpec("expert", None, self.ep, e // max(1, self.model.num_experts // self.ep))
        row_split = ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "mlp.fc.", "embed_tokens", "lm_head")
        col_split = ("o_proj.weight", "down_proj", "mlp.proj.weight")
        if any(k in logical_name for k in col_split):
            return ShardSpec("split", 1, self.tp, s.tp_rank)
        if any(k in logical_name for k in row_split):
            return ShardSpec("split", 0, self.tp, s.tp_rank)
        return ShardSpec("replicate")

    def validate(self) -> None:
        c = self.model
        if self.dp * self.tp * self.pp != self.n_gpus:
            raise ValueError(f"dp*tp*pp = {self.dp * self.tp * self.pp} != n_gpus {self.n_gpus}")
        if self.ep not in (1, self.dp):
            raise ValueError("ep must be 1 or dp")
        if len(self.stages) != self.pp:
            raise ValueError("one layer range per pipeline stage required")
        covered = []
        for a, b in self.stages:
            if b <= a:
                raise ValueError(f"empty stage {a}:{b}")
            covered.extend(range(a, b))
        if covered != list(range(c.num_layers)):
            raise ValueError("stages must cover every layer exactly once, in order")
        for r in range(self.n_gpus):
            local_dims(c, self.shard(r))      # raises on an incompatible tp/ep
        if self.placement and sorted(self.placement) != list(range(self.n_gpus)):
            raise ValueError("placement must be a permutation of GPU indices")

    # ---- serialisation -----------------------------------------------------------------------
    def to_dict(self) -> dict:
        d = asdict(self)
        d["model"] = self.model.to_dict()
        d["stages"] = [list(s) for s in self.stages]
        return {"format": FORMAT, "version": VERSION, **d}

    def to_json(self, path: Optional[str | Path] = None) -> str:
        text = json.dumps(self.to_dict(), indent=2)
        if path is not None:
            Path(path).write_text(text)
        return text

    @classmethod
    def from_dict(cls, d: dict) -> "PartitionPlan":
        if d.get("format") != FORMAT:
            raise ValueError(f"not a {FORMAT} document")
        if d.get("version", 0) > VERSION:
            raise ValueError(f"plan version {d['version']} is newer than supported {VERSION}")
        d = {k: v for k, v in d.items() if k not in ("format", "version")}
        d["model"] = ModelConfig.from_dict(d["model"])
        d["stages"] = [tuple(s) for s in d["stages"]]
        p = cls(**d)
        p.validate()
        return p

    @classmethod
    def from_json(cls, path_or_text: str | Path) -> "PartitionPlan":
        s = str(path_or_text)
        text = s if s.lstrip().startswith("{") else Path(s).read_text()
        return cls.from_dict(json.loads(text))
