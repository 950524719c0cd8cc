"""Device mesh: global rank <-> (dp, pp, tp) coordinates and the process groups of each axis.

Rank order is TP-innermost: rank = (dp * pp_size + pp) * tp_size + tp. On an MI355X node
every GPU pair has its own xGMI link (full mesh, 7 links per GPU), so "adjacent" ranks are
not physically closer; TP-innermost keeps a TP group's ranks on one node when the job spans
nodes, which is what matters for the bandwidth-heavy all-reduces. Expert parallelism reuses
the DP axis (DP-attention + expert-parallel FFN: SURVEY.md §2.6 EP row): ep_size = dp_size.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional


@dataclass(frozen=True)
class MeshCoord:
    dp: int
    pp: int
    tp: int


@dataclass(frozen=True)
class Mesh:
    dp: int = 1
    pp: int = 1
    tp: int = 1
    ep: int = 1   # 1 or == dp

    def __post_init__(self):
        if self.ep not in (1, self.dp):
            raise ValueError(f"ep ({self.ep}) must be 1 or equal to dp ({self.dp})")

    @property
    def world_size(self) -> int:
        return self.dp * self.pp * self.tp

    def coord(self, rank: int) -> MeshCoord:
        tp = rank % self.tp
        pp = (rank // self.tp) % self.pp
        dp = rank // (self.tp * self.pp)
        return MeshCoord(dp, pp, tp)

    def rank(self, dp: int, pp: int, tp: int) -> int:
        return (dp * self.pp + pp) * self.tp + tp

    def tp_group(self, rank: int) -> list[int]:
        c = self.coord(rank)
        return [self.rank(c.dp, c.pp, t) for t in range(self.tp)]

    def pp_group(self, rank: int) -> list[int]:
        c = self.coord(rank)
        return [self.rank(c.dp, p, c.tp) for p in range(self.pp)]

    def dp_group(self, rank: int) -> list[int]:
        c = self.coord(rank)
        return [self.rank(d, c.pp, c.tp) for d in range(self.dp)]

    def all_groups(self, axis: str) -> list[list[int]]:
        """Every group of one axis (torch.distributed.new_group must be called by all ranks
        for every group, in the same order)."""
        seen, out = set(), []
        fn = {"tp": self.tp_group, "pp": self.pp_group, "dp": self.dp_group,
              "ep": self.dp_group}[axis]
        for r in range(self.world_size):
            g = tuple(fn(r))
            if g not in seen:
                seen.add(g)
                out.append(list(g))
        return out

    def next_stage(self, rank: int) -> Optional[int]:
        c = self.coord(rank)
        return self.rank(c.dp, c.pp + 1, c.tp) if c.pp + 1 < self.pp else None

    def prev_stage(self, rank: int) -> Optional[int]:
        c = self.coord(rank)
        return self.rank(c.dp, c.pp - 1, c.tp) if c.pp > 0 else None
