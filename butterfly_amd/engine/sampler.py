"""Token selection over vocab-parallel logits.

Fast path (greedy and pure temperature sampling): the HIP sample kernel reduces each rank's
vocab shard to one (score, id) pair per row — Gumbel-max keyed on the GLOBAL token id and a
per-request seed, so shards are comparable — and the TP group all-gathers B x 8 bytes and
keeps the max (SURVEY.md §2.7-C "TP sampling"). No full-vocab gather, graph-capturable.

Filtered path (top-k / top-p / repetition penalty): gather the full logits row across TP and
filter with torch ops; only rows that ask for it take this path.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import ops


@dataclass
class SamplingParams:
    temperature: float = 0.0          # 0 = greedy
    top_k: int = 0                    # 0 = off
    top_p: float = 1.0
    max_tokens: int = 16
    stop_token_ids: list = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None

    @property
    def needs_filter(self) -> bool:
        return self.temperature > 0 and (self.top_k > 0 or self.top_p < 1.0)


class Sampler:
    def __init__(self, comm, vocab_size: int, vocab_start: int, tp: int):
        self.comm = comm
        self.vocab_size = vocab_size
        self.vocab_start = vocab_start
        self.tp = tp

    def _local_valid(self, logits: torch.Tensor) -> torch.Tensor:
        # drop padded vocab rows (they exist so each shard is a multiple of 128 rows)
        n = max(0, min(logits.shape[1], self.vocab_size - self.vocab_start))
        return logits[:, :n]

    def sample(self, logits: torch.Tensor, temps: Optional[torch.Tensor] = None,
               seeds: Optional[torch.Tensor] = None, params: Optional[list] = None) -> torch.Tensor:
        """logits: [R, vocab_local]. Returns int32 token ids [R] (identical on every TP rank)."""
        if params and any(p.needs_filter for p in params):
            return self._sample_filtered(logits, params, seeds)
        lv = self._local_valid(logits)
        ids, scores = ops.sample(lv, temps, seeds, vstart=self.vocab_start)
        if self.tp == 1:
            return ids
        pair = torch.stack([scores, ids.to(torch.float32)], 1)        # ids < 2^24: exact in f32
        allp = self.comm.all_gather(pair, "tp").view(self.tp, -1, 2)  # [tp, R, 2]
        best = allp[:, :, 0].argmax(0)                                 # ties -> lowest rank
        return allp.gather(0, best.view(1, -1, 1).expand(1, -1, 2))[0, :, 1].to(torch.int32)

    def _sample_filtered(self, logits, params, seeds):
        full = logits
        if self.tp > 1:
            g = self.comm.all_gather(logits.t().contiguous(), "tp")   # [tp*V_l, R]
            full = g.t()
        full = full[:, : self.vocab_size].float()
        out = torch.empty(full.shape[0], dtype=torch.int32, device=full.device)
        for r, p in enumerate(params):
            row = full[r]
            if p.temperature <= 0:
                out[r] = int(row.argmax())
                continue
            row = row / p.temperature
            if p.top_k > 0:
                kth = torch.topk(row, min(p.top_k, row.numel())).values[-1]
                row = row.masked_fill(row < kth, float("-inf"))
            if p.top_p < 1.0:
                sv, si = torch.sort(row, descending=True)
                cp = torch.softmax(sv, -1).cumsum(-1)
                drop = cp - torch.softmax(sv, -1) > p.top_p
                row = row.scatter(0, si[drop], float("-inf"))
            g = torch.Generator(device="cpu")
            g.manual_seed(int(seeds[r]) if seeds is not None else 0)
            probs = torch.softmax(row, -1).cpu()
            out[r] = int(torch.multinomial(probs, 1, generator=g))
        return out
