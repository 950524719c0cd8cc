"""Butterfly all-reduce: recursive halving (reduce-scatter) then recursive doubling
(all-gather) over point-to-point transfers — the measured alternative to RCCL's ring and our
one-shot IPC kernel that SURVEY.md §5.8 names for B3 ("the *butterfly* name suggests
recursive-doubling ... implement it only as a measured alternative").

For W = 2^k ranks, rank r in step s (s = k-1 .. 0) pairs with r XOR 2^s, splits its current
segment in two, sends the partner's half and adds the partner's copy of its own half; after
k steps every rank holds the fully reduced 1/W of the buffer, and k doubling steps in the
reverse order gather the reduced segments everywhere. Bytes per rank: 2 S (W-1)/W — a ring's
volume — but each step uses ONE peer link, where the fully connected xGMI mesh lets RCCL's
multi-channel rings and the two-shot IPC kernel (reduce-scatter + all-gather over all 7 links
at once) drive every link together; the start-up probe (`parallel/probe.py`) times it next to
them so the choice stays measured, not assumed.

Determinism: each element is summed along one fixed tree (the same pairs at the same steps
whatever the timing) on exactly one rank, then copied to the others, so every rank ends with
identical bits.
Non-power-of-two groups fall back to the group's regular all-reduce.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def is_pow2(n: int) -> bool:
    return n >= 1 and (n & (n - 1)) == 0


def _exchange(send: torch.Tensor, recv: torch.Tensor, peer: int, pg) -> None:
    """Send `send` to and receive `recv` from global rank `peer` (both posted before either
    waits, so the pair never deadlocks). Empty pieces are skipped on both sides alike: my send
    is the partner's receive, so their sizes always match."""
    ops = []
    if send.numel():
        ops.append(dist.P2POp(dist.isend, send, peer, pg))
    if recv.numel():
        ops.append(dist.P2POp(dist.irecv, recv, peer, pg))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def butterfly_all_reduce_(t: torch.Tensor, ranks: list, pg=None) -> torch.Tensor:
    """In-place sum of `t` over the global `ranks` (this process must be one of them) by
    recursive halving + doubling. `pg`: the process group holding those ranks (None = world)."""
    W = len(ranks)
    if W == 1:
        return t
    if not is_pow2(W):
        dist.all_reduce(t, group=pg)
        return t
    me = ranks.index(dist.get_rank())
    flat = t.view(-1)
    n = flat.numel()
    # segment [lo, hi) this rank is responsible for after each halving step
    lo, hi = 0, n
    bounds = []
    k = W.bit_length() - 1
    scratch = torch.empty_like(flat)
    for s in reversed(range(k)):
        partner = me ^ (1 << s)
        mid = lo + (hi - lo) // 2
        keep_lo = (me >> s) & 1 == 0          # the lower rank of the pair keeps the lower half
        klo, khi = (lo, mid) if keep_lo else (mid, hi)
        slo, shi = (mid, hi) if keep_lo else (lo, mid)
        recv = scratch[klo:khi]
        _exchange(flat[slo:shi].contiguous(), recv, ranks[partner], pg)
        flat[klo:khi].add_(recv)               # one addition per element and step: commutative
        bounds.append((lo, hi, klo, khi, keep_lo))
        lo, hi = klo, khi
    for s, (plo, phi, klo, khi, keep_lo) in zip(range(k), reversed(bounds)):
        partner = me ^ (1 << s)
        # the partner holds the other half of [plo, phi), fully reduced
        olo, ohi = (khi, phi) if keep_lo else (plo, klo)
        recv = scratch[olo:ohi]
        _exchange(flat[klo:khi].contiguous(), recv, ranks[partner], pg)
        flat[olo:ohi].copy_(recv)
    return t
