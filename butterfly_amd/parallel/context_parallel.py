"""Context parallelism (CP): one long prompt's prefill split by sequence position over a group
of ranks, with ring attention (SURVEY.md §2.6 "CP / ring attention", §5.7; K16 LSE merge).

Layout: every sequence of the batch is cut into `cp` contiguous chunks, chunk r on cp rank r
(the remainder goes to the LAST ranks, so the final token — the one that needs logits — is on
the last rank for every non-empty sequence). Each rank runs the full model (weights replicated
over the CP group; TP inside it is orthogonal) on its own tokens only: projections, MLP and
norms touch 1/cp of the tokens and the KV cache holds only the rank's chunk.

Attention (`ring_attention`): the local queries first attend causally to the local keys; then
the K/V chunks travel around the ring (rank r sends to r+1 and receives from r-1, cp-1 steps).
A chunk that came from an earlier position (source rank < r) is fully visible: non-causal flash
attention over it returns a partial output and its log-sum-exp, merged into f32 accumulators by
the LSE-merge kernel; chunks from later positions are masked entirely and only relayed. The
transfer of step j+1 is posted before step j's attention runs, so on RCCL the K/V hop over
xGMI overlaps the flash-attention kernel. The result equals single-device causal attention up to
floating-point reassociation (tests/test_context_parallel.py).

Ulysses (`ulysses_attention`, CPContext.attn = "ulysses"): instead of moving K/V around the
ring, two all-to-alls re-shard the attention from "all heads of 1/cp of the tokens" to "1/cp
of the heads of all tokens" and back; attention then runs as ordinary causal flash attention
over whole sequences. It needs Hkv % cp == 0 (GQA: at most 8-way for Llama-3) and moves
q/k/v/o once each, where the ring moves K/V cp-1 times; the ring has no head constraint.

KV sink (the serving engine's use, engine/engine.py `_cp_step`): one rank of the group — the
one that will DECODE the sequence, placed last in chunk order so it also holds the final
token's logits — collects the whole prompt's K/V into its own paged cache. With the ring this
costs no extra traffic: every other rank's chunk passes through every rank during the cp-1
hops, and the sink appends each one (kv_append at its slots) as it arrives. With Ulysses the
chunks are all-gathered once more after the attention.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops


def split_lengths(L: int, cp: int) -> list[int]:
    """Chunk lengths of an L-token sequence over cp ranks (remainder to the last ranks)."""
    base, extra = divmod(L, cp)
    return [base + (1 if r >= cp - extra else 0) for r in range(cp)]


@dataclass
class CPContext:
    """Static description of one context-parallel prefill step on one rank."""
    ranks: list                  # global ranks of the CP group, in chunk order
    rank: int                    # this rank's index in the group (= its chunk)
    pg: Optional[object]         # torch process group of `ranks` (None when cp == 1)
    lens: list                   # lens[r][i] = tokens of sequence i held by cp rank r
    attn: str = "ring"           # "ring" | "ulysses"
    sink: Optional[list] = None  # on the KV sink rank: sink[r] = its cache slots of chunk r (int32)

    @property
    def size(self) -> int:
        return len(self.ranks)

    def cu(self, r: int, device) -> torch.Tensor:
        c = [0]
        for n in self.lens[r]:
            c.append(c[-1] + n)
        return torch.tensor(c, dtype=torch.int32, device=device)

    def tokens(self, r: int) -> int:
        return sum(self.lens[r])

    def max_len(self, r: int) -> int:
        return max(self.lens[r]) if self.lens[r] else 0


def _nccl(pg) -> bool:
    return pg is not None and dist.get_backend(pg) == "nccl"


class _RingHop:
    """Send `t` to the next rank and receive the previous rank's chunk into `out`. RCCL: one
    grouped isend/irecv pair (stream-ordered, overlaps the caller's compute until `wait`).
    gloo (CPU tests / ranks sharing a GPU): blocking, even ranks send first, odd ranks receive
    first, host-staged for device tensors."""

    def __init__(self, ctx: CPContext, t: torch.Tensor, out: torch.Tensor):
        n, r = ctx.size, ctx.rank
        dst, src = ctx.ranks[(r + 1) % n], ctx.ranks[(r - 1) % n]
        self.out, self.reqs = out, []
        if _nccl(ctx.pg):
            ops_ = [dist.P2POp(dist.isend, t.contiguous(), dst, ctx.pg),
                    dist.P2POp(dist.irecv, out, src, ctx.pg)]
            self.reqs = dist.batch_isend_irecv(ops_)
            return
        host_t = t.detach().cpu().contiguous()
        host_o = torch.empty(out.shape, dtype=out.dtype)
        if r % 2 == 0:
            dist.send(host_t, dst, group=ctx.pg)
            dist.recv(host_o, src, group=ctx.pg)
        else:
            dist.recv(host_o, src, group=ctx.pg)
            dist.send(host_t, dst, group=ctx.pg)
        out.copy_(host_o)

    def wait(self) -> torch.Tensor:
        for q in self.reqs:
            q.wait()
        return self.out


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, ctx: CPContext,
                   scale: float, kv_sink=None) -> torch.Tensor:
    """Causal attention of this rank's query chunk against the whole sequence, whose K/V chunks
    live on the other CP ranks. q [T, Hq, D], k/v [T, Hkv, D] (this rank's tokens, packed per
    sequence as ctx.lens[rank]); returns [T, Hq, D] in q's dtype. `kv_sink(r, k, v)` (sink
    rank only) receives every other rank's chunk as it passes."""
    r, n = ctx.rank, ctx.size
    dev = q.device
    cu_r = ctx.cu(r, dev)
    out, lse = ops.attn_prefill(q, k, v, cu_r, ctx.max_len(r), scale, True, return_lse=True)
    if n == 1:
        return out
    sink = kv_sink
    acc_o, acc_lse = out.float(), lse
    Hkv, D = k.shape[1], k.shape[2]
    cur = torch.stack([k, v], 1).contiguous()         # [T, 2, Hkv, D]: one message per hop
    for j in range(1, n):
        src = (r - j) % n                              # whose chunk arrives at step j
        nxt = torch.empty(ctx.tokens(src), 2, Hkv, D, dtype=k.dtype, device=dev)
        hop = _RingHop(ctx, cur, nxt)
        cur = hop.wait()
        if sink is not None and ctx.tokens(src) > 0:
            sink(src, cur[:, 0], cur[:, 1])
        if src < r and ctx.tokens(src) > 0:            # earlier positions: fully visible
            o_j, lse_j = ops.attn_prefill(q, cur[:, 0], cur[:, 1], cu_r, ctx.max_len(r), scale, False,
                                          cu_seqlens_k=ctx.cu(src, dev), return_lse=True)
            ops.attn_lse_merge_(acc_o, acc_lse, o_j, lse_j)
    return acc_o.to(q.dtype)


def _pg_order(ctx: CPContext) -> list:
    """Chunk indices sorted by their rank's position in the process group (collectives that
    index by group rank, e.g. all_to_all_single, see the group's own order; the chunk order
    of an engine CP step puts the sink rank last whatever its group rank)."""
    if ctx.pg is None:
        return list(range(ctx.size))
    return sorted(range(ctx.size), key=lambda j: dist.get_group_rank(ctx.pg, ctx.ranks[j]))


def _a2a(send: torch.Tensor, send_rows: list, recv_rows: list, ctx: CPContext) -> torch.Tensor:
    """all-to-all along dim 0: rows [sum(send_rows[:j]), +send_rows[j]) go to chunk rank j;
    the blocks received from every chunk rank (recv_rows[j] from j) come back concatenated."""
    order = _pg_order(ctx)
    if order != list(range(ctx.size)):
        offs = [sum(send_rows[:j]) for j in range(ctx.size)]
        send = torch.cat([send[offs[j]:offs[j] + send_rows[j]] for j in order])
        got = _a2a_pg(send, [send_rows[j] for j in order], [recv_rows[j] for j in order], ctx)
        blocks, a = {}, 0
        for j in order:
            blocks[j] = got[a:a + recv_rows[j]]
            a += recv_rows[j]
        return torch.cat([blocks[j] for j in range(ctx.size)])
    return _a2a_pg(send, send_rows, recv_rows, ctx)


def _a2a_pg(send: torch.Tensor, send_rows: list, recv_rows: list, ctx: CPContext) -> torch.Tensor:
    out = torch.empty((sum(recv_rows),) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
    if _nccl(ctx.pg):
        dist.all_to_all_single(out, send.contiguous(), output_split_sizes=list(recv_rows),
                               input_split_sizes=list(send_rows), group=ctx.pg)
        return out
    host = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(host, send.detach().cpu().contiguous(), output_split_sizes=list(recv_rows),
                           input_split_sizes=list(send_rows), group=ctx.pg)
    return out.copy_(host)


def _gather_chunks(k: torch.Tensor, v: torch.Tensor, ctx: CPContext, kv_sink) -> None:
    """Every rank's K/V chunk to the sink rank (Ulysses keeps no whole-head K/V anywhere):
    one all-gather of the chunks padded to the longest; only the sink keeps the result."""
    n, r = ctx.size, ctx.rank
    Tm = max(ctx.tokens(j) for j in range(n))
    Hkv, D = k.shape[1], k.shape[2]
    mine = torch.zeros(Tm, 2, Hkv, D, dtype=k.dtype, device=k.device)
    mine[: k.shape[0], 0], mine[: k.shape[0], 1] = k, v
    order = _pg_order(ctx)
    if _nccl(ctx.pg):
        got = torch.empty(n * Tm, 2, Hkv, D, dtype=k.dtype, device=k.device)
        dist.all_gather_into_tensor(got, mine, group=ctx.pg)
    else:
        host = [torch.empty(Tm, 2, Hkv, D, dtype=k.dtype) for _ in range(n)]
        dist.all_gather(host, mine.detach().cpu(), group=ctx.pg)
        got = torch.cat(host).to(k.device)
    if kv_sink is None:
        return
    for gi, j in enumerate(order):           # gathered blocks come in group-rank order
        if j != r and ctx.tokens(j) > 0:
            blk = got[gi * Tm: gi * Tm + ctx.tokens(j)]
            kv_sink(j, blk[:, 0], blk[:, 1])


def ulysses_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, ctx: CPContext,
                      scale: float, kv_sink=None) -> torch.Tensor:
    """Same contract as ring_attention, by sequence<->head all-to-alls (Hkv % cp == 0)."""
    if ctx.sink is not None:
        # collective: every rank takes part when the step has a sink rank
        _gather_chunks(k, v, ctx, kv_sink)
    n, r = ctx.size, ctx.rank
    T, Hq, D = q.shape
    Hkv = k.shape[1]
    if Hkv % n or Hq % n:
        raise ValueError(f"Ulysses attention needs the head counts ({Hq}/{Hkv}) divisible by cp={n}")
    hq, hk = Hq // n, Hkv // n
    dev = q.device
    # send: block j = heads of rank j for all local tokens, [n, T, heads/n, D]
    qkv = torch.cat([q.view(T, n, hq, D), k.view(T, n, hk, D), v.view(T, n, hk, D)], 2)   # [T, n, hq+2hk, D]
    recv_rows = [ctx.tokens(j) for j in range(n)]
    got = _a2a(qkv.transpose(0, 1).reshape(n * T, hq + 2 * hk, D), [T] * n, recv_rows, ctx)   # [sum T_j, ...]
    # reorder (source rank, sequence, chunk token) -> (sequence, position)
    nseq = len(ctx.lens[0])
    src_off = [sum(recv_rows[:j]) for j in range(n)]
    perm = []
    for i in range(nseq):
        for j in range(n):
            a = src_off[j] + sum(ctx.lens[j][:i])
            perm.extend(range(a, a + ctx.lens[j][i]))
    perm_t = torch.tensor(perm, dtype=torch.long, device=dev)
    full = got.index_select(0, perm_t)
    L = [sum(ctx.lens[j][i] for j in range(n)) for i in range(nseq)]
    cu = torch.tensor([0] + [sum(L[:i + 1]) for i in range(nseq)], dtype=torch.int32, device=dev)
    o = ops.attn_prefill(full[:, :hq], full[:, hq:hq + hk], full[:, hq + hk:], cu, max(L) if L else 0, scale, True)
    back = torch.empty_like(o)
    back[perm_t] = o                                                   # (source rank, seq, token) order
    ret = _a2a(back, recv_rows, [T] * n, ctx)                          # [n * T, hq, D]: head block j
    return ret.view(n, T, hq, D).transpose(0, 1).reshape(T, Hq, D)


def cp_prefill(model, prompts: list, ctx_ranks: list, rank_in_group: int, pg=None,
               kv_caches: Optional[list] = None, slots: Optional[list] = None,
               attn: str = "ring", sink_slots: Optional[list] = None, has_sink: bool = False,
               broadcast: bool = True) -> torch.Tensor:
    """Context-parallel prefill of `prompts` (token lists) by the CP group `ctx_ranks` (chunk
    order; group ranks of `pg`); this rank processes its chunk of every prompt. `slots[i]`
    (optional) are the paged-cache slots of THIS rank's chunk of prompt i in `kv_caches` (its
    local KV shard). `sink_slots[i]` (optional, the sink rank only; `has_sink` on every rank
    of such a step) are this rank's cache slots of EVERY token of prompt i: the whole prompt's
    K/V lands in its cache. `attn`: "ring" or "ulysses" (all-to-all; head counts divisible by
    cp). Returns the last-token logits [nseq, vocab_local] on every rank of the group
    (broadcast from the last rank), or, with broadcast=False, on the last rank only (others
    get an empty tensor)."""
    from ..engine.batch import ForwardBatch

    cp = len(ctx_ranks)
    per_seq = [split_lengths(len(p), cp) for p in prompts]
    lens = [[per_seq[i][r] for i in range(len(prompts))] for r in range(cp)]
    dev = model.device
    sink = None
    if sink_slots is not None:
        sink = []
        for r in range(cp):
            sl_r = []
            for i in range(len(prompts)):
                a = sum(per_seq[i][:r])
                sl_r.extend(sink_slots[i][a:a + per_seq[i][r]])
            sink.append(torch.tensor(sl_r, dtype=torch.int32, device=dev))
        slots = None
    elif has_sink:
        sink = []                 # marks a sink step on the other ranks (Ulysses gathers)
    ctx = CPContext(list(ctx_ranks), rank_in_group, pg, lens, attn, sink)
    ids, pos, sl = [], [], []
    for i, p in enumerate(prompts):
        a = sum(per_seq[i][:rank_in_group])
        n = per_seq[i][rank_in_group]
        ids.extend(p[a:a + n])
        pos.extend(range(a, a + n))
        if sink_slots is not None:
            sl.extend(sink_slots[i][a:a + n])
        else:
            sl.extend(slots[i] if slots is not None else [-1] * n)
    i32 = dict(dtype=torch.int32, device=dev)
    cu = ctx.cu(rank_in_group, dev)
    last = rank_in_group == cp - 1
    logits_idx = (cu[1:] - 1).to(torch.int64) if last else torch.zeros(0, dtype=torch.int64, device=dev)
    fb = ForwardBatch(input_ids=torch.tensor(ids, **i32), positions=torch.tensor(pos, **i32),
                      slots=torch.tensor(sl, **i32), is_prefill=True, cu_seqlens=cu,
                      max_seqlen=ctx.max_len(rank_in_group), logits_idx=logits_idx, cp=ctx)
    logits = model.forward(fb, kv_caches)
    if cp == 1 or not broadcast:
        return logits
    V = model.dims.vocab
    buf = logits.contiguous() if last else torch.empty(len(prompts), V, dtype=model.dtype, device=dev)
    if _nccl(pg):
        dist.broadcast(buf, ctx_ranks[-1], group=pg)
    else:
        host = buf.detach().cpu()
        dist.broadcast(host, ctx_ranks[-1], group=pg)
        buf = host.to(dev)
    return buf
