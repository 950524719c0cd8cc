"""Communication schedule: the per-rank program of one engine step, derived from a PartitionPlan
(SURVEY.md §2.7-A A11 "comm scheduler / rank program", §2.7-C collective call sites).

`rank_program(plan, rank, tokens)` lists, in issue order, what rank `rank` does in one decode
step (one request group of `tokens` sequences): compute blocks (stage layer ranges) and the
communication instructions between them, with group, peer and payload. It is the program the
engine runs — `engine/engine.py:_run_stages` / `_pipe_stage` (recv residual stream -> stage
-> isend, or sample + broadcast ids) and `models/transformer.py` (vocab-parallel embedding
all-reduce, two TP all-reduces per layer, EP fixed-capacity all-to-all dispatch and return,
vocab-parallel sampling all-gather; with the IPC EP exchange, dispatch and return of the
routed rows) — written down ahead of time so that it can be

  * checked for cross-rank consistency without running anything (`check_programs`: every
    group collective is issued by all members in the same order with the same payload, every
    send has its recv at the same position of the pair's stream), then executed against each
    other under blocking semantics by the native simulator (`simulate`,
    csrc/runtime/program_sim.h), which finds wait cycles ACROSS groups (a collective of one
    group waiting on a rank stuck in another group's) and names every blocked rank;
  * priced per xGMI link (`link_bytes`: bytes each directed GPU pair carries per step, ring
    all-reduce/all-gather/reduce-scatter, chain broadcast and point-to-point hops). The
    partitioner reports it per plan (`search.link_traffic`) and uses the busiest link's bytes
    to choose among layouts whose estimated throughput is within 2 % (`search.select`); the
    cut points themselves come from the time/memory DP;
  * compared with what the engine actually issued (tests/test_schedule.py replays a decode
    step through the loopback backend, parallel/fake.py, and diffs its log against this);
  * EXECUTED: the engine-level instructions (`exec`: recv / stage / send / sample / broadcast,
    per microbatch; `exec_program`) are what engine._execute interprets for every pipelined or
    single-stage step — the peers, streams and order of the boundary transfers come from here,
    not from code in the engine;
  * ENFORCED on the in-stage collectives (BFLY_PROGRAM_CHECK): every all-reduce / all-to-all /
    EP dispatch / return the model code issues in a decode step is checked against the next
    instruction of this program before it is issued (parallel/comm.Communicator.expect,
    engine._program_check), so a divergent rank raises instead of deadlocking its group.

Stream assignment follows the engine: TP all-reduces run on the compute stream (one-shot IPC
kernel when BFLY_CUSTOM_AR is active, else RCCL, both stream-ordered), PP sends are `isend` on
RCCL's stream (they overlap the next group's compute), the token broadcast ends the step.
With native RCCL pipeline edges (`native_pp=True`, parallel/rccl.pp_edges) the boundary receive
is the FIRST node of the stage's captured decode graph (stream "graph": it lands in the graph's
static input), and the send leaves the graph's static output on the communicator's send stream
(stream "send"); both move the whole graph bucket (`bucket` rows), which is what the engine
puts on the wire.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

from ..config import ModelConfig
from .plan import PartitionPlan

BF16 = 2


@dataclass(frozen=True)
class Instr:
    op: str                      # compute | all_reduce | all_gather | reduce_scatter | all_to_all | ep_dispatch |
                                 # ep_return | send | recv | broadcast
    group: tuple = ()            # global ranks taking part (send/recv: (src, dst))
    nbytes: int = 0              # payload this rank contributes (all_gather: its own slice)
    stream: str = "compute"      # compute | comm | graph | send
    note: str = ""
    exec: str = ""               # engine-level step: recv | stage | send | sample | broadcast ("" = issued
                                 # inside the stage's model forward / sampler, or before the step)
    mb: int = 0                  # microbatch the engine-level step belongs to

    def key(self) -> tuple:
        """What must agree between the members of a collective (or a send/recv pair)."""
        return (self.op if self.op not in ("send", "recv") else "p2p", self.group, self.nbytes)


@dataclass
class RankProgram:
    rank: int
    tokens: int
    instrs: list = field(default_factory=list)

    def comm(self) -> list:
        return [i for i in self.instrs if i.op != "compute"]

    def bytes_by_op(self) -> dict:
        out: dict = {}
        for i in self.comm():
            out[i.op] = out.get(i.op, 0) + i.nbytes
        return out

    def describe(self) -> str:
        lines = [f"rank {self.rank}: decode step, {self.tokens} tokens"]
        for i in self.instrs:
            if i.op == "compute":
                lines.append(f"  [compute] {i.note}")
            else:
                lines.append(f"  [{i.stream:7s}] {i.op:14s} {str(i.group):24s} {i.nbytes:>12,d} B  {i.note}")
        return "\n".join(lines)


def rank_program(plan: PartitionPlan, rank: int, tokens: int, microbatches: int = 1,
                 dtype_bytes: int = BF16, native_pp: bool = False, bucket: Optional[int] = None,
                 ep_ipc: bool = False) -> RankProgram:
    """The decode-step program of `rank` for `tokens` sequences. With the asynchronous pipeline
    (default) a step is one tick carrying one request group (`tokens` = the group's size, one
    microbatch); the synchronous pipeline (engine._pipeline_decode) cuts the step's batch into
    `microbatches` parts that flow through the stages back to back, then broadcasts all ids."""
    # (EP x PP: each stage's MoE collectives run on that stage's EP group, the stage's ranks of
    # every replica; the asynchronous pipeline keeps them in lockstep, one microbatch per tick)
    if plan.mesh.ep > 1 and plan.mesh.pp > 1 and microbatches > 1:
        raise ValueError("expert parallelism with pipeline stages runs one microbatch per tick")
    prog = RankProgram(rank, tokens)
    M = max(1, min(microbatches, tokens))
    bounds = [tokens * i // M for i in range(M + 1)]
    for m in range(M):
        _microbatch(plan, rank, bounds[m + 1] - bounds[m], prog.instrs.append, ep_sync=(m == 0),
                    dtype_bytes=dtype_bytes, native_pp=native_pp, bucket=bucket, ep_ipc=ep_ipc, mb=m)
    if plan.mesh.pp > 1:
        prog.instrs.append(Instr("broadcast", tuple(plan.mesh.pp_group(rank)), tokens * 4, "comm",
                                 "sampled ids from the last stage", exec="broadcast"))
    return prog


def exec_program(plan: PartitionPlan, rank: int, microbatches: int = 1, native_pp: bool = False) -> list:
    """The engine-level steps of `rank`'s program (instructions with `exec` set), in issue order:
    what engine._execute runs for a step of `microbatches` microbatches. They do not depend on
    the token count (only the payloads do), so the engine builds them once per shape."""
    prog = rank_program(plan, rank, max(1, microbatches), max(1, microbatches), native_pp=native_pp)
    return [i for i in prog.instrs if i.exec]


def _microbatch(plan: PartitionPlan, rank: int, tokens: int, add, ep_sync: bool, dtype_bytes: int = BF16,
                native_pp: bool = False, bucket: Optional[int] = None, ep_ipc: bool = False, mb: int = 0) -> None:
    cfg: ModelConfig = plan.model
    mesh = plan.mesh
    c = mesh.coord(rank)
    tp_g = tuple(mesh.tp_group(rank))
    tp, pp, ep = mesh.tp, mesh.pp, mesh.ep
    a, b = plan.stages[c.pp]
    first, last = c.pp == 0, c.pp == pp - 1
    h = cfg.hidden_size
    act = tokens * h * dtype_bytes
    R = tokens
    moe = cfg.is_moe
    ep_g = tuple(next(g for g in mesh.all_groups("ep") if rank in g)) if ep > 1 else ()
    if ep > 1 and ep_sync:
        # all EP ranks agree on the padded row count, on prefill vs decode and on idling
        add(Instr("max_int", ep_g, 3 * 8, "compute", "EP step agreement (rows, prefill?, work?)"))
    if not first and native_pp:
        wire = (bucket or tokens) * h * dtype_bytes
        add(Instr("recv", (mesh.prev_stage(rank), rank), wire, "graph",
                  "residual stream from previous stage: first node of the captured decode graph",
                  exec="recv", mb=mb))
    elif not first:
        add(Instr("recv", (mesh.prev_stage(rank), rank), act, "comm", "residual stream from previous stage",
                  exec="recv", mb=mb))
    # the stage's model forward: every instruction up to the send / sampling is issued inside it
    add(Instr("compute", note=f"stage: layers {a}..{b - 1}", exec="stage", mb=mb))
    if first:
        add(Instr("compute", note="embedding gather (vocab shard)"))
        if tp > 1:
            add(Instr("all_reduce", tp_g, act, "compute", "vocab-parallel embedding"))
    for layer in range(a, b):
        add(Instr("compute", note=f"layer {layer}: norm, QKV, RoPE+KV append, attention, O"))
        if tp > 1:
            add(Instr("all_reduce", tp_g, act, "compute", f"layer {layer} attention output (+ add, RMSNorm)"))
        if moe and ep > 1 and ep_ipc:
            # byte-minimal IPC exchange (parallel/ep_ipc.py): each token row travels once to
            # each rank owning one of its experts, and its output once back. The bytes depend
            # on the routing: the payload here is the bound, min(k, ep) ranks per token.
            k = cfg.experts_per_token
            hits = tokens * min(k, ep)
            add(Instr("compute", note=f"layer {layer}: router"))
            add(Instr("ep_dispatch", ep_g, hits * (h * dtype_bytes + 8 * k), "compute",
                      f"layer {layer} EP: routed rows + expert ids / weights into the owners' IPC blocks"))
            add(Instr("compute", note=f"layer {layer}: local experts on routed rows only"))
            add(Instr("ep_return", ep_g, hits * h * dtype_bytes, "compute",
                      f"layer {layer} EP: routed rows' expert outputs back into the sources' IPC blocks"))
        elif moe and ep > 1:
            # fixed-capacity dispatch (models/transformer.py _moe_alltoall_fixed): `tokens`
            # rows reserved per destination, expert ids + gate weights (f32) alongside
            k = cfg.experts_per_token
            add(Instr("compute", note=f"layer {layer}: router, pack rows per destination rank"))
            add(Instr("all_to_all", ep_g, ep * act, "compute", f"layer {layer} EP: token rows to expert owners"))
            add(Instr("all_to_all", ep_g, ep * tokens * 2 * k * 4, "compute",
                      f"layer {layer} EP: expert ids + gate weights"))
            add(Instr("compute", note=f"layer {layer}: local experts on routed rows only"))
            add(Instr("all_to_all", ep_g, ep * act, "compute", f"layer {layer} EP: weighted expert outputs back"))
        else:
            add(Instr("compute", note=f"layer {layer}: " + ("router + experts" if moe else "gate/up, SiLU, down")))
            if tp > 1:
                # fused with the next layer's add+RMSNorm; after a stage's last layer it is a
                # plain all-reduce (last stage: only the sampled rows are reduced)
                nb = R * h * dtype_bytes if (last and layer == b - 1) else act
                add(Instr("all_reduce", tp_g, nb, "compute", f"layer {layer} FFN output"))
    if last:
        add(Instr("compute", note="final norm, LM head (vocab shard) in the stage; sampling", exec="sample", mb=mb))
        if tp > 1:
            add(Instr("all_gather", tp_g, R * 2 * 4, "compute", "vocab-parallel argmax: (score, id) pairs"))
    elif native_pp:
        wire = (bucket or tokens) * h * dtype_bytes
        add(Instr("send", (rank, mesh.next_stage(rank)), wire, "send",
                  "residual stream to next stage: the graph's static output (A/B instance), send stream",
                  exec="send", mb=mb))
    else:
        add(Instr("send", (rank, mesh.next_stage(rank)), act, "comm", "residual stream to next stage",
                  exec="send", mb=mb))


def check_programs(progs: dict) -> None:
    """Raise ValueError unless the programs of all ranks are mutually consistent: for every group
    the members issue the same sequence of collectives (op, payload), and every (src, dst) pair
    sees its sends and recvs in the same order with the same payloads."""
    by_group: dict = {}
    for r, p in progs.items():
        for i in p.comm():
            if i.op in ("send", "recv"):
                by_group.setdefault(("p2p",) + i.group, {}).setdefault(r, []).append(i.nbytes)
            else:
                by_group.setdefault(i.group, {}).setdefault(r, []).append((i.op, i.nbytes))
    for g, seqs in by_group.items():
        if g and g[0] == "p2p":
            src, dst = g[1], g[2]
            if seqs.get(src) != seqs.get(dst):
                raise ValueError(f"p2p {src}->{dst}: sends {seqs.get(src)} vs recvs {seqs.get(dst)}")
            continue
        members = set(g)
        if set(seqs) != members:
            raise ValueError(f"group {g}: only ranks {sorted(seqs)} issue collectives")
        ref = seqs[min(seqs)]
        for r, s in seqs.items():
            if s != ref:
                raise ValueError(f"group {g}: rank {r} issues {s[:4]}... vs {ref[:4]}...")
    # consistent per group and per pair; now run them against each other (cross-group cycles)
    sim = simulate(progs)
    if not sim["ok"]:
        raise ValueError(f"programs deadlock: {sim['error'] or ''} blocked {sim['blocked'][:8]}")


def simulate(progs: dict, rendezvous: bool = False) -> dict:
    """Run every rank's communication program against the others under blocking semantics
    (native runtime, csrc/runtime/program_sim.h): collectives meet all members, recvs wait for
    their message, sends are buffered (`rendezvous`: block until the receiver is at the
    matching recv, except side-stream sends). Finds wait cycles ACROSS groups, which the
    per-group sequence comparison of `check_programs` cannot see. Returns {ok, error,
    blocked: [(rank, index, instruction)], completed}."""
    from .. import _native_loader

    native = _native_loader.native()
    n = max(progs) + 1
    flat = [[(i.op, list(i.group), int(i.nbytes), i.stream) for i in progs[r].comm()] if r in progs else []
            for r in range(n)]
    return native.simulate_programs(flat, rendezvous)


def link_bytes(plan: PartitionPlan, progs: dict) -> dict:
    """Bytes per directed GPU pair for one step. Ring collectives over a group of n move
    2(n-1)/n of the payload (all-reduce) or (n-1)/n of the gathered tensor (all-gather /
    reduce-scatter) through each member's link to its ring successor; p2p goes direct."""
    out: dict = {}
    place = plan.placement

    def put(src, dst, nb):
        k = f"{place[src]}-{place[dst]}"
        out[k] = out.get(k, 0.0) + nb

    for r, p in progs.items():
        for i in p.comm():
            n = len(i.group)
            if i.op == "send":
                put(i.group[0], i.group[1], i.nbytes)
            elif i.op in ("all_to_all", "ep_dispatch", "ep_return") and n > 1:
                me = i.group.index(r)
                for j, peer in enumerate(i.group):      # direct: block j to member j
                    if j != me:
                        put(r, peer, i.nbytes / n)
            elif i.op in ("all_reduce", "all_gather", "reduce_scatter", "broadcast") and n > 1:
                nxt = i.group[(i.group.index(r) + 1) % n]
                if i.op == "all_reduce":
                    put(r, nxt, 2.0 * (n - 1) / n * i.nbytes)
                elif i.op == "all_gather":
                    put(r, nxt, (n - 1) * i.nbytes)
                elif i.op == "reduce_scatter":
                    put(r, nxt, (n - 1) / n * i.nbytes)
                elif i.group.index(r) == n - 1:
                    # broadcast from the last member as a chain: root -> successor -> ... ,
                    # n-1 hops of the full payload
                    hop = i.group.index(r)
                    for _ in range(n - 1):
                        a_, b_ = i.group[hop], i.group[(hop + 1) % n]
                        put(a_, b_, i.nbytes)
                        hop = (hop + 1) % n
    return out


def programs(plan: PartitionPlan, tokens: int, microbatches: int = 1, dtype_bytes: int = BF16,
             native_pp: bool = False, bucket: Optional[int] = None, ep_ipc: bool = False) -> dict:
    """rank_program for every rank (each DP replica decodes `tokens` sequences); activations
    are `dtype_bytes` wide (bf16 on the GPU, fp32 on the CPU reference path)."""
    return {r: rank_program(plan, r, tokens, microbatches, dtype_bytes, native_pp, bucket, ep_ipc)
            for r in range(plan.n_gpus)}
