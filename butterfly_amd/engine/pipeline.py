"""Asynchronous pipeline-parallel decode: `pp` request groups in flight across engine steps.

Per-step microbatching (engine._pipeline_decode) pays a fill/drain bubble every step — with
M = pp microbatches a step lasts (M + pp - 1) stage-slots for M slots of work, and every
microbatch re-streams the stage's weights from HBM. Here the replica's sequences are split
into `pp` groups, each with its own continuous-batching scheduler over the shared KV block
manager, and the engine advances in ticks: at tick k group (k mod pp) enters stage 0 while
stage s works on the group that entered at tick k - s. In steady state every stage streams
its weights once per tick for one group, and one group's tokens leave the last stage per tick
— no bubble, and the same RCCL send/recv of the residual stream between neighbouring stages
(SURVEY.md §2.6 PP row, §3.2 (4) "PP steady-state loop").

Determinism across ranks: every rank of the replica runs the same tick loop, schedules the
entering group itself (the schedulers are replicated, as in the synchronous engine), receives
the sampled ids of the group leaving the last stage by a broadcast over the pp group, and
advances its scheduler by one token per sequence at the start of the next tick — exactly when
that group is scheduled again (it entered pp ticks earlier). The token VALUES are not needed
for that: stage 0 gathers the group's new input ids from the broadcast tensor on the device,
and the host reads the values (copied asynchronously to pinned memory) one tick later, so no
tick waits on the device (engine._pp_tick). A group's block tables, positions and tokens
only change at its own scheduling / completion, so a plan made at tick k stays valid while
stages 1..pp-1 process it at ticks k+1..k+pp-1.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional


class GroupedScheduler:
    """`groups` replicated C++ schedulers (runtime/scheduler.cpp) sharing one KV block manager;
    new requests go to the least-loaded group (deterministic: ties -> lowest index). `mixed`:
    every group runs the scheduler's mixed mode (its decode rows and prompt chunks in one plan,
    long prompts prefilled over several ticks), with automatic prefix caching over the shared
    block manager when `prefix_cache`."""

    def __init__(self, native, kv_manager, groups: int, max_batch: int, max_prefill_tokens: int,
                 mixed: bool = False, prefix_cache: bool = False):
        self.group_batch = max(1, -(-max_batch // groups))
        self.mixed, self.prefix_cache = mixed, mixed and prefix_cache
        self.groups = [native.Scheduler(kv_manager, self.group_batch, max_prefill_tokens, mixed, self.prefix_cache)
                       for _ in range(groups)]
        self.owner: dict[int, int] = {}

    def add(self, rid: int, prompt_len: int, max_new: int, tokens: Optional[list] = None) -> None:
        g = self._least_loaded()
        if self.prefix_cache and tokens is not None:
            self.groups[g].add(rid, prompt_len, max_new, tokens)
        else:
            self.groups[g].add(rid, prompt_len, max_new)
        self.owner[rid] = g

    def _least_loaded(self) -> int:
        return min(range(len(self.groups)),
                   key=lambda i: (self.groups[i].num_running + self.groups[i].num_waiting, i))

    def can_admit_prefilled(self, prompt_len: int) -> bool:
        """A context-parallel prefill (engine._cp_step) can hand its sequence to the group that
        would take it now (the least-loaded one)."""
        return bool(self.groups[self._least_loaded()].can_admit_prefilled(prompt_len))

    def admit_prefilled(self, rid: int, prompt_len: int, max_new: int) -> list:
        """Admit a sequence whose prompt K/V is already cached (context-parallel prefill):
        it joins the least-loaded group as a running sequence; returns its cache slots."""
        g = self._least_loaded()
        slots = self.groups[g].admit_prefilled(rid, prompt_len, max_new)
        if slots:
            self.owner[rid] = g
        return slots

    @property
    def prefix_hit_tokens(self) -> int:
        return sum(g.prefix_hit_tokens for g in self.groups)

    def on_token(self, rid: int) -> None:
        self.groups[self.owner[rid]].on_token(rid)

    def finish(self, rid: int) -> None:
        self.groups[self.owner.pop(rid)].finish(rid)

    @property
    def num_waiting(self) -> int:
        return sum(g.num_waiting for g in self.groups)

    @property
    def num_running(self) -> int:
        return sum(g.num_running for g in self.groups)

    def running(self) -> list:
        return [r for g in self.groups for r in g.running()]

    def waiting(self) -> list:
        return [r for g in self.groups for r in g.waiting()]


@dataclass
class PipePlan:
    """One group's step plan travelling through the stages."""
    tick: int                 # tick at which it entered stage 0
    group: int
    plan: object              # native StepPlan (kind 1 prefill / 2 decode / 3 mixed)
    rids: list                # sequences whose row is sampled (mixed: decode rows and prompts
                              # whose final chunk this plan runs), in logits-row order
    tokens: int               # rows of the residual stream between stages
    cow: list = field(default_factory=list)
    seqs: list = field(default_factory=list)   # every sequence with a row in the plan
    ep_pad: int = 0           # expert parallelism: rows every EP rank pads this step to
    ep_prefill: bool = False  # some EP rank prefills this step (variable exchange, no graphs)
    idle: bool = False        # EP x PP: an empty plan that only joins its peers' MoE exchanges
    ids: Optional[object] = None   # sampled ids tensor (last stage / after broadcast)
    host: Optional[object] = None  # pinned host copy of `ids` (async D2H at broadcast time)
    event: Optional[object] = None # marks that copy complete

    @property
    def kind(self) -> str:
        if self.idle:
            return "ep-idle"
        return {1: "prefill", 3: "mixed"}.get(self.plan.kind, "decode")
