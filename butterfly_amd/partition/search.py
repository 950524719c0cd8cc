"""Partition search: choose (dp, tp, pp, ep) and pipeline cut points for N GPUs
(SURVEY.md §2.7 A8, §3.2 (2)).

For every factorisation dp * tp * pp = N that the model admits (tp divides the heads and is
compatible with the kv heads, pp <= layers, ep in {1, dp} for MoE):
  1. price one layer with the cost model at the replica's batch (decode) or tokens (prefill);
  2. cut the layers into pp contiguous stages with the C++ min-max dynamic program
     (runtime/partition_search.cpp), charging the embedding to stage 0, the LM head to the
     last stage and a boundary transfer to each cut, under the per-GPU memory capacity
     (weights + the stage's KV for its sequences);
  3. estimate the steady-state step: pp == 1 -> the stage time; pp > 1 -> the asynchronous
     pipeline's ticks (slowest stage x groups; engine/pipeline.py), or with BFLY_PP_ASYNC=0
     the per-step microbatched pipeline, slowest stage plus the fill/drain share;
  4. score: throughput = generated tokens / s for the node, latency = step time.
  5. link-aware selection (`select`): among plans within 2 % of the best objective, the
     fewest bytes on the busiest xGMI link per generated token (from the rank programs of
     schedule.py).
xGMI placement: a full mesh gives every GPU pair its own link, so no two logical edges
(ring all-reduce neighbours, pipeline neighbours) of different groups ever share a link and
every bijective placement has the same per-link loads; placement is therefore the identity,
and link traffic is minimised through the choice of layout (step 5) instead.
"""
from __future__ import annotations

from typing import Optional, Union

from .._native_loader import native
from ..config import ModelConfig
from ..models.shard import Shard, local_dims
from ..utils import flags
from .costmodel import CostModel
from .hw import MI355X, Hardware
from .plan import PartitionPlan


def factorizations(n: int) -> list[tuple[int, int, int]]:
    out = []
    for tp in range(1, n + 1):
        if n % tp:
            continue
        for pp in range(1, n // tp + 1):
            if (n // tp) % pp:
                continue
            out.append((n // (tp * pp), tp, pp))
    return out


def _tp_ok(cfg: ModelConfig, tp: int) -> bool:
    if cfg.num_heads % tp:
        return False
    if not (cfg.num_kv_heads % tp == 0 or tp % cfg.num_kv_heads == 0):
        return False
    return cfg.intermediate_size % (16 * tp) == 0


def evaluate(cfg: ModelConfig, dp: int, tp: int, pp: int, ep: int, *, batch_per_gpu: int,
             ctx: int, objective: str, hw: Hardware = MI355X, decode: bool = True,
             microbatches: Optional[int] = None) -> Optional[PartitionPlan]:
    n = dp * tp * pp
    cm = CostModel(cfg, hw)
    global_batch = batch_per_gpu * n
    B = max(1, global_batch // dp)                 # sequences per replica
    mb = microbatches or (pp if pp > 1 else 1)
    mb = max(1, min(mb, B))
    tokens = B // mb if decode else B * ctx // mb
    lcs = cm.layer_costs(tokens, tp, ctx, decode, seqs=max(1, B // mb), ep=ep)
    first_t, last_t = cm.embed_head_time(tokens, tokens if decode else max(1, B // mb), tp)
    emb_b, head_b = cm.embed_head_bytes(tp)
    kv_per_layer = 2.0 * max(1, cfg.num_kv_heads // tp) * cfg.head_dim * 2 * B * (ctx + 64)
    cap = hw.hbm_bytes * hw.usable_hbm_fraction - 4e9
    boundary = cm.p2p(2.0 * tokens * cfg.hidden_size) if pp > 1 else 0.0
    # min-max cut DP over the per-layer costs; the embedding is charged to stage 0 and the
    # final norm + LM head + sampling to the last stage, so the cuts shift layers off them
    cuts = native().pipeline_cuts([c.seconds for c in lcs], [c.weight_bytes + kv_per_layer for c in lcs], pp,
                                  first_t, emb_b, last_t, head_b, boundary, cap)
    if not cuts:
        return None
    stages = [(cuts[i], cuts[i + 1]) for i in range(pp)]
    stage_t = []
    for s, (a, b) in enumerate(stages):
        t = sum(c.seconds for c in lcs[a:b]) + (first_t if s == 0 else 0) + (last_t if s == pp - 1 else 0)
        if s != pp - 1:
            t += boundary
        stage_t.append(t)
    if pp == 1:
        step = stage_t[0]
        step_latency = step
    elif decode and ep == 1 and flags.get("BFLY_PP_ASYNC"):
        # asynchronous pipeline (engine/pipeline.py): mb = pp groups in flight, one tick per
        # group per stage, no fill/drain; a sequence gets a token every pp ticks
        step = max(stage_t) * mb
        step_latency = max(stage_t) * pp
    else:
        step = max(stage_t) * (mb + pp - 1) / mb * mb   # all microbatches through the pipe
        step_latency = sum(stage_t)
    tokens_per_step = global_batch if decode else global_batch * ctx
    tps = tokens_per_step / step
    weight_bytes, kv_budget = [], []
    for s, (a, b) in enumerate(stages):
        w = sum(c.weight_bytes for c in lcs[a:b]) + (emb_b if s == 0 else 0) + (head_b if s == pp - 1 else 0)
        weight_bytes.append(w)
        kv_budget.append(max(0.0, cap - w))
    plan = PartitionPlan(model=cfg, n_gpus=n, dp=dp, tp=tp, pp=pp, ep=ep, stages=stages,
                         placement=list(range(n)), objective=objective,
                         kv_budget_bytes=[kv_budget[(r // tp) % pp] for r in range(n)],
                         weight_bytes=[weight_bytes[(r // tp) % pp] for r in range(n)],
                         estimate={"step_seconds": step, "tokens_per_second": tps,
                                   "token_latency_seconds": step_latency,
                                   "batch_per_replica": B, "microbatches": mb,
                                   "stage_seconds": stage_t, "decode": decode, "ctx": ctx})
    plan.link_bytes_per_token = link_traffic(plan)
    plan.estimate["max_link_bytes_per_token"] = max(plan.link_bytes_per_token.values(), default=0.0)
    return plan


def link_traffic(plan: PartitionPlan) -> dict:
    """xGMI bytes per generated token on each directed GPU pair, from the plan's communication
    schedule (schedule.py: ring TP all-reduces incl. the embedding one, PP hops of the full
    residual stream between same-TP-index ranks, the sampling all-gather, the token broadcast)."""
    from .schedule import link_bytes, programs

    return link_bytes(plan, programs(plan, 1))


def partition(cfg: Union[ModelConfig, str], n_gpus: int, strategy: Union[str, dict] = "auto",
              objective: str = "throughput", batch_per_gpu: int = 64, ctx: int = 1024,
              hw: Hardware = MI355X, decode: bool = True, link_tolerance: float = 0.02) -> PartitionPlan:
    """The partitioning API: returns the best PartitionPlan for `n_gpus` GPUs.

    strategy: "auto" (search every factorisation), or a dict fixing some of
    {"dp", "tp", "pp", "ep"} (the rest are searched), e.g. {"tp": 2, "pp": 4}.
    objective: "throughput" (max node tokens/s) or "latency" (min per-token step time).
    Among plans within `link_tolerance` of the best objective, the one with the least traffic
    on its busiest xGMI link wins (`select`). `hw` may carry a measured communication table
    (parallel/probe.py; bench.py probes the node before partitioning).
    """
    if isinstance(cfg, str):
        cfg = ModelConfig.from_preset(cfg)
    fixed = {} if strategy == "auto" else dict(strategy)
    feasible = []
    for dp, tp, pp in factorizations(n_gpus):
        if any(fixed.get(k, v) != v for k, v in (("dp", dp), ("tp", tp), ("pp", pp))):
            continue
        if not _tp_ok(cfg, tp) or pp > cfg.num_layers:
            continue
        eps = [1]
        # expert parallelism spans the DP replicas (per pipeline stage when pp > 1: the
        # asynchronous pipeline keeps each stage's EP group in lockstep)
        if cfg.is_moe and dp > 1 and cfg.num_experts % dp == 0 and tp == 1:
            eps.append(dp)
        if "ep" in fixed:
            eps = [e for e in eps if e == fixed["ep"]]
        for ep in eps:
            try:
                local_dims(cfg, Shard(tp_size=tp, ep_size=ep))
            except ValueError:
                continue
            p = evaluate(cfg, dp, tp, pp, ep, batch_per_gpu=batch_per_gpu, ctx=ctx,
                         objective=objective, hw=hw, decode=decode)
            if p is not None:
                feasible.append(p)
    if not feasible:
        raise ValueError(f"no feasible partition of {cfg.name} on {n_gpus} GPUs with strategy {strategy}")
    best = select(feasible, objective, link_tolerance)
    best.validate()
    return best


def _score(p: PartitionPlan, objective: str) -> float:
    return p.estimate["tokens_per_second"] if objective == "throughput" else -p.estimate["token_latency_seconds"]


def select(plans: list, objective: str = "throughput", link_tolerance: float = 0.02) -> PartitionPlan:
    """Link-aware choice: among the plans whose objective is within `link_tolerance` of the
    best one, take the one that puts the fewest bytes on its busiest xGMI link per generated
    token (ties: the better objective). The cost model already charges collective and hop time
    to each step; this second criterion prefers the layout that leaves the links idle when the
    estimates are too close to call."""
    best = max(_score(p, objective) for p in plans)
    margin = abs(best) * link_tolerance
    close = [p for p in plans if _score(p, objective) >= best - margin]
    return min(close, key=lambda p: (p.estimate["max_link_bytes_per_token"], -_score(p, objective)))
