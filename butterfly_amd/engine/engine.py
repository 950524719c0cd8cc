"""LLMEngine: the distributed inference engine ("Core logic for splitting transformer
computations across nodes", /root/reference/CLAUDE.md:19) for one rank.

Every rank of a model replica (its TP x PP ranks) runs an identical engine: the same requests,
the same deterministic C++ scheduler (runtime/scheduler.cpp) and therefore the same step
plans, so no scheduling messages are exchanged. Data-parallel replicas run independent engines
on their own request streams.

Per step:
  prefill  : pack the admitted prompts, run the stage (flash prefill), sample the first tokens
  decode   : one token per running sequence through the hipGraph-replayed stage
  PP       : stage s receives the residual stream from s-1 and sends to s+1 (RCCL send/recv
             over xGMI); the last stage samples and broadcasts token ids to the replica's
             ranks. Default (BFLY_PP_ASYNC): pp request groups stay in flight across steps,
             one step = one tick in which every stage advances one group (engine/pipeline.py);
             otherwise each step splits the batch into microbatches (fill/drain per step).
  TP       : handled inside the model (all-reduces) and the sampler (score/id all-gather).
  CP       : (EngineConfig.cp_prefill_min_tokens, pp == 1, no EP) a long prompt is prefilled
             by every data-parallel replica together, context-parallel (ring / Ulysses), and
             its K/V lands in the cache of the replica that decodes it (`_cp_step`). The
             replicas then agree once per step on whether such a prefill is due, so they
             step in lockstep (`lockstep_dp`, `has_unfinished_global`).
"""
from __future__ import annotations

import itertools
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..config import EngineConfig, ModelConfig
from ..models import Shard, build_model
from ..parallel.comm import Communicator, NativeWork
from ..parallel.mesh import Mesh
from ..partition.plan import PartitionPlan
from ..partition.schedule import exec_program
from ..utils import flags, trace
from ..utils.health import FaultInjector, StepWatchdog
from ..utils.metrics import Metrics
from .batch import empty_batch
from .kv_cache import KVCache, device_kv_budget, kv_blocks_for_budget
from .model_runner import ModelRunner
from .pipeline import GroupedScheduler, PipePlan
from . import state
from .sampler import Sampler, SamplingParams


@dataclass
class Request:
    rid: int
    prompt: list
    params: SamplingParams
    output: list = field(default_factory=list)
    arrival: float = 0.0
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    finished: bool = False
    finish_reason: Optional[str] = None
    n_gen: int = 0                # tokens generated, including ones whose value is still in flight
    stopping: bool = False        # stop token seen while a plan holding the sequence is in flight
    sched_done: bool = False      # released from the scheduler

    @property
    def tokens(self) -> list:
        return self.prompt + self.output


@dataclass
class StepOutput:
    kind: str
    rids: list
    new_tokens: list
    finished: list
    seconds: float
    prefill_tokens: int = 0       # prompt tokens this step put through the model


class LLMEngine:
    def __init__(self, cfg: ModelConfig, mesh: Mesh = Mesh(), engine_cfg: EngineConfig = EngineConfig(),
                 comm: Optional[Communicator] = None, device=None, stage_layers: Optional[list] = None,
                 model=None, eos_token_id: Optional[int] = None):
        self.cfg = cfg
        self.ecfg = engine_cfg
        self.mesh = mesh
        self.comm = comm or Communicator.single()
        self.rank = self.comm.rank
        coord = mesh.coord(self.rank)
        self.coord = coord
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        if stage_layers is None:
            stage_layers = balanced_stages(cfg.num_layers, mesh.pp)
        if mesh.ep > 1 and mesh.pp > 1 and not flags.get("BFLY_PP_ASYNC"):
            # EP x PP: each stage's MoE layers exchange tokens with that stage's ranks of the
            # other replicas; only the asynchronous pipeline keeps those EP groups in lockstep
            # (every replica's plan of tick k reaches stage s at tick k + s, idle plans included)
            raise ValueError("expert parallelism with pipeline stages needs the asynchronous pipeline "
                             "(BFLY_PP_ASYNC=1)")
        # the rank's step program (partition/schedule.py) drives the stage execution below:
        # boundary receives / sends, stage runs, sampling and the id broadcast, with their peers
        self.plan = PartitionPlan(model=cfg, n_gpus=mesh.world_size, dp=mesh.dp, tp=mesh.tp, pp=mesh.pp,
                                  ep=mesh.ep, stages=[tuple(x) for x in stage_layers],
                                  placement=list(range(mesh.world_size)))
        self._exec_ops: dict = {}
        if mesh.world_size > 1:
            # every rank's program of a step, run against the others before anything is issued
            # (csrc/runtime/program_sim.h): a cross-group wait cycle or a mismatched collective
            # fails here, naming the ranks, instead of hanging the first step
            from ..partition.schedule import check_programs, programs

            for mb in sorted({1, mesh.pp} if mesh.ep == 1 else {1}):   # (EP x PP: async only)
                check_programs(programs(self.plan, max(1, engine_cfg.max_batch), microbatches=mb))
        a, b = stage_layers[coord.pp]
        shard = Shard(tp_rank=coord.tp, tp_size=mesh.tp, layer_start=a, layer_end=b,
                      ep_rank=coord.dp if mesh.ep > 1 else 0, ep_size=mesh.ep)
        dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.model = model or build_model(cfg, shard, device=self.device, dtype=dtype, comm=self.comm)
        if model is None:
            self.model.init_random(engine_cfg.seed)
        self.eos = eos_token_id
        # ---- KV cache sizing ------------------------------------------------------------
        bs = engine_cfg.block_size
        self.kv_dtype = kv_cache_dtype(engine_cfg.kv_cache_dtype, self.model.dtype)
        per_tok = self.model.kv_bytes_per_token(self.kv_dtype)
        if engine_cfg.kv_cache_tokens:
            nblocks = (engine_cfg.kv_cache_tokens + bs - 1) // bs
        else:
            act_reserve = self._activation_reserve()
            budget = device_kv_budget(self.device, engine_cfg.hbm_utilization, act_reserve)
            nblocks = kv_blocks_for_budget(budget, per_tok, bs)
            need = engine_cfg.max_batch * ((engine_cfg.max_seq_len + bs - 1) // bs)
            nblocks = min(nblocks, max(need, 1))
        if nblocks <= 0:
            raise RuntimeError("no HBM left for the KV cache")
        if (self.device.type == "cuda" and flags.get("BFLY_PACKED_DECODE") and mesh.ep == 1
                and engine_cfg.max_batch <= 512):
            # decode-layout copies of the projection weights, only from HBM the KV cache leaves free
            free = device_kv_budget(self.device, engine_cfg.hbm_utilization, self._activation_reserve())
            room = free - nblocks * per_tok * bs - (2 << 30)
            if room > 0:
                kinds = [k.strip() for k in flags.get("BFLY_PACKED_KINDS").split(",") if k.strip()]
                self.model.pack_decode_weights(budget_bytes=room, kinds=kinds)
        self.kv = KVCache(self.model, nblocks, bs, self.kv_dtype)
        native = __import__("butterfly_amd._native_loader", fromlist=["native"]).native()
        # pipeline parallelism without per-step fill/drain: pp request groups in flight
        # (engine/pipeline.py); EP layouts keep the synchronous path (EP collectives span DP ranks)
        # (pp == 1 with EngineConfig.async_decode: the same machinery with one group overlaps
        # the host's scheduling of step k+1 with the device's step k)
        # (EP layouts, pp == 1, too: the EP ranks agree on padding / step mode over the gloo
        # control plane, which never waits for the device)
        # (context-parallel prefill over the DP replicas, pp == 1, runs inside the asynchronous
        # engine too: a tick that runs one is a CP tick, _pp_tick)
        self.async_pp = flags.get("BFLY_PP_ASYNC") and (mesh.pp > 1 or bool(engine_cfg.async_decode))
        # mixed steps (chunked prefill riding along decode rows, prefix caching): every layout;
        # in the asynchronous pipeline each group's plans are mixed. Expert-parallel replicas
        # agree per step on the padded row count and on whether any of them runs prompt rows
        # (which switches every peer's MoE layer to the variable exchange): _ep_agree
        self.mixed = bool(engine_cfg.mixed_prefill) and (mesh.pp == 1 or self.async_pp)
        self.prefix_cache = self.mixed and bool(engine_cfg.prefix_caching)
        if self.async_pp:
            self.scheduler = GroupedScheduler(native, self.kv.manager, mesh.pp, engine_cfg.max_batch,
                                              engine_cfg.max_prefill_tokens, self.mixed, self.prefix_cache)
        else:
            self.scheduler = native.Scheduler(self.kv.manager, engine_cfg.max_batch, engine_cfg.max_prefill_tokens,
                                              self.mixed, self.prefix_cache)
        self._tick = 0
        self._inflight: list = []        # PipePlans entered at ticks k-pp+1 .. k
        self._pending: Optional[PipePlan] = None   # left the last stage at the previous tick
        self._valued: Optional[PipePlan] = None    # advanced; token values applied next tick
        self._last_left: dict = {}                  # group -> its plan that left most recently
        self._sends: list = []
        # boundary activations of the async pipeline (overlap executor): the
        # receive of the group arriving next tick is posted at the end of this tick on a
        # dedicated comm stream, into one of two persistent buffers; the compute stream waits
        # on it only when that group's stage work starts, and a buffer is re-posted only after
        # an event marks the compute that read it
        self._prepost = bool(self.async_pp and coord.pp > 0 and flags.get("BFLY_PP_PREPOST")
                             and self.comm.prepost_ok())
        self._posted: dict = {}           # plan tick -> (buffer view, work, slot)
        self._bbufs: list = []
        self._bslot = 0
        self._bevents: list = [None, None]
        # native RCCL pipeline edges: a non-first stage's decode graph receives the boundary
        # rows itself (model_runner.set_pipeline_io) and stages send their graphs' static
        # outputs on the communicator's send stream — no pre-posted buffers, no copies
        self._native_pp = bool(self.async_pp and mesh.pp > 1 and getattr(self.comm, "native_p2p", False))
        if self._native_pp:
            self._prepost = False
        self._comm_stream = (torch.cuda.Stream(self.device)
                             if self._prepost and self.device.type == "cuda" else None)
        d = self.model.dims
        self.sampler = Sampler(self.comm, cfg.vocab_size, d.vocab0, mesh.tp)
        if self.device.type == "cuda":
            ops.reserve_workspace(self.device, max_tokens=max(engine_cfg.max_prefill_tokens, engine_cfg.max_batch),
                                  max_n=self._max_gemm_n(), max_k=self._max_gemm_k(),
                                  max_batch=max(engine_cfg.graph_batch_sizes + [engine_cfg.max_batch]),
                                  max_ctx=engine_cfg.max_seq_len, num_kv_heads=d.hkv, head_dim=cfg.head_dim,
                                  shapes=self.model.gemm_shapes())
        buckets = [b for b in engine_cfg.graph_batch_sizes if b <= engine_cfg.max_batch] or [engine_cfg.max_batch]
        if self.async_pp and self.scheduler.group_batch not in buckets:
            buckets.append(self.scheduler.group_batch)    # a full group replays one graph
        self.runner = ModelRunner(self.model, self.kv, engine_cfg.max_seq_len, engine_cfg.use_graphs,
                                  buckets, max_batch=engine_cfg.max_batch)
        if self.async_pp and flags.get("BFLY_GRAPH_SAMPLING") and self.comm.capturable("tp"):
            # the last stage's decode graphs end with the sampler on per-request temperatures /
            # seeds staged with the other inputs: one replay per step yields the tokens
            # (top-k / top-p rows and poisoned steps sample eagerly from the graph's logits).
            # Only the asynchronous engine reads the graph's ids (_pp_stage_work); the
            # synchronous paths sample eagerly, so their graphs carry no sampler (TP merge:
            # an all-gather, capturable only on a capturable TP group)
            check = bool(flags.get("BFLY_NAN_CHECK"))
            self.runner.sample_fn = lambda lg, t, sd: self.sampler.sample(lg, t, sd, None, check_finite=check)
        # byte-minimal EP dispatch for the decode MoE layer (collective over the EP group, so
        # every EP rank sets it up here, eagerly, before any graph capture)
        self.ep_ipc = self.ep_ipc_prefill = False
        if mesh.ep > 1 and cfg.is_moe and flags.get("BFLY_EP_IPC"):
            self.ep_ipc = self.comm.enable_ep_ipc(max(self.runner.buckets[-1], engine_cfg.max_batch),
                                                  cfg.hidden_size, cfg.experts_per_token)
            if flags.get("BFLY_EP_IPC_PREFILL"):
                # prefill steps (and decode steps beside an EP peer's prefill): the same exchange
                # sized for the prefill budget, bounded by device-resident counts (no host sync)
                self.ep_ipc_prefill = self.comm.enable_ep_ipc_prefill(
                    max(engine_cfg.max_prefill_tokens, engine_cfg.max_batch, self.runner.buckets[-1]),
                    cfg.hidden_size, cfg.experts_per_token)
        if self._native_pp:
            self.runner.set_pipeline_io(recv_fn=None if coord.pp == 0 else self.comm.recv_native,
                                        sends=coord.pp < mesh.pp - 1)
        if flags.get("BFLY_PROGRAM_CHECK") and mesh.world_size > 1:
            self.runner.conform = self._program_check()
        if self.runner.use_graphs and not self.comm.graph_safe():
            # a data-path collective on gloo (ranks sharing one GPU) cannot be captured: decode
            # eagerly instead of attempting (and invalidating) a capture
            self.runner.use_graphs = False
        self.requests: dict[int, Request] = {}
        self._ids = itertools.count()
        self.metrics = Metrics()
        self.pp_first = coord.pp == 0
        self.pp_last = coord.pp == mesh.pp - 1
        self.faults = FaultInjector()
        self._poison = False
        self.nan_check = flags.get("BFLY_NAN_CHECK")
        # a step that outlives BFLY_STEP_TIMEOUT_S (hung collective, wedged GPU) dumps every
        # thread's stack and terminates the rank (0 = off; first steps include graph capture)
        st = flags.get("BFLY_STEP_TIMEOUT_S")
        self.watchdog = StepWatchdog(st) if st > 0 else None
        self.steps_done = 0
        # context-parallel prefill of long prompts over the DP replicas (parallel/context_parallel.py)
        self.cp_min = engine_cfg.cp_prefill_min_tokens if (
            mesh.dp > 1 and mesh.pp == 1 and mesh.ep == 1) else 0
        self._cp_queue: deque = deque()

    @property
    def lockstep_dp(self) -> bool:
        """Every step is collective over the data-parallel group (EP MoE layers, CP prefill
        agreement): the replicas must keep stepping until ALL of them are done."""
        return self.mesh.ep > 1 or bool(self.cp_min)

    def has_unfinished_global(self) -> bool:
        """has_unfinished() of this replica, or of any replica when steps are collective."""
        mine = int(self.has_unfinished())
        if not self.lockstep_dp:
            return bool(mine)
        return bool(self.comm.all_reduce_max_int([mine], "dp")[0])

    # ------------------------------------------------------------------------------------
    def _activation_reserve(self) -> int:
        e, c = self.ecfg, self.cfg
        T = max(e.max_prefill_tokens, e.max_batch)
        h = c.hidden_size
        d = self.model.dims
        width = max(3 * h, (d.hq + 2 * d.hkv) * c.head_dim, 2 * d.ffn * max(1, d.experts), d.vocab)
        return int(T * width * 2 * 6) + (2 << 30)

    def _max_gemm_n(self) -> int:
        c, d = self.cfg, self.model.dims
        return max((d.hq + 2 * d.hkv) * c.head_dim, c.hidden_size, 2 * d.ffn * max(1, d.experts), d.vocab)

    def _max_gemm_k(self) -> int:
        c, d = self.cfg, self.model.dims
        return max(c.hidden_size, d.ffn * max(1, d.experts), d.hq * c.head_dim)

    # ------------------------------------------------------------------------------------
    def precapture_decode(self, rows: int) -> bool:
        """Capture the decode graph for `rows` concurrent sequences now (ModelRunner.precapture)
        instead of inside the first decode step; every rank of the model group calls it."""
        return self.device.type == "cuda" and self.runner.precapture(rows)

    def add_request(self, prompt: list, params: Optional[SamplingParams] = None, rid: Optional[int] = None) -> int:
        rid = next(self._ids) if rid is None else rid
        params = params or SamplingParams()
        if len(prompt) + params.max_tokens > self.ecfg.max_seq_len:
            raise ValueError(f"prompt ({len(prompt)}) + max_tokens ({params.max_tokens}) exceeds max_seq_len")
        self.requests[rid] = Request(rid, list(prompt), params, arrival=time.perf_counter())
        if self.cp_min and len(prompt) >= self.cp_min:
            self._cp_queue.append(rid)        # prefilled by the DP group together (_cp_step)
        elif self.prefix_cache:
            self.scheduler.add(rid, len(prompt), params.max_tokens, list(prompt))
        else:
            self.scheduler.add(rid, len(prompt), params.max_tokens)
        return rid

    def _admit_resumed(self, req: Request) -> None:
        """Scheduler admission of a restored request (engine/state.py): its prompt plus the
        tokens it already generated are prefilled as one sequence, the rest is generated."""
        toks = req.tokens
        remaining = req.params.max_tokens - len(req.output)
        if len(toks) + remaining > self.ecfg.max_seq_len:
            raise ValueError(f"restored request {req.rid} exceeds max_seq_len")
        if self.prefix_cache:
            self.scheduler.add(req.rid, len(toks), remaining, list(toks))
        else:
            self.scheduler.add(req.rid, len(toks), remaining)

    def reset_ids(self, next_id: int) -> None:
        self._ids = itertools.count(next_id)

    # request-state snapshots (engine/state.py)
    def snapshot(self) -> dict:
        return state.snapshot(self)

    def restore(self, snap: dict) -> list:
        return state.restore(self, snap)

    def save_state(self, path) -> None:
        state.save(self, path)

    def has_unfinished(self) -> bool:
        return (self.scheduler.num_waiting + self.scheduler.num_running > 0 or bool(self._cp_queue)
                or self._pending is not None or self._valued is not None)

    def _sample_params(self, rids):
        temps = [self.requests[r].params.temperature for r in rids]
        if all(t <= 0 for t in temps):
            return None, None, None
        tt = torch.tensor(temps, dtype=torch.float32, device=self.device)
        seeds = torch.tensor([(self.requests[r].params.seed or r) * 1000003 + self.requests[r].n_gen
                              for r in rids], dtype=torch.int64, device=self.device)
        return tt, seeds, [self.requests[r].params for r in rids]

    def step(self) -> StepOutput:
        if self.watchdog is not None:
            self.watchdog.arm(f"engine step {self.steps_done}")
        with trace.range("engine.step", step=self.steps_done):
            out = self._step()
        if self.watchdog is not None:
            self.watchdog.disarm()
        self.steps_done += 1
        if self.steps_done % 256 == 0:
            self.comm.check_health()
        state.maybe_periodic(self)
        return out

    def _maybe_poison(self, t: torch.Tensor) -> torch.Tensor:
        """Fault injection (BFLY_FAULT=rank:step:nan): this step's output becomes NaN."""
        if self._poison:
            self._poison = False
            t = t.clone()
            t.fill_(float("nan"))
        return t

    def _decode_sampling(self, rids: list) -> tuple:
        """Per-row temperatures / seeds of a decode plan for the graph's sampler (the values
        _sample_params gives the eager sampler), and whether some row needs the top-k / top-p
        filter (sampled eagerly instead)."""
        reqs = [self.requests[r] for r in rids]
        temps = np.asarray([max(0.0, q.params.temperature) for q in reqs], dtype=np.float32)
        seeds = np.asarray([(q.params.seed or r) * 1000003 + q.n_gen for q, r in zip(reqs, rids)], dtype=np.int64)
        return temps, seeds, any(q.params.needs_filter for q in reqs)

    def _sample(self, logits: torch.Tensor, rids: list, graph_ids=None) -> torch.Tensor:
        if graph_ids is not None and not self._poison:
            return graph_ids
        return self._sample_eager(logits, rids)

    def _sample_eager(self, logits: torch.Tensor, rids: list) -> torch.Tensor:
        """Sample one token per row. With BFLY_NAN_CHECK the sampling kernel also flags rows
        with non-finite logits (id -1, no extra kernel, no host sync); a poisoned or corrupted
        step then raises in _apply_tokens instead of emitting garbage tokens."""
        logits = self._maybe_poison(logits)
        temps, seeds, params = self._sample_params(rids)
        return self.sampler.sample(logits, temps, seeds, params, check_finite=bool(self.nan_check))

    def _step(self) -> StepOutput:
        t0 = time.perf_counter()
        if self.faults.maybe_inject(self.rank, self.steps_done) == "nan":
            self._poison = True
        if self.async_pp:
            return self._pp_tick(t0)
        if self.cp_min:
            out = self._cp_step(t0)
            if out is not None:
                return out
        plan = self.scheduler.schedule()
        ep_pad, any_prefill = 0, plan.kind in (1, 3)
        if self.mesh.ep > 1:
            # expert-parallel ranks must run the same number of MoE collectives with the same
            # row count: agree on the padded token count; idle ranks run an empty step.
            ep_pad, any_prefill, anyw = self._ep_agree(plan)
            if not anyw:
                return StepOutput("idle", [], [], [], 0.0)
            if plan.kind == 0:
                eb = empty_batch(self.device, ep_pad)
                eb.ep_alltoall = any_prefill
                self._run_stages(lambda h: self.runner.run(eb, h), 0, 0, [])
                return StepOutput("ep-idle", [], [], [], time.perf_counter() - t0)
        elif plan.kind == 0:
            return StepOutput("idle", [], [], [], 0.0)
        rids = list(plan.seq_ids)
        if plan.cow:
            self.kv.copy_blocks(list(plan.cow))
        m = self.kv.manager
        self.metrics.set("kv_blocks_free", m.num_free)
        self.metrics.set("kv_blocks_used_fraction", 1.0 - m.num_free / max(1, m.num_blocks))
        if self.prefix_cache:
            self.metrics.set("prefix_cache_hit_tokens", self.scheduler.prefix_hit_tokens)
            self.metrics.set("prefix_cache_blocks", m.num_cached_blocks)
        if plan.preempted:
            self.metrics.inc("preempted_sequences", len(plan.preempted))
        if self.mixed and plan.kind in (1, 3):
            # chunked prefill (+ decode rows): sample the decode rows and completed prompts
            fb, sample = self.runner.mixed_batch(plan, lambda r: self.requests[r].tokens)
            fb.ep_tokens = ep_pad
            fb.ep_alltoall = self.mesh.ep > 1
            logits = self.runner.run(fb)
            new = []
            if sample:
                new = self._sample(logits, sample).tolist()
            out = self._apply_tokens("prefill" if plan.kind == 1 else "mixed", sample, new, t0)
            out.prefill_tokens = int(sum(plan.prefill_lens))
            return out
        if plan.kind == 1:
            fb = self.runner.prefill_batch(plan, lambda r: self.requests[r].tokens)
            fb.ep_tokens = ep_pad
            fb.ep_alltoall = self.mesh.ep > 1
            tokens = self._run_stages(lambda h: self.runner.run(fb, h), fb.num_tokens, len(rids), rids)
            out = self._apply_tokens("prefill", rids, tokens.tolist(), t0)
            out.prefill_tokens = fb.num_tokens
            return out
        else:
            last = [self.requests[r].tokens[-1] for r in rids]
            inp = self.runner.decode_inputs(plan, last)
            if self.mesh.pp > 1:
                tokens = self._pipeline_decode(inp, rids)
            else:
                tokens = self._run_stages(
                    lambda h: self.runner.run_decode(inp, h, ep_tokens=ep_pad, graphs_ok=not any_prefill,
                                                     ep_alltoall=self.mesh.ep > 1 and any_prefill),
                    len(rids), len(rids), rids)
            kind = "decode"
        return self._apply_tokens(kind, rids, tokens.tolist(), t0)

    def _cp_step(self, t0: float) -> Optional[StepOutput]:
        """Context-parallel prefill across the DP replicas. Every replica offers the head of its
        long-prompt queue (if its scheduler could admit it now); the lowest offering replica
        owns this step: its prompt is broadcast, every replica prefills one chunk of it (the
        owner last in chunk order, so it holds the final token and its logits), and the owner's
        cache collects the whole prompt's K/V in passing (context_parallel KV sink). The owner
        samples the first token; the sequence then decodes there like any other. Returns None
        when no replica has a long prompt due (the caller runs a normal step)."""
        from ..parallel.context_parallel import cp_prefill, split_lengths

        dp, me = self.mesh.dp, self.coord.dp
        want = [0] * dp
        if self._cp_queue:
            L = len(self.requests[self._cp_queue[0]].prompt)
            if self.scheduler.can_admit_prefilled(L):
                want[me] = L
        want = self.comm.all_reduce_max_int(want, "dp")
        owner = next((i for i, n in enumerate(want) if n > 0), None)
        if owner is None:
            return None
        L = want[owner]
        g = self.comm.groups["dp"]
        rid = self._cp_queue[0] if me == owner else None
        prompt = self.comm.broadcast_ints(self.requests[rid].prompt if rid is not None else None, L, owner, "dp")
        order = [r for i, r in enumerate(g.ranks) if i != owner] + [g.ranks[owner]]
        sink = None
        if rid is not None:
            self._cp_queue.popleft()
            req = self.requests[rid]
            slots = self.scheduler.admit_prefilled(rid, L, req.params.max_tokens)
            if not slots:
                raise RuntimeError("context-parallel prefill: admission check and allocation disagree")
            sink = [list(slots)]
        with trace.range("engine.cp_prefill", tokens=L, owner=owner):
            logits = cp_prefill(self.model, [prompt], order, order.index(self.rank), g.pg, self.kv.layers,
                                attn=self.ecfg.cp_attention, sink_slots=sink, has_sink=True, broadcast=False)
        mine = split_lengths(L, dp)[order.index(self.rank)]
        self.metrics.inc("cp_prefill_tokens", mine)
        if rid is None:
            return StepOutput("cp-prefill", [], [], [], time.perf_counter() - t0, prefill_tokens=mine)
        out = self._apply_tokens("prefill", [rid], self._sample(logits, [rid]).tolist(), t0)
        out.prefill_tokens = mine
        return out

    def _apply_tokens(self, kind: str, rids: list, new: list, t0: float) -> StepOutput:
        """Append one sampled token per sequence, retire finished ones, record metrics."""
        finished = []
        now = time.perf_counter()
        if any(int(t) < 0 for t in new):
            raise RuntimeError(f"rank {self.rank}: non-finite logits at engine step {self.steps_done}")
        for r, t in zip(rids, new):
            req = self.requests[r]
            req.output.append(int(t))
            req.n_gen = len(req.output)
            if req.first_token_time is None:
                req.first_token_time = now
            self.scheduler.on_token(r)
            reason = None
            if len(req.output) >= req.params.max_tokens:
                reason = "length"
            elif not req.params.ignore_eos and (int(t) in req.params.stop_token_ids or
                                                (self.eos is not None and int(t) == self.eos)):
                reason = "stop"
            if reason:
                req.finished, req.finish_reason, req.finish_time = True, reason, now
                self.scheduler.finish(r)
                finished.append(r)
        dt = time.perf_counter() - t0
        self.metrics.observe_step(kind, len(rids), dt)
        return StepOutput(kind, rids, new, finished, dt)

    def _ep_agree(self, plan) -> tuple:
        """Expert-parallel step agreement (host integers over the control plane, no device
        sync): (padded rows every EP rank runs, whether any rank's plan has prompt rows —
        then every peer's MoE layer takes the variable exchange —, whether any rank has work).
        A plan's rows: its decode rows plus its prompt chunks (mixed plans hold both)."""
        k = plan.kind
        if k == 0:
            rows = 0
        elif k == 2:
            rows = len(plan.seq_ids)
        else:
            rows = int(sum(plan.prefill_lens)) + (plan.num_decode if k == 3 else 0)
        pad, anyp, anyw = self.comm.all_reduce_max_int([rows, int(k in (1, 3)), int(k != 0)], "ep")
        return pad, bool(anyp), bool(anyw)

    def _program_check(self):
        """rows -> the collectives this rank's decode-step program (schedule.rank_program for
        one microbatch of `rows` sequences) has the stage's model code issue, in order: what
        ModelRunner.run enforces through comm.expect under BFLY_PROGRAM_CHECK. Engine-level
        transfers (boundary send / recv, id broadcast) are program-driven already (_execute);
        the EP agreement and the sampling all-gather run outside the stage's forward."""
        from ..partition.schedule import rank_program

        elt = torch.empty((), dtype=self.model.dtype).element_size()
        checked = ("all_reduce", "all_to_all", "ep_dispatch", "ep_return")
        cache: dict = {}

        def instrs(rows: int) -> list:
            v = cache.get(rows)
            if v is None:
                prog = rank_program(self.plan, self.rank, rows, 1, dtype_bytes=elt, native_pp=self._native_pp,
                                    ep_ipc=bool(self.ep_ipc))
                v = cache[rows] = [i for i in prog.comm() if not i.exec and i.op in checked]
            return v
        return instrs

    def _ops(self, microbatches: int, native_pp: bool = False) -> list:
        """Engine-level instructions of this rank's step program (schedule.exec_program)."""
        key = (microbatches, native_pp)
        ops = self._exec_ops.get(key)
        if ops is None:
            ops = self._exec_ops[key] = exec_program(self.plan, self.rank, microbatches, native_pp)
        return ops

    @staticmethod
    def _execute(ops, recv, run, send, sample, broadcast=None) -> None:
        """Interpret a step program: each engine-level instruction calls its hook with the
        instruction (peers, stream, microbatch) — the order and the peers come from the program."""
        h: dict = {}
        out: dict = {}
        for ins in ops:
            e = ins.exec
            if e == "recv":
                h[ins.mb] = recv(ins)
            elif e == "stage":
                out[ins.mb] = run(ins.mb, h.get(ins.mb))
            elif e == "send":
                send(ins, out[ins.mb])
            elif e == "sample":
                sample(ins.mb, out[ins.mb])
            elif e == "broadcast" and broadcast is not None:
                broadcast(ins)

    def _run_stages(self, fn, T: int, R: int, rids) -> torch.Tensor:
        """Run this rank's pipeline stage on one batch; return sampled ids [R] (int32, on
        every rank of the replica). pp > 1: recv residual stream -> stage -> send, or sample
        on the last stage; then the ids broadcast — as the step program lists them."""
        if self.mesh.pp == 1:
            return self._sample(fn(None), rids)
        m, res = self.model, {}

        def recv(ins):
            h = torch.empty(T, self.cfg.hidden_size, dtype=m.dtype, device=self.device)
            self.comm.recv(h, ins.group[0])
            return h

        def send(ins, out):
            self.comm.send(self._maybe_poison(out), ins.group[1])

        def sample(mb, out):
            res["ids"] = self._sample(out, rids)

        def broadcast(ins):
            ids = res.get("ids")
            if ids is None:
                ids = torch.empty(R, dtype=torch.int32, device=self.device)
            self.comm.broadcast_(ids, src_in_group=len(ins.group) - 1, group="pp")
            res["ids"] = ids

        self._execute(self._ops(1), recv, lambda mb, h: fn(h), send, sample, broadcast)
        return res["ids"]

    def _pipeline_decode(self, inp: dict, rids) -> torch.Tensor:
        """Synchronous pipeline decode (BFLY_PP_ASYNC=0, and EP layouts): the batch is cut
        into M = pp microbatches; stage s
        works on microbatch m while stage s+1 works on m-1 (RCCL send/recv of the residual
        stream over xGMI is stream-ordered, so the overlap needs no host synchronisation).
        Each microbatch replays its own hipGraph bucket. The order of receives, stage runs,
        sends and the final broadcast is the step program's (M microbatches)."""
        B = len(rids)
        M = max(1, min(self.mesh.pp, B))
        bounds = [B * i // M for i in range(M + 1)]
        H = self.cfg.hidden_size
        reqs, keep, ids_mb, res = [], [], {}, {}

        def recv(ins):
            h = torch.empty(bounds[ins.mb + 1] - bounds[ins.mb], H, dtype=self.model.dtype, device=self.device)
            self.comm.recv(h, ins.group[0])
            return h

        def run(mb, h):
            a, b = bounds[mb], bounds[mb + 1]
            return self.runner.run_decode({k: v[a:b] for k, v in inp.items()}, h)

        def send(ins, out):
            # copy out of the graph's static output before the next replay can reuse it
            snd = self._maybe_poison(out.clone())
            reqs.append(self.comm.isend(snd, ins.group[1]))
            keep.append(snd)

        def sample(mb, out):
            ids_mb[mb] = self._sample(out, rids[bounds[mb]:bounds[mb + 1]])

        def broadcast(ins):
            for r in reqs:
                r.wait()
            ids = torch.cat([ids_mb[i] for i in range(M)]) if ids_mb else \
                torch.empty(B, dtype=torch.int32, device=self.device)
            self.comm.broadcast_(ids, src_in_group=len(ins.group) - 1, group="pp")
            res["ids"] = ids

        self._execute(self._ops(M), recv, run, send, sample, broadcast)
        return res["ids"]

    # ------------------------------------------------------------------------------------
    # asynchronous pipeline (engine/pipeline.py): one tick = every stage advances one group
    def _pp_tick(self, t0: float) -> StepOutput:
        """Tick k: stage s runs the group that entered at tick k - s. No host wait on this or
        the previous tick's device work: the group that left the last stage at tick k - 1 is
        ADVANCED now (value-free bookkeeping: lengths, length limits, KV slots — right before
        that group is scheduled again) and its first-stage input ids are gathered on the
        device from the broadcast ids; the token VALUES, copied to pinned host memory
        asynchronously, are applied one tick later (they landed long ago). Returns the tokens
        applied this tick, or an empty 'pipeline' output while the pipe fills."""
        pp, s = self.mesh.pp, self.coord.pp
        k = self._tick
        self._tick += 1
        # sends of the previous tick: the next stage posted (or is about to post) their recvs
        # at the start of its tick k, which depends on nothing this rank does in tick k
        for w in self._sends:
            w.wait()
        self._sends = []
        if self.cp_min:
            # context-parallel prefill of a long prompt over the DP replicas (pp == 1): when one
            # is due it is this tick's work on every replica (the agreement is collective, so
            # all replicas take the same branch); the group in flight is advanced next tick.
            # Its first token is sampled and applied synchronously: the sequence is new, in no
            # plan in flight, and joins the least-loaded group as a running sequence
            out = self._cp_step(t0)
            if out is not None:
                return out
        # this rank's stage works on the plan that entered s ticks ago; stages >= 1 enqueue
        # their device work before blocking on the previous tick's ids (keeps the GPU fed)
        mine = next((p for p in self._inflight if p.tick == k - s), None)
        if s > 0 and mine is not None:
            with trace.range("pp.stage_work", tick=k, stage=s):
                self._pp_stage_work(mine)
        out = StepOutput("pipeline", [], [], [], 0.0)
        if self._valued is not None:          # left at tick k - 2: values are on the host
            v, self._valued = self._valued, None
            out = self._apply_values(v, t0)
            out.prefill_tokens = int(sum(v.plan.prefill_lens)) if v.plan.kind in (1, 3) else 0
        if self._pending is not None:         # left at tick k - 1: advance, values next tick
            p, self._pending = self._pending, None
            self._advance(p)
            if not p.idle:
                self._last_left[p.group] = p
            self._valued = p
        # schedule the group entering stage 0 (every rank: replicated deterministic state)
        g = k % pp
        plan = self.scheduler.groups[g].schedule()
        ep_pad = any_prefill = 0
        if self.mesh.ep > 1:
            # every EP rank runs a step whenever one of them has work (the MoE exchange meets
            # every peer), padded to the same rows; a prefill anywhere switches the step to the
            # variable exchange. Host integers over the gloo control plane: no device sync.
            ep_pad, any_prefill, anyw = self._ep_agree(plan)
            if plan.kind == 0 and anyw:
                if pp == 1:
                    eb = empty_batch(self.device, ep_pad)
                    eb.ep_alltoall = bool(any_prefill)
                    self.runner.run(eb)
                else:
                    # EP x PP: this replica's idle plan travels the pipeline like any other, so
                    # at tick k + s its stage s joins the MoE exchanges of the other replicas'
                    # plans of tick k (no rows: nothing is sent between stages, nothing sampled)
                    self._inflight.append(PipePlan(k, g, plan, [], 0, [], seqs=[], ep_pad=ep_pad,
                                                   ep_prefill=bool(any_prefill), idle=True))
                    if s == 0:
                        with trace.range("pp.stage_work", tick=k, stage=0):
                            self._pp_stage_work(self._inflight[-1])
                if not out.new_tokens:
                    out.kind = "ep-idle"
        if plan.kind != 0:
            seqs = list(plan.seq_ids)
            nd = plan.num_decode if plan.kind != 1 else 0
            if plan.kind == 2:
                rids, T = seqs, len(seqs)
            else:   # prefill / mixed: decode rows, then chunks; a prompt's final chunk is sampled
                fin = list(plan.prefill_final)
                rids = seqs[:nd] + [r for r, f in zip(seqs[nd:], fin) if f]
                T = nd + int(sum(plan.prefill_lens))
            if plan.preempted:
                self.metrics.inc("preempted_sequences", len(plan.preempted))
            self._inflight.append(PipePlan(k, g, plan, rids, T, list(plan.cow), seqs=seqs, ep_pad=ep_pad,
                                           ep_prefill=bool(any_prefill)))
            if s == 0:
                with trace.range("pp.stage_work", tick=k, stage=0):
                    self._pp_stage_work(self._inflight[-1])
        # the plan that entered pp-1 ticks ago leaves the last stage now: broadcast its ids
        leaving = next((p for p in self._inflight if p.tick == k - pp + 1), None)
        if leaving is not None:
            self._inflight.remove(leaving)
            if leaving.ids is None:
                leaving.ids = torch.empty(len(leaving.rids), dtype=torch.int32, device=self.device)
            if leaving.rids:   # (a plan of non-final prompt chunks samples nothing: every rank knows)
                self.comm.broadcast_(leaving.ids, src_in_group=pp - 1, group="pp")
            # stream-ordered copy to pinned host memory; read one tick later
            if leaving.ids.is_cuda:
                leaving.host = torch.empty(len(leaving.rids), dtype=torch.int32, pin_memory=True)
                leaving.host.copy_(leaving.ids, non_blocking=True)
                leaving.event = torch.cuda.Event()
                leaving.event.record()
            else:
                leaving.host = leaving.ids
            self._pending = leaving
        if self._prepost:
            self._prepost_recv(k + 1 - s)
        out.seconds = time.perf_counter() - t0
        return out

    def _prepost_recv(self, tick: int) -> None:
        """Post the receive of the plan that enters this stage next tick (it entered stage 0 at
        `tick` and is already in flight; its previous stage sent it this tick)."""
        p = next((q for q in self._inflight if q.tick == tick), None)
        if p is None or p.idle or tick in self._posted:
            return
        H = self.cfg.hidden_size
        if not self._bbufs:
            rows = max(self.ecfg.max_prefill_tokens, self.ecfg.max_batch)
            self._bbufs = [torch.empty(rows, H, dtype=self.model.dtype, device=self.device) for _ in range(2)]
        slot = self._bslot
        self._bslot ^= 1
        buf = self._bbufs[slot][: p.tokens]
        src = self.mesh.prev_stage(self.rank)
        if self._comm_stream is not None:
            if self._bevents[slot] is not None:      # the compute that read this buffer is done
                self._comm_stream.wait_event(self._bevents[slot])
            with torch.cuda.stream(self._comm_stream):
                work = self.comm.irecv(buf, src)
        else:
            work = self.comm.irecv(buf, src)
        self._posted[tick] = (buf, work, slot)

    def _advance(self, p: PipePlan) -> None:
        """Value-free part of applying a plan that left the pipeline: one more token per
        sequence (KV length, scheduler state), length-limit completion, and the deferred
        release of sequences whose stop token was seen while this plan was in flight."""
        sampled = set(p.rids)
        for r in p.seqs:
            req = self.requests[r]
            if req.sched_done:
                continue
            if req.stopping:                  # stopped earlier; this plan's token is discarded
                req.stopping = False
                req.sched_done = True
                self.scheduler.finish(r)
                continue
            if r not in sampled:              # a prompt chunk that does not complete the prompt
                continue
            self.scheduler.on_token(r)
            req.n_gen += 1
            if req.n_gen >= req.params.max_tokens:
                req.sched_done = True
                self.scheduler.finish(r)

    def _apply_values(self, p: PipePlan, t0: float) -> StepOutput:
        """Token values of a plan advanced one tick ago: append them, detect stop tokens
        (releasing the sequence now, or when the plan that still holds it leaves)."""
        if p.event is not None:
            with trace.range("pp.values_wait", tick=self._tick):
                p.event.synchronize()         # recorded two ticks ago: normally long done
        new = [int(t) for t in p.host.tolist()]
        if any(t < 0 for t in new):
            raise RuntimeError(f"rank {self.rank}: non-finite logits at engine step {self.steps_done}")
        now = time.perf_counter()
        rids, toks, finished = [], [], []
        inflight = {r for q in self._inflight for r in q.seqs}
        if self._pending is not None:
            inflight.update(self._pending.seqs)
        for r, t in zip(p.rids, new):
            req = self.requests[r]
            if req.finished:
                continue                      # a token after the stop token: discarded
            req.output.append(t)
            rids.append(r)
            toks.append(t)
            if req.first_token_time is None:
                req.first_token_time = now
            stop = not req.params.ignore_eos and (t in req.params.stop_token_ids or
                                                  (self.eos is not None and t == self.eos))
            if stop or len(req.output) >= req.params.max_tokens:
                req.finished, req.finish_time = True, now
                req.finish_reason = "stop" if stop else "length"
                finished.append(r)
                if stop and not req.sched_done:
                    if r in inflight:
                        req.stopping = True   # released when that plan leaves (_advance)
                    else:
                        req.sched_done = True
                        self.scheduler.finish(r)
        dt = time.perf_counter() - t0
        self.metrics.observe_step(p.kind, len(rids), dt)
        return StepOutput(p.kind, rids, toks, finished, dt)

    def _first_stage_ids(self, p: PipePlan, rids: Optional[list] = None):
        """Input ids of the decode rows (`rids`, default the plan's) of a plan entering stage
        0: the sequences' last tokens. Those sampled by the group's previous plan (values not on
        the host yet) are gathered on the device from its broadcast ids; older ones come from
        the host."""
        rids = p.rids if rids is None else rids
        src = self._last_left.get(p.group)
        where = {r: i for i, r in enumerate(src.rids)} if src is not None and src is self._valued else {}
        if not where or not any(r in where for r in rids):
            return np.asarray([self.requests[r].tokens[-1] for r in rids], dtype=np.int32)
        # one H2D copy of [host ids | source rows] and one row gather (ops.gather_rows: rows
        # with source -1 keep their host id)
        n = len(rids)
        staged = torch.tensor([0 if r in where else self.requests[r].tokens[-1] for r in rids] +
                              [where.get(r, -1) for r in rids], dtype=torch.int32).to(src.ids.device, non_blocking=True)
        ids = staged[:n]
        ops.gather_rows(src.ids.view(-1, 1), staged[n:], out=ids.view(-1, 1))
        return ids

    def _chunk_tokens(self, p: PipePlan):
        """tokens_of(sid) for the prompt chunks of a plan: the request's host tokens. A
        sequence preempted for recompute may need the token its group's previous plan sampled,
        whose value is not applied yet (it is applied next tick): that plan's pinned copy is
        read now (one event wait, only in this case)."""
        need = {}
        nd = p.plan.num_decode if p.plan.kind != 1 else 0
        for j, sid in enumerate(list(p.plan.seq_ids)[nd:]):
            need[sid] = int(p.plan.prefill_starts[j]) + int(p.plan.prefill_lens[j]) if self.mixed \
                else len(p.plan.prefill_slots[j])
        v = self._valued
        extra = {}
        if v is not None and v.rids and any(len(self.requests[r].tokens) < n for r, n in need.items()):
            if v.event is not None:
                v.event.synchronize()
            extra = {r: int(t) for r, t in zip(v.rids, v.host.tolist())}
            self.metrics.inc("pp_value_peeks")
        if not extra:
            return lambda r: self.requests[r].tokens
        return lambda r: self.requests[r].tokens + ([extra[r]] if r in extra else [])

    def _pp_stage_work(self, p: PipePlan) -> None:
        """recv the residual stream (stage > 0) -> run this stage -> isend (not last) or sample
        (last stage: ids kept on the plan for the broadcast, which the tick issues when the plan
        leaves the pipeline) — the step program's instructions of one microbatch."""
        if p.idle:
            # EP x PP idle plan: this stage's MoE layers join the EP exchanges with padded empty
            # rows; no boundary transfer (every rank of the replica knows the plan is empty)
            eb = empty_batch(self.device, p.ep_pad)
            eb.ep_alltoall = p.ep_prefill
            h = None if self.pp_first else torch.empty(0, self.cfg.hidden_size, dtype=self.model.dtype,
                                                       device=self.device)
            self.runner.run(eb, h)
            p.ids = torch.empty(0, dtype=torch.int32, device=self.device)
            return
        native_dec = self._native_pp and p.plan.kind == 2   # the decode graph receives itself
        state: dict = {}

        def recv(ins):
            posted = self._posted.pop(p.tick, None)
            if posted is not None:
                h, work, _ = posted
                work.wait()      # RCCL: the compute stream waits for the transfer, the host does not
                self.metrics.inc("pp_preposted_recvs")
                state["posted"] = posted
                return h
            if ins.stream == "graph":
                return None
            h = torch.empty(p.tokens, self.cfg.hidden_size, dtype=self.model.dtype, device=self.device)
            self.comm.recv(h, ins.group[0])
            return h

        def run(mb, h):
            if p.cow:
                self.kv.copy_blocks(p.cow)
            if self.mixed and p.plan.kind in (1, 3):
                fb, _ = self.runner.mixed_batch(p.plan, self._chunk_tokens(p))
                fb.ep_tokens = p.ep_pad
                fb.ep_alltoall = self.mesh.ep > 1
                nd = p.plan.num_decode
                if self.pp_first and nd:
                    ids = self._first_stage_ids(p, list(p.plan.seq_ids)[:nd])
                    if isinstance(ids, torch.Tensor):
                        fb.input_ids[:nd].copy_(ids)
                out = self.runner.run(fb, h)
            elif p.plan.kind == 1:
                fb = self.runner.prefill_batch(p.plan, self._chunk_tokens(p))
                fb.ep_tokens = p.ep_pad
                fb.ep_alltoall = self.mesh.ep > 1
                out = self.runner.run(fb, h)
            else:
                ids = self._first_stage_ids(p) if self.pp_first else np.zeros(len(p.rids), dtype=np.int32)
                inp = self.runner.decode_inputs(p.plan, ids)
                filtered = False
                if self.pp_last and self.runner.sample_fn is not None:
                    inp["temps"], inp["seeds"], filtered = self._decode_sampling(p.rids)
                state["filtered"] = filtered
                out = self.runner.run_decode(inp, h, ep_tokens=p.ep_pad,
                                             graphs_ok=not p.ep_prefill, ep_alltoall=p.ep_prefill)
            posted = state.get("posted")
            if posted is not None and self._comm_stream is not None:
                ev = torch.cuda.Event()
                ev.record()          # after every kernel that reads the boundary buffer
                self._bevents[posted[2]] = ev
            return out

        def send(ins, out):
            if ins.stream == "send":
                # the whole bucket of the instance just replayed, straight from its static output;
                # the runner replays that instance again only after this send completed
                g = self.runner.last_instance
                w = self.comm.isend(self._maybe_poison(g.output), ins.group[1])
                g.send_done = w.event
                self.metrics.inc("pp_native_graph_sends")
            else:
                snd = out.clone() if p.plan.kind == 2 else out   # graph outputs are reused by the next replay
                w = self.comm.isend(self._maybe_poison(snd), ins.group[1])
                if not isinstance(w, NativeWork):   # native sends keep their tensor alive themselves
                    self._sends.append(w)

        def sample(mb, out):
            graph_ids = self.runner.last_ids if (p.plan.kind == 2 and not state.get("filtered")) else None
            p.ids = self._sample(out, p.rids, graph_ids) if p.rids else \
                torch.empty(0, dtype=torch.int32, device=self.device)

        self._execute(self._ops(1, native_dec), recv, run, send, sample)

    def close(self) -> dict:
        """Release the engine's device resources in dependency order: captured graphs first
        (they hold the native communicators' kernels), then the communicator's IPC buffers and
        native RCCL communicators (bounded finalize-or-abort). Returns the teardown statuses."""
        # pipeline sends still in flight at shutdown may never be matched (the peer stopped
        # stepping): they are dropped, not waited for
        self._sends = []
        self.runner.close()
        if self.watchdog is not None:
            self.watchdog.disarm()
        return self.comm.close()

    # ------------------------------------------------------------------------------------
    def generate(self, prompts: list, params: Optional[SamplingParams] = None) -> list:
        rids = [self.add_request(p, params) for p in prompts]
        while self.has_unfinished_global():
            self.step()
        return [self.requests[r].output for r in rids]


def kv_cache_dtype(name: str, model_dtype: torch.dtype) -> torch.dtype:
    """EngineConfig.kv_cache_dtype -> torch dtype ("auto": the model's own dtype)."""
    name = (name or "auto").lower()
    if name in ("auto", "model"):
        return model_dtype
    if name in ("fp8", "fp8_e4m3", "float8_e4m3fn"):
        return torch.float8_e4m3fn
    if name in ("bf16", "bfloat16"):
        return torch.bfloat16
    raise ValueError(f"unknown kv_cache_dtype {name!r} (auto | bf16 | fp8)")


def balanced_stages(num_layers: int, pp: int) -> list:
    if not 1 <= pp <= num_layers:
        raise ValueError(f"cannot split {num_layers} layers into {pp} pipeline stages")
    base, extra = divmod(num_layers, pp)
    out, a = [], 0
    for s in range(pp):
        n = base + (1 if s < extra else 0)
        out.append((a, a + n))
        a += n
    return out
