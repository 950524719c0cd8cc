"""Python API ("Client-facing API for submitting inference requests",
/root/reference/CLAUDE.md:23).

    import butterfly_amd as bfly
    plan = bfly.partition("llama3-70b", n_gpus=8, strategy={"tp": 2, "pp": 4})
    llm = bfly.LLM("llama3-70b", plan=plan)              # random-init weights
    llm = bfly.LLM("/ckpts/llama3-70b", plan="auto")     # butterfly-ckpt directory
    outs = llm.generate(["The capital of France is"], bfly.SamplingParams(max_tokens=32))

Multi-GPU runs are SPMD: launch one process per GPU (`python -m butterfly_amd launch -n 8 ...`
or torchrun) and construct the same LLM on every rank; `generate` returns the outputs on every
rank of the replica (data-parallel ranks serve the prompts `dp_split` assigns them).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, Union

import torch

from .config import EngineConfig, ModelConfig
from .engine.engine import LLMEngine
from .engine.sampler import SamplingParams
from .parallel.comm import Communicator, init_distributed
from .partition import PartitionPlan, partition
from .utils import flags
from .utils.tokenizer import load_tokenizer


@dataclass
class RequestOutput:
    prompt: Union[str, list]
    token_ids: list
    text: Optional[str]
    finish_reason: Optional[str]
    ttft_s: Optional[float] = None
    e2e_s: Optional[float] = None
    metrics: dict = field(default_factory=dict)


class LLM:
    def __init__(self, model: Union[str, ModelConfig], plan: Union[str, dict, PartitionPlan, None] = "auto",
                 engine_config: Optional[EngineConfig] = None, tokenizer: Optional[str] = None,
                 seed: int = 0, objective: str = "throughput"):
        rank, world, local = init_distributed()
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        ckpt = None
        if isinstance(model, ModelConfig):
            cfg = model
        elif Path(str(model)).is_dir():
            from .ckpt import model_config

            ckpt = str(model)
            cfg = model_config(ckpt)
        else:
            cfg = ModelConfig.from_preset(str(model))
        ecfg = engine_config or EngineConfig(seed=seed)
        if not isinstance(plan, PartitionPlan):
            plan = partition(cfg, world, plan or "auto", objective=objective,
                             batch_per_gpu=max(1, ecfg.max_batch // max(1, world)), ctx=ecfg.max_seq_len)
        if plan.n_gpus != world:
            raise ValueError(f"plan is for {plan.n_gpus} GPUs but WORLD_SIZE={world}")
        self.cfg, self.plan, self.rank, self.world = cfg, plan, rank, world
        self.comm = Communicator.from_mesh(plan.mesh)
        device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
        self.engine = LLMEngine(cfg, plan.mesh, ecfg, comm=self.comm, device=device,
                                stage_layers=plan.stages, model=None if ckpt is None else self._load(ckpt, plan, device))
        self.tokenizer = load_tokenizer(tokenizer)
        self.health = None
        period = flags.get("BFLY_HEARTBEAT_S")
        if world > 1 and period > 0:
            # rank heartbeats through the job's TCPStore: a dead or wedged rank aborts the
            # whole job instead of leaving its peers blocked in a collective
            import torch.distributed as dist

            from .utils.health import HealthMonitor

            self.health = HealthMonitor(dist.distributed_c10d._get_default_store(), rank, world,
                                        period=period, timeout=max(30.0, 6 * period)).start()

    def _load(self, path, plan, device):
        from .ckpt import load_into
        from .models import build_model

        m = build_model(self.cfg, plan.shard(self.rank), device=device,
                        dtype=torch.bfloat16 if device.type == "cuda" else torch.float32, comm=self.comm)
        load_into(m, path)
        return m

    @property
    def dp_rank(self) -> int:
        return self.plan.mesh.coord(self.rank).dp

    def dp_split(self, prompts: list) -> list:
        """The share of `prompts` this rank's data-parallel replica serves."""
        dp = self.plan.dp
        return prompts[self.dp_rank::dp] if dp > 1 else prompts

    def generate(self, prompts: list, params: Optional[SamplingParams] = None) -> list:
        params = params or SamplingParams()
        mine = self.dp_split(prompts)
        ids = [self.tokenizer.encode(p) if isinstance(p, str) else list(p) for p in mine]
        eng = self.engine
        t0 = time.perf_counter()
        rids = [eng.add_request(x, params) for x in ids]
        while eng.has_unfinished_global():
            eng.step()
        outs = []
        for p, r in zip(mine, rids):
            req = eng.requests[r]
            text = self.tokenizer.decode(req.output) if isinstance(p, str) else None
            outs.append(RequestOutput(prompt=p, token_ids=list(req.output), text=text,
                                      finish_reason=req.finish_reason,
                                      ttft_s=(req.first_token_time - req.arrival) if req.first_token_time else None,
                                      e2e_s=(req.finish_time or time.perf_counter()) - req.arrival))
        self.last_generate_s = time.perf_counter() - t0
        return outs

    def metrics(self) -> dict:
        return self.engine.metrics.summary()

    def close(self) -> dict:
        """Stop the heartbeat monitor and release the engine's graphs, IPC buffers and native
        communicators (bounded; LLMEngine.close). Returns the teardown statuses."""
        if self.health is not None:
            self.health.stop()
            self.health = None
        return self.engine.close()

    # ---- request-state snapshots (engine/state.py) -------------------------
    def save_state(self, directory) -> Optional[Path]:
        """Write this replica's request state to <directory>/replica-<dp>.json (one rank per
        replica writes; the others return None)."""
        from .engine import state

        c = self.plan.mesh.coord(self.rank)
        if c.tp != 0 or c.pp != 0:
            return None
        return state.save(self.engine, state.replica_path(directory, c.dp))

    def resume(self, directory, job: Optional[str] = None) -> list:
        """Replay a snapshot written by save_state() or by EngineConfig.snapshot_every into this
        (fresh) LLM: re-admit the replica's unfinished requests (prompt + tokens generated so far
        are prefilled again), run them to completion, and return every request of the snapshot,
        finished ones included, in request-id order. `job`: only a snapshot with this job
        fingerprint (engine/state.py job_fingerprint) is accepted."""
        from .engine import state

        eng = self.engine
        rids = state.restore(eng, state.load(state.replica_path(directory, self.dp_rank)), job=job)
        t0 = time.perf_counter()
        while eng.has_unfinished_global():
            eng.step()
        self.last_generate_s = time.perf_counter() - t0
        outs = []
        for r in rids:
            req = eng.requests[r]
            outs.append(RequestOutput(prompt=req.prompt, token_ids=list(req.output),
                                      text=self.tokenizer.decode(req.output), finish_reason=req.finish_reason))
        return outs
