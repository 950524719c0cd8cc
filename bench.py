#!/usr/bin/env python3
"""Headline benchmark: node decode throughput (tokens/s) + p50 token latency for Llama-3-70B
(BASELINE.json metric) split across N MI355X GPUs of one node.

Launch:  python bench.py                                   (N = 1)
         python bench.py --gpus N                          (self-launches N ranks, one per GPU)
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher environment (no WORLD_SIZE) and --gpus N > 1 this process becomes the
launcher: it never touches the GPU (no torch import), starts N ranks through
butterfly_amd/launch.py (one process per GPU, RCCL over xGMI), lets rank 0's JSON line through
on stdout, and exits non-zero when any rank fails.

What one "step" is: one engine decode step of the whole node — every running sequence of
every data-parallel replica generates one token through the full model (all 80 layers,
paged attention over its growing KV, LM head, sampling, TP all-reduces / PP transfers),
hipGraph-replayed. Synthetic random prompts (no datasets here) are prefilled before the timed
region; random-init weights of the exact Llama-3-70B architecture in bf16.
Scaling is WEAK: --batch-per-gpu sequences per GPU (global batch = batch_per_gpu x N).
value = generated tokens across the node / wall time of the K timed steps (max over ranks).

BASELINE.json configs are one flag each (--baseline-config):
  1 GPT-2 small, 2-stage layer split, CPU/gloo, 2 ranks      3 Llama-3-70B PP=8
  2 Llama-3-8B on one GPU                                     4 Llama-3-70B TP=2 x PP=4
  5 Mixtral 8x7B expert-parallel over 8 GPUs (all-to-all)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
BASELINE = os.path.join(ROOT, "BASELINE.json")

# BASELINE.json "configs", in order: (model, plan, gpus, extra env)
BASELINE_CONFIGS = {
    1: ("gpt2-small", "pp2", 2, {"BFLY_DIST_BACKEND": "gloo", "BFLY_FORCE_CPU": "1"}),
    2: ("llama3-8b", "auto", 1, {}),
    3: ("llama3-70b", "pp8", 8, {}),
    4: ("llama3-70b", "tp2xpp4", 8, {}),
    5: ("mixtral-8x7b", "ep8", 8, {}),
}
MODEL_NAMES = {"llama3-70b": "Llama-3-70B", "llama3-8b": "Llama-3-8B", "mixtral-8x7b": "Mixtral-8x7B",
               "gpt2-small": "GPT-2-small"}


def groups_of(eng, mesh) -> int:
    """Request groups in flight (the asynchronous pipeline keeps pp of them)."""
    return mesh.pp if eng.async_pp else 1


def parse_plan(s: str):
    """"auto" or an axis product such as tp2xpp4, dp2xtp4, pp8, ep8 (Mixtral: dp = ep)."""
    if s == "auto":
        return "auto"
    d = {}
    for part in s.split("x"):
        k = part.rstrip("0123456789")
        if k not in ("dp", "tp", "pp", "ep") or not part[len(k):]:
            raise SystemExit(f"bad --plan component {part!r} (want e.g. tp2xpp4)")
        d[k] = int(part[len(k):])
    if "ep" in d:
        d.setdefault("dp", d["ep"])
    return d


def log(msg, rank=0):
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (GPUs) of the job (default 1)")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--model", default=None, help="model preset (default llama3-70b)")
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--plan", default=None, help="auto | e.g. tp8, tp2xpp4, dp2xtp4, pp8, ep8")
    ap.add_argument("--baseline-config", type=int, default=None, choices=sorted(BASELINE_CONFIGS),
                    help="run BASELINE.json config N (sets model, plan and default GPU count)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the start-up collective probe (N > 1)")
    ap.add_argument("--kv-dtype", default="auto", help="KV-cache elements: auto (= bf16) | fp8")
    ap.add_argument("--sync-decode", action="store_true",
                    help="single-stage layouts: host waits for each step's tokens before scheduling the "
                         "next (default: EngineConfig.async_decode, the next step overlaps the host work)")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    return ap


def resolve(a) -> None:
    """Fill model / plan / gpus from --baseline-config and the defaults."""
    if a.baseline_config is not None:
        model, plan, gpus, env = BASELINE_CONFIGS[a.baseline_config]
        a.model = a.model or model
        a.plan = a.plan or plan
        a.gpus = a.gpus or gpus
        for k, v in env.items():
            os.environ.setdefault(k, v)
    a.model = a.model or "llama3-70b"
    a.plan = a.plan or "auto"
    a.gpus = a.gpus or 1


def self_launch(a, argv: list) -> int:
    """Parent of an N-rank job started from a bare shell. Loads only butterfly_amd/launch.py
    (stdlib), so this process never initialises HIP before spawning the ranks."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("_bfly_launch", os.path.join(ROOT, "butterfly_amd", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    log(f"launching {a.gpus} ranks (one process per GPU)")
    code = mod.launch([sys.executable, os.path.abspath(__file__), *argv], a.gpus, prefix_output=False)
    if code != 0:
        log(f"a rank failed with exit code {code}")
    return 0 if code == 0 else (code if 0 < code < 256 else 1)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = build_parser().parse_args(argv)
    resolve(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(a, argv)
    return run(a)


def run(a) -> int:
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    from butterfly_amd.config import EngineConfig, ModelConfig
    from butterfly_amd.engine.engine import LLMEngine
    from butterfly_amd.engine.sampler import SamplingParams
    from butterfly_amd.parallel.comm import Communicator, init_distributed
    from butterfly_amd.parallel.probe import apply_policy, ar_policy, probe_comm, summarize
    from butterfly_amd.partition import partition
    from butterfly_amd.partition.hw import MI355X
    from butterfly_amd.utils import flags

    use_gpu = torch.cuda.is_available() and os.environ.get("BFLY_FORCE_CPU", "0") != "1"

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    rank, world, local = init_distributed()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    if world > 1:
        # a multi-GPU step that hangs (wedged collective / peer) dumps every thread's stack and
        # ends the rank with exit 75 instead of waiting for the driver's kill (utils/health.py)
        os.environ.setdefault("BFLY_STEP_TIMEOUT_S", "300")
    if use_gpu:
        # one GPU per rank; ranks sharing a GPU (gloo test mode) all use device 0
        torch.cuda.set_device(local % torch.cuda.device_count())
    backend = dist.get_backend() if world > 1 else ("single-gpu" if use_gpu else "single-cpu")
    # bounded-time checks of every cross-device path before anything depends on them
    # (parallel/preflight.py): failed features fall back on every rank, a failed mandatory
    # check ends the job here, a hang exits 75 naming the rank and the check
    preflight = None
    if world > 1 and flags.get("BFLY_PREFLIGHT"):
        from butterfly_amd.parallel.preflight import PreflightError, run_preflight

        try:
            rep = run_preflight()
        except PreflightError as e:
            print(f"[bench] rank {rank}: {e}", file=sys.stderr, flush=True)
            return 3
        preflight = rep.summary()
        log(f"preflight {preflight['seconds']}s: checks {preflight['checks']} disabled {rep.disabled} "
            f"enabled {rep.enabled}", rank)
        if not rep.allow_tp and a.plan == "auto":
            a.plan = f"dp{world}"
        if flags.get("BFLY_DISABLE_GRAPHS"):
            a.no_graphs = True
    ranks_seen = 1
    if world > 1:
        # proof that the collective backend spans every rank: all-reduce of ones on the world
        dev = "cuda" if backend == "nccl" else "cpu"
        one = torch.ones(1, dtype=torch.int32, device=dev)
        dist.all_reduce(one)
        ranks_seen = int(one.item())
    cfg = ModelConfig.from_preset(a.model)
    # measure this node's collectives before choosing the layout (parallel/probe.py): the
    # partitioner prices all-reduces / hops from the table, and the runtime's all-reduce
    # routing (IPC one-shot / two-shot / RCCL) follows the measured crossovers
    hw = MI355X
    probe = {}
    if world > 1 and backend == "nccl" and not a.no_probe:
        t_probe = time.perf_counter()
        table = probe_comm(world, custom_ar=flags.get("BFLY_CUSTOM_AR"))
        pol = ar_policy(table)
        hw = MI355X.with_comm_table(dict(table, policy=pol))
        probe = summarize(table)
        log(f"comm probe: {time.perf_counter() - t_probe:.1f}s, all-reduce policy {probe.get('ar_policy')}", rank)
    plan = partition(cfg, a.gpus, parse_plan(a.plan), batch_per_gpu=a.batch_per_gpu,
                     ctx=a.prompt_len + a.warmup + a.steps, hw=hw)
    mesh = plan.mesh
    if hw.comm:
        probe["applied"] = apply_policy(hw.comm["policy"], mesh.tp)
    comm = Communicator.from_mesh(mesh)
    log(f"model={cfg.name} gpus={a.gpus} backend={backend} ranks_seen={ranks_seen} plan={plan.name} "
        f"stages={plan.stages} est={plan.estimate['tokens_per_second']:.0f} tok/s", rank)

    replica_batch = a.batch_per_gpu * a.gpus // mesh.dp
    prefill_budget = max(a.prompt_len, min(16384, replica_batch * a.prompt_len // 4))
    # with mixed steps the first-admitted requests already decode while later prompts prefill:
    # leave them enough tokens that the whole batch is still decoding through the timed steps
    prefill_steps = -(-replica_batch * a.prompt_len // prefill_budget) + 2
    gen = a.warmup + a.steps + 2 + prefill_steps + mesh.pp
    max_seq = a.prompt_len + gen + 8
    ecfg = EngineConfig(max_batch=replica_batch, max_seq_len=max_seq,
                        max_prefill_tokens=prefill_budget,
                        kv_cache_tokens=replica_batch * (max_seq + 32),
                        use_graphs=not a.no_graphs,
                        graph_batch_sizes=[replica_batch],
                        kv_cache_dtype=a.kv_dtype, async_decode=not a.sync_decode)
    health = None
    if world > 1 and flags.get("BFLY_HEARTBEAT_S") > 0:
        # rank heartbeats through the job's TCPStore (utils/health.py): a rank that dies or
        # wedges OUTSIDE a step (where the step watchdog cannot see it) aborts the whole job,
        # native communicators first, instead of leaving its peers in a collective
        from butterfly_amd.utils.health import HealthMonitor

        period = flags.get("BFLY_HEARTBEAT_S")
        health = HealthMonitor(dist.distributed_c10d._get_default_store(), rank, world,
                               period=period, timeout=max(60.0, 12 * period)).start()
    t0 = time.perf_counter()
    device = None if use_gpu else torch.device("cpu")
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, stage_layers=plan.stages, device=device)
    sync()
    log(f"engine ready in {time.perf_counter() - t0:.1f}s: {eng.model.local_bytes() / 1e9:.1f} GB weights/rank, "
        f"KV {eng.kv.bytes() / 1e9:.1f} GB ({eng.kv.capacity_tokens} tokens)", rank)

    dp_idx = mesh.coord(rank).dp
    g = torch.Generator().manual_seed(1234 + dp_idx)
    params = SamplingParams(max_tokens=gen, ignore_eos=True)
    for i in range(replica_batch):
        prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
        eng.add_request(prompt, params)
    # the decode graph is captured before the prefill clock starts (a server captures at
    # start-up); one rank only here: a multi-rank capture's warm-up runs issue collectives
    if world == 1 and not a.no_graphs:
        eng.precapture_decode(replica_batch // groups_of(eng, mesh))
    # prefill (untimed; reported separately)
    tp0 = time.perf_counter()
    prefill_tokens = 0
    # with the asynchronous pipeline (pp > 1) one step advances every stage by one request
    # group (replica_batch / pp sequences) and each sequence gets a token every pp steps
    groups = groups_of(eng, mesh)
    decode_streak = 0
    while eng.scheduler.num_waiting > 0 or decode_streak < groups:
        out = eng.step()
        prefill_tokens += out.prefill_tokens
        decode_streak = decode_streak + 1 if out.kind == "decode" else 0
    sync()
    prefill_s = time.perf_counter() - tp0
    log(f"prefill {prefill_tokens} tokens in {prefill_s:.2f}s ({prefill_tokens / prefill_s:.0f} tok/s/replica)", rank)
    for _ in range(a.warmup):
        eng.step()
    if world > 1:
        dist.barrier()
    sync()
    step_times = []
    gen_tokens = 0
    t_start = time.perf_counter()
    for _ in range(a.steps):
        ts = time.perf_counter()
        out = eng.step()
        step_times.append(time.perf_counter() - ts)
        assert out.kind == "decode", out.kind
        gen_tokens += len(out.new_tokens)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if replica_batch % groups == 0:   # every step carried one full group
        assert gen_tokens == a.steps * replica_batch // groups, (gen_tokens, a.steps, replica_batch, groups)
    if world > 1:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed, gen_tokens], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
    # tokens of the whole node: every DP replica generates gen_tokens (same work per replica)
    tokens = gen_tokens * mesh.dp
    value = tokens / elapsed
    # per-token latency of a sequence = `groups` steps (one step when pp == 1)
    p50 = statistics.median(step_times) * 1e3 * groups
    p99 = sorted(step_times)[max(0, int(len(step_times) * 0.99) - 1)] * 1e3 * groups
    with open(BASELINE) as f:
        base = json.load(f)
    pub = base.get("published") or {}
    ref = pub.get("tokens_per_sec") if isinstance(pub, dict) else None
    runner = eng.runner
    res = {
        "metric": base["metric"],
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": a.gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "p50_latency_ms": round(p50, 3),
        "p99_latency_ms": round(p99, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (value / ref) if ref else None,
        "dtype": {torch.bfloat16: "bf16", torch.float32: "fp32"}.get(eng.model.dtype, str(eng.model.dtype)),
        "data": "synthetic random prompts; random-init weights (deterministic hash init)",
        "prefill_tokens_per_s_per_replica": round(prefill_tokens / prefill_s, 1),
        "world_size": world,
        "backend": backend,
        "rccl_ranks_seen": ranks_seen,
        "plan": {"name": plan.name, "dp": mesh.dp, "tp": mesh.tp, "pp": mesh.pp, "ep": mesh.ep,
                 "estimate_tokens_per_s": round(plan.estimate["tokens_per_second"], 1)},
        "graphs_captured": runner.captured_buckets,
        "graphs_failed": sorted(runner.eager_buckets),
        "custom_ar_active": comm.custom_ar is not None,
        "ep_ipc_active": comm.ep_ipc is not None,
        "ep_ipc_link_bytes_rank0": comm.ep_ipc.stats() if comm.ep_ipc is not None else None,
        "comm_probe": probe or None,
        "preflight": preflight,
        "native_rccl": any(g is not None and g.native is not None for g in comm.groups.values()),
        "config": {"model": MODEL_NAMES.get(a.model, a.model),
                   "global_batch": a.batch_per_gpu * a.gpus, "seq_len": a.prompt_len,
                   "parallelism": plan.name, "stages": [list(s) for s in plan.stages],
                   "hipgraph": bool(runner.captured_buckets) and not runner.eager_buckets,
                   "kv_cache_dtype": str(eng.kv_dtype).replace("torch.", ""),
                   "pp_async_groups": groups if groups > 1 else None,
                   "async_decode": bool(eng.async_pp and mesh.pp == 1),
                   "mixed": bool(eng.mixed), "prefix_caching": bool(eng.prefix_cache),
                   "packed_decode_weights_gb": round(sum(t.numel() * t.element_size()
                                                         for t in eng.model.packed.values()) / 1e9, 1)},
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    # orderly teardown: graphs, then IPC buffers and native RCCL communicators (bounded
    # finalize-or-abort, never a hang), then the heartbeat and the process group
    closed = eng.close()
    if health is not None:
        health.stop()
    if closed:
        log(f"teardown: {closed}", rank)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
