#!/usr/bin/env python3
"""Headline benchmark: node decode throughput (tokens/s) + p50 token latency for Llama-3-70B
(BASELINE.json metric) split across N MI355X GPUs of one node.

Launch:  python bench.py                                   (N = 1)
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N --steps K --warmup W

What one "step" is: one engine decode step of the whole node — every running sequence of
every data-parallel replica generates one token through the full model (all 80 layers,
paged attention over its growing KV, LM head, sampling, TP all-reduces / PP transfers),
hipGraph-replayed. Synthetic random prompts (no datasets here) are prefilled before the timed
region; random-init weights of the exact Llama-3-70B architecture in bf16.
Scaling is WEAK: --batch-per-gpu sequences per GPU (global batch = batch_per_gpu x N).
value = generated tokens across the node / wall time of the K timed steps (max over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from butterfly_amd.config import EngineConfig, ModelConfig  # noqa: E402
from butterfly_amd.engine.engine import LLMEngine  # noqa: E402
from butterfly_amd.engine.sampler import SamplingParams  # noqa: E402
from butterfly_amd.parallel.comm import Communicator, init_distributed  # noqa: E402
from butterfly_amd.parallel.mesh import Mesh  # noqa: E402
from butterfly_amd.partition import partition  # noqa: E402

BASELINE = os.path.join(ROOT, "BASELINE.json")


def parse_plan(s: str, n: int):
    if s == "auto":
        return "auto"
    d = {}
    for part in s.split("x"):
        k = part.rstrip("0123456789")
        d[k] = int(part[len(k):])
    return d


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def log(msg, rank=0):
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--plan", default="auto", help="auto | e.g. tp8, tp2xpp4, dp2xtp4")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv-dtype", default="auto", help="KV-cache elements: auto (= bf16) | fp8")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    a = ap.parse_args()

    rank, world, local = init_distributed()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    if torch.cuda.is_available():
        # one GPU per rank; ranks sharing a GPU (gloo test mode) all use device 0
        torch.cuda.set_device(local % torch.cuda.device_count())
    cfg = ModelConfig.from_preset(a.model)
    plan = partition(cfg, a.gpus, parse_plan(a.plan, a.gpus), batch_per_gpu=a.batch_per_gpu,
                     ctx=a.prompt_len + a.warmup + a.steps)
    mesh = plan.mesh
    comm = Communicator.from_mesh(mesh)
    log(f"model={cfg.name} gpus={a.gpus} plan={plan.name} stages={plan.stages}", rank)

    replica_batch = a.batch_per_gpu * a.gpus // mesh.dp
    prefill_budget = max(a.prompt_len, min(16384, replica_batch * a.prompt_len // 4))
    # with mixed steps the first-admitted requests already decode while later prompts prefill:
    # leave them enough tokens that the whole batch is still decoding through the timed steps
    prefill_steps = -(-replica_batch * a.prompt_len // prefill_budget) + 2
    gen = a.warmup + a.steps + 2 + prefill_steps
    max_seq = a.prompt_len + gen + 8
    ecfg = EngineConfig(max_batch=replica_batch, max_seq_len=max_seq,
                        max_prefill_tokens=prefill_budget,
                        kv_cache_tokens=replica_batch * (max_seq + 32),
                        use_graphs=not a.no_graphs,
                        graph_batch_sizes=[replica_batch],
                        kv_cache_dtype=a.kv_dtype)
    t0 = time.perf_counter()
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, stage_layers=plan.stages)
    sync()
    log(f"engine ready in {time.perf_counter() - t0:.1f}s: {eng.model.local_bytes() / 1e9:.1f} GB weights/rank, "
        f"KV {eng.kv.bytes() / 1e9:.1f} GB ({eng.kv.capacity_tokens} tokens)", rank)

    dp_idx = mesh.coord(rank).dp
    g = torch.Generator().manual_seed(1234 + dp_idx)
    params = SamplingParams(max_tokens=gen, ignore_eos=True)
    for i in range(replica_batch):
        prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=g).tolist()
        eng.add_request(prompt, params)
    # prefill (untimed; reported separately)
    tp0 = time.perf_counter()
    prefill_tokens = 0
    # with the asynchronous pipeline (pp > 1) one step advances every stage by one request
    # group (replica_batch / pp sequences) and each sequence gets a token every pp steps
    groups = mesh.pp if eng.async_pp else 1
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
        dev = "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"
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
        "config": {"model": "Llama-3-70B" if a.model == "llama3-70b" else a.model,
                   "global_batch": a.batch_per_gpu * a.gpus, "seq_len": a.prompt_len,
                   "parallelism": plan.name, "stages": [list(s) for s in plan.stages],
                   "hipgraph": eng.runner.use_graphs, "kv_cache_dtype": str(eng.kv_dtype).replace("torch.", ""), "pp_async_groups": groups if groups > 1 else None},
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
