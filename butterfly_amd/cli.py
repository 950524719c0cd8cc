"""Command line: `python -m butterfly_amd <command>`.

  partition  --model llama3-70b --gpus 8 [--strategy tp2xpp4] [--objective latency] [--out plan.json]
             [--schedule RANK]   (that rank's decode-step communication program)
  generate   --model llama-tiny|CKPT_DIR --prompt "..." [--max-tokens N] [--plan auto|tp2]
  serve      --model ... [--host 127.0.0.1 --port 8000]         (run under `launch` for N GPUs)
  bench      ...                                                  (forwards to bench.py)
  launch     -n 8 -- <program args...>                            one process per GPU
  ckpt       convert-hf SRC DST | reshard SRC DST --gpus N [--strategy ...] | inspect DIR
  info                                                            build / device / flag report
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys


def _strategy(s: str | None):
    if not s or s == "auto":
        return "auto"
    d = {}
    for part in s.split("x"):
        k = part.rstrip("0123456789")
        d[k] = int(part[len(k):])
    return d


def cmd_partition(a) -> int:
    from .partition import partition

    plan = partition(a.model, a.gpus, _strategy(a.strategy), objective=a.objective,
                     batch_per_gpu=a.batch_per_gpu, ctx=a.ctx)
    text = plan.to_json(a.out)
    est = plan.estimate
    print(f"plan {plan.name}: stages={plan.stages} est {est['tokens_per_second']:.0f} tok/s, "
          f"step {est['step_seconds'] * 1e3:.2f} ms", file=sys.stderr)
    if a.schedule is not None:
        # the communication program of one decode step on the given rank (partition/schedule.py)
        from .partition.schedule import check_programs, programs

        from .utils import flags

        B = a.batch_per_gpu * a.gpus // plan.mesh.dp
        m = plan.mesh
        if not 0 <= a.schedule < a.gpus:
            print(f"--schedule: rank {a.schedule} is not in [0, {a.gpus})", file=sys.stderr)
            return 2
        # the engine's choice: asynchronous pipeline -> one step (tick) carries one of pp request
        # groups; synchronous pipeline -> the step's batch is cut into pp microbatches
        if m.pp > 1 and m.ep == 1 and flags.get("BFLY_PP_ASYNC"):
            progs = programs(plan, B // m.pp)
        else:
            progs = programs(plan, B, microbatches=m.pp)
        check_programs(progs)
        print(progs[a.schedule].describe(), file=sys.stderr)
        return 0
    if not a.out:
        print(text)
    return 0


def cmd_generate(a) -> int:
    from .api import LLM
    from .config import EngineConfig
    from .engine.sampler import SamplingParams

    from .engine import state

    snap_every = a.snapshot_every if a.snapshot_dir else 0
    llm = LLM(a.model, plan=_strategy(a.plan),
              engine_config=EngineConfig(max_batch=8, max_seq_len=a.max_seq_len, use_graphs=not a.no_graphs,
                                         snapshot_dir=a.snapshot_dir, snapshot_every=snap_every),
              tokenizer=a.tokenizer)
    prompts = a.prompt or ["Hello"]
    params = SamplingParams(max_tokens=a.max_tokens, temperature=a.temperature, seed=a.seed, ignore_eos=True)
    # a restart is BFLY_RESTART (launch --max-restarts) or torchrun's TORCHELASTIC_RESTART_COUNT
    restart = max(int(os.environ.get("BFLY_RESTART", "0") or 0),
                  int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0))
    # the snapshot carries this job's fingerprint: a run resumes only its own job's state (a
    # restart, or a manual re-run of the same job), never a stale snapshot an earlier, different
    # job left in the directory — and only such a foreign snapshot is ever deleted
    job = state.job_fingerprint(a.model, prompts, params)
    llm.engine.job_id = job
    snap = state.replica_path(a.snapshot_dir, llm.dp_rank) if a.snapshot_dir else None
    ours = snap is not None and snap.exists() and state.snapshot_job(snap) == job
    if snap is not None and snap.exists() and not ours:
        print(f"ignoring {snap}: written by another job", file=sys.stderr)
        if llm.engine.coord.tp == 0 and llm.engine.coord.pp == 0:
            snap.unlink()
    if ours:
        # replay the request state of the interrupted attempt (engine/state.py)
        outs = llm.resume(a.snapshot_dir, job=job)
        print(f"resumed {len(outs)} requests from {a.snapshot_dir} (restart {restart})", file=sys.stderr)
    else:
        outs = llm.generate(prompts, params)
    if llm.rank == 0:
        for o in outs:
            print(json.dumps({"prompt": o.prompt, "text": o.text, "token_ids": o.token_ids,
                              "ttft_s": o.ttft_s, "e2e_s": o.e2e_s}))
    llm.close()
    return 0


def cmd_serve(a) -> int:
    from .api import LLM
    from .config import EngineConfig
    from .server import serve

    llm = LLM(a.model, plan=_strategy(a.plan), tokenizer=a.tokenizer,
              engine_config=EngineConfig(max_batch=a.max_batch, max_seq_len=a.max_seq_len))
    serve(llm, a.host, a.port)
    return 0


def cmd_launch(a) -> int:
    from .launch import launch

    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        print("launch: missing program", file=sys.stderr)
        return 2
    placement = None
    if a.plan:
        from .partition import PartitionPlan

        plan = PartitionPlan.from_json(open(a.plan).read())
        if plan.n_gpus != a.nproc:
            print(f"launch: plan is for {plan.n_gpus} GPUs, -n {a.nproc}", file=sys.stderr)
            return 2
        placement = plan.placement or None
    return launch(cmd, a.nproc, a.master_port, placement=placement, max_restarts=a.max_restarts)


def cmd_ckpt(a) -> int:
    from . import ckpt

    if a.action == "convert-hf":
        from .ckpt.hf import convert_hf

        cfg = convert_hf(a.src, a.dst)
        print(f"converted {cfg.arch} ({cfg.param_count() / 1e9:.2f} B params) -> {a.dst}")
    elif a.action == "reshard":
        from .partition import partition

        plan = partition(ckpt.model_config(a.src), a.gpus, _strategy(a.strategy))
        ckpt.reshard(a.src, a.dst, plan)
        print(f"resharded {a.src} -> {a.dst} for plan {plan.name}")
    elif a.action == "inspect":
        m = ckpt.read_manifest(a.src)
        n = sum(1 for _ in m["tensors"])
        print(json.dumps({"format": m["format"], "version": m["version"], "model": m["model"]["name"],
                          "dtype": m["dtype"], "tensors": n, "plan": m.get("plan", {}).get("name") or m.get("plan")},
                         indent=1))
    return 0


def cmd_info(a) -> int:
    import torch

    from . import ops
    from .utils import flags

    info = {"torch": torch.__version__, "hip": torch.version.hip, "gpu": torch.cuda.is_available(),
            "kernels_loaded": ops.load_library(), "kernel_lib": ops.library_path(), "flags": flags.dump()}
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        info["device"] = {"name": p.name, "arch": getattr(p, "gcnArchName", ""), "memory_gb": p.total_memory / 1e9,
                          "cus": p.multi_processor_count, "count": torch.cuda.device_count()}
    print(json.dumps(info, indent=1, default=str))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="butterfly_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("partition")
    p.add_argument("--model", default="llama3-70b")
    p.add_argument("--gpus", type=int, default=8)
    p.add_argument("--strategy", default="auto")
    p.add_argument("--objective", default="throughput", choices=["throughput", "latency"])
    p.add_argument("--batch-per-gpu", type=int, default=64)
    p.add_argument("--ctx", type=int, default=1024)
    p.add_argument("--out", default=None)
    p.add_argument("--schedule", type=int, default=None, metavar="RANK",
                   help="print RANK's decode-step communication program instead of the plan JSON")
    p.set_defaults(fn=cmd_partition)
    g = sub.add_parser("generate")
    g.add_argument("--model", default="llama-tiny")
    g.add_argument("--prompt", action="append")
    g.add_argument("--max-tokens", type=int, default=16)
    g.add_argument("--max-seq-len", type=int, default=1024)
    g.add_argument("--temperature", type=float, default=0.0)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--plan", default="auto")
    g.add_argument("--tokenizer", default=None)
    g.add_argument("--no-graphs", action="store_true")
    g.add_argument("--snapshot-dir", default=None,
                   help="write request-state snapshots here; a restarted job (launch --max-restarts) resumes from them")
    g.add_argument("--snapshot-every", type=int, default=4, help="engine steps between snapshots")
    g.set_defaults(fn=cmd_generate)
    s = sub.add_parser("serve")
    s.add_argument("--model", default="llama-tiny")
    s.add_argument("--plan", default="auto")
    s.add_argument("--tokenizer", default=None)
    s.add_argument("--host", default="127.0.0.1")
    s.add_argument("--port", type=int, default=8000)
    s.add_argument("--max-batch", type=int, default=64)
    s.add_argument("--max-seq-len", type=int, default=4096)
    s.set_defaults(fn=cmd_serve)
    b = sub.add_parser("bench", add_help=False)
    b.add_argument("rest", nargs=argparse.REMAINDER)
    b.set_defaults(fn=lambda a: subprocess.call([sys.executable, os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"), *a.rest]))
    la = sub.add_parser("launch")
    la.add_argument("-n", "--nproc", type=int, default=1)
    la.add_argument("--master-port", type=int, default=None)
    la.add_argument("--plan", default=None, help="PartitionPlan JSON: its placement maps ranks to GPUs")
    la.add_argument("--max-restarts", type=int, default=0,
                    help="start a failed job again up to N times (BFLY_RESTART=<attempt> in its environment)")
    la.add_argument("cmd", nargs=argparse.REMAINDER)
    la.set_defaults(fn=cmd_launch)
    c = sub.add_parser("ckpt")
    c.add_argument("action", choices=["convert-hf", "reshard", "inspect"])
    c.add_argument("src")
    c.add_argument("dst", nargs="?")
    c.add_argument("--gpus", type=int, default=1)
    c.add_argument("--strategy", default="auto")
    c.set_defaults(fn=cmd_ckpt)
    i = sub.add_parser("info")
    i.set_defaults(fn=cmd_info)
    a = ap.parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
