#!/usr/bin/env python3
"""Expert-parallel decode of a real-size MoE model on ONE GPU, for kernel traces.

Two modes:
* threads (default): `ep` EP ranks run as threads of this process on cuda:0 and meet in the
  in-process loopback backend (parallel/fake.py); the exchange is the loopback emulation.
  Eager only (the loopback collectives synchronise threads on the host).
* processes (RANK set, e.g. `python -m butterfly_amd launch -n 4 -- python tools/ep_trace.py`
  with BFLY_DIST_BACKEND=gloo): one process per EP rank, all on cuda:0, over gloo; the decode
  MoE exchange runs the byte-minimal IPC kernels (csrc/kernels/ep_ipc.hip) and the decode step
  replays from hipGraphs. Each rank prints its link-row statistics. Profile one rank per
  rocprofv3 through a wrapper, e.g. `launch -n 4 -- bash tools/prof_rank.sh TAG python3
  tools/ep_trace.py` (the launcher itself never touches the GPU).
usage: python tools/ep_trace.py [--model mixtral-8x7b] [--ep 2] [--batch 64] [--prompt 128] [--steps 4]"""
import argparse
import json
import os
import sys
import time

# every EP rank shares cuda:0 here: opt in to shared-GPU IPC groups (refused in production)
os.environ.setdefault("BFLY_IPC_SHARED_DEVICE", "1")

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd.config import EngineConfig, ModelConfig  # noqa: E402
from butterfly_amd.engine.engine import LLMEngine  # noqa: E402
from butterfly_amd.engine.sampler import SamplingParams  # noqa: E402
from butterfly_amd.parallel.fake import FakeWorld  # noqa: E402
from butterfly_amd.parallel.mesh import Mesh  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="mixtral-8x7b")
ap.add_argument("--ep", type=int, default=2)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--prompt", type=int, default=128)
ap.add_argument("--steps", type=int, default=4)
a = ap.parse_args()
cfg = ModelConfig.from_preset(a.model)
procs = "RANK" in os.environ
if procs:
    a.ep = int(os.environ["WORLD_SIZE"])
mesh = Mesh(dp=a.ep, ep=a.ep)
DEV = "cuda:0" if torch.cuda.is_available() else "cpu"
if DEV != "cpu":
    torch.cuda.set_device(0)
sync = torch.cuda.synchronize if DEV != "cpu" else (lambda: None)


def rank_main(rank, comm, graphs):
    ecfg = EngineConfig(max_batch=a.batch, max_seq_len=a.prompt + a.steps + 16, max_prefill_tokens=4096,
                        kv_cache_tokens=a.batch * (a.prompt + a.steps + 48), use_graphs=graphs,
                        graph_batch_sizes=[a.batch])
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device=DEV)
    g = torch.Generator().manual_seed(rank)
    for _ in range(a.batch):
        eng.add_request(torch.randint(0, cfg.vocab_size, (a.prompt,), generator=g).tolist(),
                        SamplingParams(max_tokens=a.steps + 8, ignore_eos=True))
    while eng.scheduler.num_waiting > 0:
        eng.step()
    eng.step()
    eng.step()                       # graph capture (processes) happens on the first decode steps
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = eng.step()
        assert out.kind == "decode", out.kind
    sync()
    dt = time.perf_counter() - t0
    ipc = comm.ep_ipc
    return dt, (ipc.stats() if ipc is not None else None), eng.runner.captured_buckets


if procs:
    import torch.distributed as dist

    from butterfly_amd.parallel.comm import Communicator

    dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=a.ep)
    comm = Communicator.from_mesh(mesh)
    dt, st, caps = rank_main(comm.rank, comm, True)
    print(json.dumps({"rank": comm.rank, "model": cfg.name, "ep": a.ep, "batch_per_rank": a.batch,
                      "ms_per_step": round(dt / a.steps * 1e3, 2), "ep_ipc": st, "graphs": caps,
                      "note": "all EP ranks time-share one GPU"}), flush=True)
    dist.destroy_process_group()
else:
    world = FakeWorld(mesh, timeout_s=600)
    res = world.run(lambda r, c: rank_main(r, c, False))
    print(f"{cfg.name} ep={a.ep} batch/rank={a.batch}: {max(t for t, _, _ in res) / a.steps * 1e3:.2f} ms per "
          f"decode step (all {a.ep} EP ranks serialised on one GPU)", flush=True)
