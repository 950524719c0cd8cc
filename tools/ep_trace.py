#!/usr/bin/env python3
"""Expert-parallel decode on ONE GPU, for kernel traces: `ep` EP ranks run as threads of this
process on cuda:0 and meet in the in-process loopback backend (parallel/fake.py), so a single
`rocprofv3 --kernel-trace -- python tools/ep_trace.py` records the whole EP decode path of the
real model size: router, dispatch packing, fixed-capacity all-to-all (device copies here),
moe_align + grouped expert GEMMs on routed rows only, return and combine. Eager (no graphs:
the loopback collectives synchronise threads on the host).
usage: python tools/ep_trace.py [--model mixtral-8x7b] [--ep 2] [--batch 64] [--prompt 128] [--steps 4]"""
import argparse
import os
import sys
import time

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
mesh = Mesh(dp=a.ep, ep=a.ep)
world = FakeWorld(mesh, timeout_s=600)
DEV = "cuda:0" if torch.cuda.is_available() else "cpu"
if DEV != "cpu":
    torch.cuda.set_device(0)
sync = torch.cuda.synchronize if DEV != "cpu" else (lambda: None)


def rank_main(rank, comm):
    ecfg = EngineConfig(max_batch=a.batch, max_seq_len=a.prompt + a.steps + 16, max_prefill_tokens=4096,
                        kv_cache_tokens=a.batch * (a.prompt + a.steps + 48), use_graphs=False)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device=DEV)
    g = torch.Generator().manual_seed(rank)
    for _ in range(a.batch):
        eng.add_request(torch.randint(0, cfg.vocab_size, (a.prompt,), generator=g).tolist(),
                        SamplingParams(max_tokens=a.steps + 8, ignore_eos=True))
    while eng.scheduler.num_waiting > 0:
        eng.step()
    eng.step()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = eng.step()
        assert out.kind == "decode", out.kind
    sync()
    return time.perf_counter() - t0


ts = world.run(rank_main)
print(f"{cfg.name} ep={a.ep} batch/rank={a.batch}: {max(ts) / a.steps * 1e3:.2f} ms per decode step "
      f"(all {a.ep} EP ranks serialised on one GPU)", flush=True)
