#!/usr/bin/env python3
"""Per-GPU compute time of one tensor-parallel rank's decode step, on ONE GPU.

Builds TP rank 0's shard of the model (Shard(tp_size=tp)) with a single-rank communicator, so
every TP all-reduce is a no-op and the step time is the rank's kernels only: the compute side
of a tp-way decode step at `batch` sequences per replica (weak scaling: batch = 64 x tp). Each
step is one hipGraph replay of the whole forward (all layers, LM head shard), timed with
events. Prints the measurement next to the partitioner's compute-only estimate for the same
shard (partition/costmodel.py without its collective ops), so the cost model's GEMM / attention
pricing at the TP batch sizes can be checked against the kernels without a multi-GPU node.

usage: python tools/shard_bench.py --model llama3-70b --tp 2 [--batch 128] [--ctx 1040] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402
from butterfly_amd.config import ModelConfig  # noqa: E402
from butterfly_amd.engine.batch import ForwardBatch  # noqa: E402
from butterfly_amd.models.shard import Shard  # noqa: E402
from butterfly_amd.models.transformer import TransformerLM  # noqa: E402
from butterfly_amd.parallel.comm import Communicator  # noqa: E402
from butterfly_amd.partition.costmodel import CostModel  # noqa: E402
from butterfly_amd.partition.hw import MI355X  # noqa: E402
from butterfly_amd.utils import flags  # noqa: E402


def compute_estimate(cfg, tp: int, batch: int, ctx: int) -> float:
    """Cost-model seconds of the shard's decode step with the collectives left out."""
    cm = CostModel(cfg, MI355X)
    ir = cm._ir(tp, 1)
    t = 0.0
    for layer in ir.layers:
        cm._cur_ep = 1
        t += sum(cm.op_time(o, batch, ctx, True, batch, tp) for o in layer.ops if o.kind != "collective")
    first, last = cm.embed_head_time(batch, batch, tp)
    return t + first + last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0, help="sequences per replica (default 64 x tp)")
    ap.add_argument("--ctx", type=int, default=1040)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    assert torch.cuda.is_available() and ops.load_library(), "needs a GPU and the built kernels"
    cfg = ModelConfig.from_preset(a.model)
    B, tp, ctx = a.batch or 64 * a.tp, a.tp, a.ctx
    t0 = time.perf_counter()
    model = TransformerLM(cfg, Shard(tp_rank=0, tp_size=tp), device="cuda", comm=Communicator.single())
    model.init_random(seed=0)
    packed_gb = 0.0
    if flags.get("BFLY_PACKED_DECODE"):   # as the engine does when HBM allows (all of it fits a shard)
        kinds = [k.strip() for k in flags.get("BFLY_PACKED_KINDS").split(",") if k.strip()]
        packed_gb = model.pack_decode_weights(kinds=kinds) / 1e9
    BS = 32
    nb = -(-(ctx + 1) // BS)
    kv = model.allocate_kv_cache(B * nb, BS)
    dev = "cuda"
    tables = torch.arange(B * nb, dtype=torch.int32, device=dev).view(B, nb)
    pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
    slots = tables[:, (ctx - 1) // BS] * BS + (ctx - 1) % BS
    fb = ForwardBatch(input_ids=torch.randint(0, cfg.vocab_size, (B,), dtype=torch.int32, device=dev),
                      positions=pos, slots=slots.contiguous(), is_prefill=False, block_tables=tables,
                      ctx_lens=torch.full((B,), ctx, dtype=torch.int32, device=dev), max_ctx=ctx + 1)
    ops.reserve_workspace(dev, B, max(cfg.vocab_size // tp, 4 * cfg.intermediate_size // tp, 16384),
                          max(cfg.hidden_size, cfg.intermediate_size // tp), B, ctx + 1,
                          max(1, cfg.num_kv_heads // tp), cfg.head_dim, shapes=model.gemm_shapes())
    print(f"[shard_bench] {cfg.name} tp{tp} rank-0 shard, batch {B}, ctx {ctx}: "
          f"{model.local_bytes() / 1e9:.1f} GB weights, built in {time.perf_counter() - t0:.1f}s", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            model.forward(fb, kv)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        model.forward(fb, kv)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(a.steps):
        st.record()
        g.replay()
        en.record()
        en.synchronize()
        times.append(st.elapsed_time(en))
    times.sort()
    ms = times[len(times) // 2]
    est = compute_estimate(cfg, tp, B, ctx) * 1e3
    print(json.dumps({"model": cfg.name, "tp": tp, "batch": B, "ctx": ctx, "ms_per_step_p50": round(ms, 3),
                      "ms_min": round(times[0], 3), "tokens_per_s_per_replica": round(B / ms * 1e3, 1),
                      "costmodel_compute_ms": round(est, 3), "ratio_measured_over_model": round(ms / est, 3),
                      "packed_decode_weights_gb": round(packed_gb, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
