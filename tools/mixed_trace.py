#!/usr/bin/env python3
"""Chunked prefill over cached prefixes, for a kernel trace ("a mixed-step
trace shows no at::native kernel").

One engine on cuda:0 (default Llama-3-8B, random weights) with mixed chunked prefill and prefix
caching: a first request fills the prefix cache with a shared prompt head, then a batch of
requests that start with that head prefill only their tails — in chunks smaller than a prompt,
beside the decode rows of the requests already running. Every such chunk attends to a paged
prefix (its cached head, or its own earlier chunks): ops.attn_prefill_paged. Prints the
engine's prefix-hit and step statistics; run it under rocprofv3 and summarise the trace with
`--summary CSV` (every kernel of the run, at::native ones flagged).

usage: rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_mixed -o run -- \\
           python3 tools/mixed_trace.py
       python3 tools/mixed_trace.py --summary gpurun_out/prof_mixed/run_kernel_trace.csv"""
import argparse
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summary(path: str) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    cnt, dur = collections.Counter(), collections.Counter()
    for r in rows:
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        cnt[name] += 1
        dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("| kernel | calls | total us | torch (at::native) |")
    print("|---|---|---|---|")
    for name, n in sorted(cnt.items(), key=lambda kv: -dur[kv[0]]):
        print(f"| {name} | {n} | {dur[name]:.1f} | {'YES' if 'at::native' in name else ''} |")
    nat = {k: v for k, v in cnt.items() if "at::native" in k}
    print(f"\n{len(rows)} dispatches; at::native kernels: {sum(nat.values())} "
          f"({', '.join(f'{k} x{v}' for k, v in nat.items()) or 'none'})")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--head", type=int, default=1024, help="shared prompt head (cached prefix)")
    ap.add_argument("--tail", type=int, default=700, help="per-request prompt tail")
    ap.add_argument("--requests", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=512, help="max_prefill_tokens per step")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--summary", default=None, help="summarise a rocprofv3 kernel_trace.csv and exit")
    a = ap.parse_args()
    if a.summary:
        summary(a.summary)
        return 0
    import torch

    from butterfly_amd.config import EngineConfig, ModelConfig
    from butterfly_amd.engine.engine import LLMEngine
    from butterfly_amd.engine.sampler import SamplingParams
    from butterfly_amd.parallel.mesh import Mesh

    cfg = ModelConfig.from_preset(a.model)
    ecfg = EngineConfig(max_batch=32, max_seq_len=a.head + a.tail + 64, max_prefill_tokens=a.chunk,
                        kv_cache_tokens=(a.requests + 2) * (a.head + a.tail + 64), use_graphs=a.device != "cpu",
                        mixed_prefill=True, prefix_caching=True, async_decode=False)
    eng = LLMEngine(cfg, Mesh(), ecfg, device=a.device)
    g = torch.Generator().manual_seed(0)
    head = torch.randint(0, cfg.vocab_size, (a.head,), generator=g).tolist()
    eng.add_request(head + torch.randint(0, cfg.vocab_size, (a.tail,), generator=g).tolist(),
                    SamplingParams(max_tokens=24, ignore_eos=True))
    kinds = collections.Counter()
    for _ in range(6):                       # the first request's chunks register the head's pages
        kinds[eng.step().kind] += 1
    for _ in range(a.requests):
        eng.add_request(head + torch.randint(0, cfg.vocab_size, (a.tail,), generator=g).tolist(),
                        SamplingParams(max_tokens=8, ignore_eos=True))
    while eng.has_unfinished():
        kinds[eng.step().kind] += 1
    if a.device != "cpu":
        torch.cuda.synchronize()
    print(json.dumps({"model": cfg.name, "steps": dict(kinds),
                      "prefix_hit_tokens": int(eng.scheduler.prefix_hit_tokens),
                      "mixed": True, "chunk": a.chunk}), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
