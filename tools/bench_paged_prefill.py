#!/usr/bin/env python3
"""Paged-prefix prefill attention (attention_paged.hip) at serving shapes: a chunk of C tokens
of each of S sequences over a cached prefix of P tokens, Llama-3-8B (32 q / 8 kv heads) and
-70B (64 / 8) head layouts, bf16 pages scattered over the pool. Device time per call and
causal TF/s (4 x q_tokens x keys_seen x 128 x Hq). BFLY_ATTN_PAGED_LDS=0 selects the register
kernel (the env is read once per process).
usage: python tools/bench_paged_prefill.py [--iters N]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from butterfly_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    D, BS = 128, 32
    res = {"lds": os.environ.get("BFLY_ATTN_PAGED_LDS", "1")}
    for name, Hq, Hkv, S, P, C in (("8b_1x512_p1024", 32, 8, 1, 1024, 512), ("8b_2x512_p1536", 32, 8, 2, 1536, 512),
                                   ("70b_1x512_p1024", 64, 8, 1, 1024, 512), ("70b_4x256_p4096", 64, 8, 4, 4096, 256)):
        L = P + C
        nb = (L + BS - 1) // BS
        pool = S * nb + 16
        kc = torch.randn(pool, Hkv, BS, D, device=dev).to(torch.bfloat16)
        vc = torch.randn(pool, Hkv, D, BS, device=dev).to(torch.bfloat16)
        tables = torch.randperm(pool, device=dev)[: S * nb].view(S, nb).to(torch.int32)
        q = torch.randn(S * C, Hq, D, device=dev).to(torch.bfloat16)
        cu = torch.arange(0, S * C + 1, C, dtype=torch.int32, device=dev)
        pos = torch.arange(P, P + C, dtype=torch.int32, device=dev).repeat(S)
        out = torch.empty_like(q)
        fn = lambda: ops.attn_prefill_paged(q, kc, vc, tables, cu, pos, C, D ** -0.5, out=out)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        flops = 4 * S * sum(P + i + 1 for i in range(C)) * D * Hq
        res[name] = {"us": round(us, 1), "TFps": round(flops / us / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
