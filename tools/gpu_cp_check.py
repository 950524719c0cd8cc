#!/usr/bin/env python3
"""Context-parallel prefill on ONE GPU: N ranks share cuda:0 over gloo (RCCL refuses two ranks
on one device); each runs its chunk of the prompts through the HIP kernels (flash prefill with
LSE, LSE merge) and the last-token logits must match a single-process prefill.
With a third argument "engine", the serving engine's CP path is checked instead: Mesh(dp=N)
replicas with cp_prefill_min_tokens set prefill each other's long prompts together, the owner's
cache collects the K/V: the first tokens must equal a single-process engine's and the owner's
cached K/V of every long prompt (first and last layer) must match the single engine's pages
(full sequences are reported; bf16 near ties of random weights may split them later).
usage: python -m butterfly_amd launch -n 2 -- python tools/gpu_cp_check.py [preset|-] [ring|ulysses] [engine]"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd.config import ModelConfig  # noqa: E402
from butterfly_amd.engine.batch import make_prefill_batch  # noqa: E402
from butterfly_amd.models import build_model  # noqa: E402
from butterfly_amd.parallel.context_parallel import cp_prefill  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "-" else "llama-small"
attn = sys.argv[2] if len(sys.argv) > 2 else "ring"
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo", rank=rank, world_size=world)
cfg = ModelConfig.from_preset(preset)
if len(sys.argv) > 3 and sys.argv[3] == "engine":
    from butterfly_amd.config import EngineConfig  # noqa: E402
    from butterfly_amd.engine.engine import LLMEngine  # noqa: E402
    from butterfly_amd.engine.sampler import SamplingParams  # noqa: E402
    from butterfly_amd.parallel.comm import Communicator  # noqa: E402
    from butterfly_amd.parallel.mesh import Mesh  # noqa: E402

    mine = [[(37 * rank + 11 * j) % cfg.vocab_size + 1 for j in range(700 + 150 * rank)],
            [(5 * j + rank) % cfg.vocab_size + 1 for j in range(40)],
            [(29 * j + 3 * rank) % cfg.vocab_size + 1 for j in range(300)]]
    sp = SamplingParams(max_tokens=8, ignore_eos=True)

    def ecfg(cp_min):
        return EngineConfig(max_batch=8, max_seq_len=2048, kv_cache_tokens=8192, seed=5,
                            cp_prefill_min_tokens=cp_min, cp_attention=attn)

    def cached_kv(e, rid, L):
        """K/V of a sequence's first L cached tokens, first and last layer, from its pages."""
        bt = e.kv.manager.block_table(rid)
        BS = e.kv.block_size
        idx = torch.tensor([bt[p // BS] for p in range(L)], device="cuda:0")
        off = torch.tensor([p % BS for p in range(L)], device="cuda:0")
        out = []
        for li in (0, len(e.kv.layers) - 1):
            kc, vc = e.kv.layers[li]
            out.append(kc[idx, :, off, :].float())
            out.append(vc[idx, :, :, off].float())
        return out

    mesh = Mesh(dp=world)
    eng = LLMEngine(cfg, mesh, ecfg(256), comm=Communicator.from_mesh(mesh), device="cuda:0")
    rids = [eng.add_request(p, sp) for p in mine]
    got_kv = {}
    while eng.has_unfinished_global():
        eng.step()
        for r, p in zip(rids, mine):
            if len(p) >= 256 and r not in got_kv and eng.requests[r].output:
                got_kv[r] = cached_kv(eng, r, len(p))
    got = [eng.requests[r].output for r in rids]
    cp_tok = eng.metrics.counters.get("cp_prefill_tokens", 0)
    ref = LLMEngine(cfg, Mesh(), ecfg(0), device="cuda:0")
    rrids = [ref.add_request(p, sp) for p in mine]
    want_kv = {}
    while ref.has_unfinished():
        ref.step()
        for r, rr, p in zip(rids, rrids, mine):
            if len(p) >= 256 and r not in want_kv and ref.requests[rr].output:
                want_kv[r] = cached_kv(ref, rr, len(p))
    want = [ref.requests[r].output for r in rrids]
    kv_rel = max(((a - b).norm() / b.norm()).item() for r in got_kv for a, b in zip(got_kv[r], want_kv[r]))
    first = all(a[0] == b[0] for a, b in zip(got, want))
    full = sum(a == b for a, b in zip(got, want))
    ok = first and cp_tok > 0 and len(got_kv) == 2 and kv_rel < 2e-2
    print(f"rank {rank} engine cp{world} {attn}: cp prefill tokens {int(cp_tok)}, collected K/V rel err {kv_rel:.2e}, "
          f"first tokens equal {first}, sequences equal {full}/3 (bf16 near ties may differ later) "
          f"-> {'PASS' if ok else 'FAIL'}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)
prompts = [[(31 * i + 7 * j) % cfg.vocab_size + 1 for j in range(n)] for i, n in enumerate((1000, 333, 64, 3))]
m = build_model(cfg, device="cuda:0", dtype=torch.bfloat16)
m.init_random(5)
got = cp_prefill(m, prompts, list(range(world)), rank, dist.group.WORLD, attn=attn)
want = m.forward(make_prefill_batch(prompts, [[-1] * len(p) for p in prompts], device="cuda:0"), None)
torch.cuda.synchronize()
V = cfg.vocab_size
g, w = got[:, :V].float(), want[:, :V].float()
rel = ((g - w).norm() / w.norm()).item()
same = (g.argmax(-1) == w.argmax(-1)).float().mean().item()
ok = rel < 2e-2 and same == 1.0
print(f"rank {rank} cp{world} {attn} {preset}: logits rel err {rel:.2e}, argmax agree {same:.2f} -> {'PASS' if ok else 'FAIL'}",
      flush=True)
dist.barrier()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
