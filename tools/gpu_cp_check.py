#!/usr/bin/env python3
"""Context-parallel prefill on ONE GPU: N ranks share cuda:0 over gloo (RCCL refuses two ranks
on one device); each runs its chunk of the prompts through the HIP kernels (flash prefill with
LSE, LSE merge) and the last-token logits must match a single-process prefill.
With a third argument "engine", the serving engine's CP path is checked instead: Mesh(dp=N)
replicas with cp_prefill_min_tokens set prefill each other's long prompts together, the owner's
cache collects the K/V, and the first tokens (and, allowing a bf16 near tie, most full
sequences) must equal a single-process engine's.
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

    mesh = Mesh(dp=world)
    eng = LLMEngine(cfg, mesh, ecfg(256), comm=Communicator.from_mesh(mesh), device="cuda:0")
    got = eng.generate(mine, sp)
    cp_tok = eng.metrics.counters.get("cp_prefill_tokens", 0)
    want = LLMEngine(cfg, Mesh(), ecfg(0), device="cuda:0").generate(mine, sp)
    first = all(a[0] == b[0] for a, b in zip(got, want))
    full = sum(a == b for a, b in zip(got, want))
    ok = first and full >= 2 and cp_tok > 0
    print(f"rank {rank} engine cp{world} {attn}: cp prefill tokens {int(cp_tok)}, first tokens equal {first}, "
          f"sequences equal {full}/3 -> {'PASS' if ok else 'FAIL'}", flush=True)
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
