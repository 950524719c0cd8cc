#!/usr/bin/env python3
"""Context-parallel prefill on ONE GPU: N ranks share cuda:0 over gloo (RCCL refuses two ranks
on one device); each runs its chunk of the prompts through the HIP kernels (flash prefill with
LSE, LSE merge) and the last-token logits must match a single-process prefill.
usage: python -m butterfly_amd launch -n 2 -- python tools/gpu_cp_check.py [preset|-] [ring|ulysses]"""
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
