#!/usr/bin/env python3
"""The real tensor-parallel decode path at PRODUCTION dimensions, ranks sharing ONE MI355X.

The Llama-3-70B preset cut to 2 layers (every projection, the 128k-vocab embedding and LM head
at full size), TP = world (2 or 4) over gloo with the IPC all-reduce (BFLY_IPC_SHARED_DEVICE=1,
tests only), at the weak-scaling decode batch (64 sequences per GPU: 128 rows at tp2, 256 at
tp4). What runs is what a tp2 / tp4 node runs: the shard's QKV / O / gate-up / down projections
on the mid-M plans the table picks for those shapes, the O and down projections' split-K slabs
deferred into the IPC all-reduce, which reduces them while publishing and fuses the residual add
and RMSNorm (8192 columns), the vocab-parallel embedding / LM head. Checked:

* prefill logits (a short prompt per sequence) and the decode step's logits, gathered over TP,
  against an fp32 PyTorch model holding the same weights (ops.reference_mode: plain torch ops,
  no kernel of ours), on rank 0;
* the decode step captured in a hipGraph and replayed: bitwise equal to the eager step;
* the IPC all-reduce actually took the deferred slabs (its call counter moved, no RCCL / gloo
  all-reduce inside the decode step).

usage: python -m butterfly_amd launch -n 2 -- python tools/gpu_tp_fullsize.py [preset] [rows_per_gpu]
"""
import dataclasses
import os
import sys

os.environ.setdefault("BFLY_IPC_SHARED_DEVICE", "1")   # ranks share cuda:0 (refused in production)
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402
from butterfly_amd.config import ModelConfig  # noqa: E402
from butterfly_amd.engine.batch import make_decode_batch, make_prefill_batch  # noqa: E402
from butterfly_amd.models import Shard, build_model  # noqa: E402
from butterfly_amd.parallel.comm import Communicator  # noqa: E402
from butterfly_amd.parallel.mesh import Mesh  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "-" else "llama3-70b"
per_gpu = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("gloo", rank=rank, world_size=world)
mesh = Mesh(tp=world)
comm = Communicator.from_mesh(mesh)
fails = []
if comm.custom_ar is None:
    fails.append("IPC all-reduce not active")
cfg = dataclasses.replace(ModelConfig.from_preset(preset), num_layers=2)
V, BS = cfg.vocab_size, 32
m = build_model(cfg, Shard(tp_rank=rank, tp_size=world), device=dev, dtype=torch.bfloat16, comm=comm)
m.init_random(seed=5)
if not m.defer_reduce:
    fails.append("split-K reduces are not deferred into the all-reduce")
B, P = per_gpu * world, 16
gen = torch.Generator().manual_seed(11)
prompts = [torch.randint(0, V, (P,), generator=gen).tolist() for _ in range(B)]
nb = (P + 1 + BS - 1) // BS + 1
tables = [list(range(i * nb, (i + 1) * nb)) for i in range(B)]
slots = [[tables[i][j // BS] * BS + j % BS for j in range(P)] for i in range(B)]
kv = m.allocate_kv_cache(B * nb + 1, BS)
ops.reserve_workspace(dev, max_tokens=B * P, max_n=max(V // world, 2 * cfg.intermediate_size // world, 16384),
                      max_k=max(cfg.hidden_size, cfg.intermediate_size // world), max_batch=B, max_ctx=nb * BS,
                      num_kv_heads=max(1, cfg.num_kv_heads // world), head_dim=cfg.head_dim, shapes=m.gemm_shapes())


def gather_vocab(lg):
    """[rows, V/tp] logits shard -> [rows, V] on every rank (gloo: through the host)."""
    parts = [torch.empty_like(lg).cpu() for _ in range(world)]
    dist.all_gather(parts, lg.contiguous().cpu())
    return torch.cat(parts, 1)[:, :V].float()


fb = make_prefill_batch(prompts, slots).to(dev)
lp = gather_vocab(m.forward(fb, kv))
toks = [int(t) for t in lp.argmax(-1)]          # identical on every rank (gathered logits)
pos = [P] * B
sl = [tables[i][P // BS] * BS + P % BS for i in range(B)]
db = make_decode_batch(toks, pos, sl, tables, nb, nb * BS).to(dev)
kv_before = [(k.clone(), v.clone()) for k, v in kv]
calls0 = comm.stats["calls"]
ld = m.forward(db, kv)
torch.cuda.synchronize()
eager = ld.clone()
kv_eager = [(k.clone(), v.clone()) for k, v in kv]
ar_calls = comm.stats["calls"] - calls0
if ar_calls != 2 * cfg.num_layers + 1:
    fails.append(f"decode step issued {ar_calls} all-reduces, want {2 * cfg.num_layers + 1}")

# hipGraph capture of the decode step (every all-reduce on the IPC kernel: capturable), replay
for (k, v), (k0, v0) in zip(kv, kv_before):
    k.copy_(k0)
    v.copy_(v0)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    m.forward(db, kv)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out_g = m.forward(db, kv)
for it in range(3):
    for (k, v), (k0, v0) in zip(kv, kv_before):
        k.copy_(k0)
        v.copy_(v0)
    g.replay()
    torch.cuda.synchronize()
    if not torch.equal(out_g, eager):
        fails.append(f"graph replay {it} differs from eager: {(out_g.float() - eager.float()).abs().max().item():.3e}")
        break
if not all(torch.equal(k, ke) and torch.equal(v, ve) for (k, v), (ke, ve) in zip(kv, kv_eager)):
    fails.append("graph replay KV appends differ from eager")
ld_full = gather_vocab(eager)

if rank == 0:
    full = build_model(cfg, device=dev, dtype=torch.bfloat16)
    full.init_random(seed=5)        # the partition-independent hash init: the same global weights
    with ops.reference_mode():
        r = build_model(cfg, device=dev, dtype=torch.float32)
        for k, v in full.p.items():
            r.p[k].copy_(v.float())
        del full
        kr = r.allocate_kv_cache(B * nb + 1, BS)
        lr = r.forward(fb, kr)[:, :V].float().cpu()
        dr = r.forward(db, kr)[:, :V].float().cpu()
    rel_p = ((lp - lr).norm() / lr.norm()).item()
    rel_d = ((ld_full - dr).norm() / dr.norm()).item()
    if not rel_p < 2e-2:
        fails.append(f"prefill logits rel err {rel_p:.3e}")
    if not rel_d < 3e-2:
        fails.append(f"decode logits rel err {rel_d:.3e}")
    shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * cfg.head_dim // world, cfg.hidden_size),
              "o": (cfg.hidden_size, cfg.num_heads * cfg.head_dim // world),
              "gate_up": (2 * cfg.intermediate_size // world, cfg.hidden_size),
              "down": (cfg.hidden_size, cfg.intermediate_size // world)}
    plans = []
    for name, (n, k) in shapes.items():
        pl = ops.gemm_plan(B, n, k)
        plans.append(f"{name} {pl['kind']} {pl['bm']}x{pl['bn']} sk{pl['splitk']}")
    print(f"tp{world} {preset} (2 layers) rows {B}: prefill rel {rel_p:.2e} decode rel {rel_d:.2e} "
          f"all-reduces/step {ar_calls} plans: " + ", ".join(plans), flush=True)
ok = not fails
print(f"rank {rank}: tp{world} fullsize -> {'PASS' if ok else 'FAIL ' + '; '.join(fails)}", flush=True)
dist.barrier()
comm.close()
dist.destroy_process_group()
sys.exit(0 if ok else 1)
