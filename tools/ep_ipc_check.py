#!/usr/bin/env python3
"""GPU check of the byte-minimal EP dispatch (csrc/kernels/ep_ipc.hip, parallel/ep_ipc.py).

N ranks share cuda:0 (gloo carries only the hipIpc handle exchange and the reference data):
every rank routes random tokens (top-k experts over N ranks, empty rows, graph-padding rows)
through the IPC buffers, the expert rank "computes" y = x * (rank + 1) on its received block,
and the returned rows are combined. Checked bitwise against the fixed-capacity all-to-all
layout (ops.reference.ep_pack / ep_combine on every source's inputs, gathered over gloo):
received rows, expert ids and weights, the combined output, the link-row statistics; then the
same exchange captured in a hipGraph and replayed with new inputs. On a multi-GPU node the same
script runs one rank per GPU.
usage: python -m butterfly_amd launch -n 4 -- python tools/ep_ipc_check.py [--bench]"""
import os
import sys

# ranks share cuda:0 here: opt in to shared-GPU IPC groups (refused in production)
os.environ.setdefault("BFLY_IPC_SHARED_DEVICE", "1")
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd.ops import reference as ref  # noqa: E402
from butterfly_amd.parallel.ep_ipc import EpIpc  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
local = int(os.environ.get("LOCAL_RANK", "0"))
dev_idx = local if torch.cuda.device_count() > local and os.environ.get("BFLY_CAR_SHARED") != "1" else 0
torch.cuda.set_device(dev_idx)
dev = torch.device("cuda", dev_idx)
dist.init_process_group("gloo", rank=rank, world_size=world)
H, K, CAPMAX, El = 1024, 2, 64, 2
ipc = EpIpc(list(range(world)), rank, dist.group.WORLD, CAPMAX, H, K, device=dev)
fails = []
if not ipc.ok:
    print(f"rank {rank}: EP IPC self-test FAILED", flush=True)
    sys.exit(1)


def inputs(r, T, salt):
    g = torch.Generator().manual_seed(7919 * salt + r)
    x = torch.randn(T, H, generator=g).to(torch.bfloat16)
    ids = torch.randint(-1, world * El, (T, K), generator=g, dtype=torch.int32)
    w = torch.rand(T, K, generator=g)
    slots = torch.arange(T, dtype=torch.int32)
    if T > 2:
        slots[T // 2] = -1
    return x, ids, w, slots


def expected(T, salt):
    """This rank's received block and each source's combined output, from the all-to-all
    layout of every source's inputs (rank d's expert output = its received rows * (d + 1))."""
    packs = [ref.ep_pack(*inputs(r, T, salt), El, world, CAPMAX) for r in range(world)]
    recv_x = torch.cat([p[0][rank * CAPMAX:(rank + 1) * CAPMAX] for p in packs])
    recv_m = torch.cat([p[1][rank * CAPMAX:(rank + 1) * CAPMAX] for p in packs])
    sent = [int((p[2] >= 0).sum()) for p in packs]
    send, meta, slot = packs[rank]
    back = torch.cat([(send[d * CAPMAX:(d + 1) * CAPMAX].float() * (d + 1)).to(torch.bfloat16)
                      for d in range(world)])
    out = ref.ep_combine(back, slot)
    counts = [int((packs[s][2][:, rank] >= 0).sum()) for s in range(world)]
    return recv_x, recv_m, out, counts, sent, slot


def exchange(x, ids, w, slots, T):
    """dispatch -> expert step -> return + combine. The received views are snapshotted before
    the combine: once every rank has combined, peers may dispatch the next call into this
    rank's buffer (in the model the expert FFN has consumed them by then)."""
    r = ipc.dispatch(x, ids, w, slots, El, T)
    snap = type(r)(r.x.clone(), r.ids.clone(), r.w.clone(), r.slot, r.T, r.path)
    y = (r.x.float() * (rank + 1)).to(torch.bfloat16)
    return snap, ipc.combine(y, r)


def check(tag, T, salt, r, out):
    recv_x, recv_m, want, counts, sent, slot = expected(T, salt)
    gx, gi, gw = r.x.cpu(), r.ids.cpu(), r.w.cpu()
    for s in range(world):
        n = counts[s]
        blk = slice(s * CAPMAX, s * CAPMAX + n)
        if not torch.equal(gx[blk], recv_x[blk]):
            fails.append(f"{tag} T={T}: rows from rank {s} differ")
    if not torch.equal(gi, recv_m[:, :K].contiguous().view(torch.int32)) or not torch.equal(gw, recv_m[:, K:]):
        fails.append(f"{tag} T={T}: expert ids / weights differ")
    pos = torch.where(slot >= 0, slot - torch.arange(world, dtype=torch.int32) * CAPMAX, slot)
    if not torch.equal(r.slot.cpu(), pos):
        fails.append(f"{tag} T={T}: slot map differs")
    if not torch.equal(out.cpu(), want):
        fails.append(f"{tag} T={T}: combined output differs (max err "
                     f"{(out.cpu().float() - want.float()).abs().max().item():.3e})")
    return sum(c for s, c in enumerate(counts) if s != rank), sum(
        int((slot[:, d] >= 0).sum()) for d in range(world) if d != rank)


# 1. eager, several shapes (T <= CAPMAX), link rows counted by the kernels
base = torch.ops.bfly.ep_ipc_stats(ipc._ptr)
exp_out = exp_back = 0
for salt, T in enumerate([1, 5, 37, 64]):
    x, ids, w, slots = (t.to(dev) for t in inputs(rank, T, salt))
    r, out = exchange(x, ids, w, slots, T)
    torch.cuda.synchronize()
    back_rows, out_rows = check("eager", T, salt, r, out)
    exp_out += out_rows
    exp_back += back_rows
now = torch.ops.bfly.ep_ipc_stats(ipc._ptr)
if [now[0] - base[0], now[1] - base[1]] != [exp_out, exp_back]:
    fails.append(f"link rows {now[0] - base[0]}/{now[1] - base[1]} != {exp_out}/{exp_back}")

# 2. hipGraph capture / replay with new inputs in the static buffers
T = 48
sx = torch.zeros(T, H, dtype=torch.bfloat16, device=dev)
si = torch.zeros(T, K, dtype=torch.int32, device=dev)
sw = torch.zeros(T, K, device=dev)
ss = torch.zeros(T, dtype=torch.int32, device=dev)
for t, v in zip((sx, si, sw, ss), inputs(rank, T, 100)):
    t.copy_(v)
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    exchange(sx, si, sw, ss, T)              # warm-up on the capture stream
torch.cuda.current_stream().wait_stream(st)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    gr, gout = exchange(sx, si, sw, ss, T)
for it in range(3):
    salt = 200 + it
    for t, v in zip((sx, si, sw, ss), inputs(rank, T, salt)):
        t.copy_(v)
    g.replay()
    torch.cuda.synchronize()
    check(f"graph replay {it}", T, salt, gr, gout)
if ipc.error():
    fails.append(f"device error word {ipc.error()}")

# 4. prefill-sized dispatch (device scan route, counts in the receivers' headers, no empty-row
#    markers): ranks send different token counts (one sends none); received rows, counts,
#    slots and the combined output against the all-to-all layout at the prefill capacity
PCAP = 1536
pipc = EpIpc(list(range(world)), rank, dist.group.WORLD, PCAP, H, K, device=dev)
if not pipc.ok:
    fails.append("prefill EP IPC self-test failed")
else:
    for salt, base_t in ((400, 1200), (401, 7)):
        Ts = [0 if (r == world - 1 and salt == 400) else base_t + 37 * r for r in range(world)]
        ins = [inputs(r, Ts[r], salt) for r in range(world)]
        packs = [ref.ep_pack(x_, i_, w_, None, El, world, PCAP) for x_, i_, w_, _ in ins]
        x, ids, w, _ = (t.to(dev) for t in ins[rank])
        r = pipc.dispatch_prefill(x, ids, w, El)
        counts = r.counts.cpu().tolist()
        want_counts = [int((packs[s_][2][:, rank] >= 0).sum()) for s_ in range(world)]
        if counts != want_counts:
            fails.append(f"prefill T={Ts}: counts {counts} != {want_counts}")
        gx, gi = r.x.cpu(), r.ids.cpu()
        for s_ in range(world):
            n = want_counts[s_]
            blk = slice(s_ * PCAP, s_ * PCAP + n)
            if not torch.equal(gx[blk], packs[s_][0][rank * PCAP:rank * PCAP + n]):
                fails.append(f"prefill T={Ts}: rows from rank {s_} differ")
            if not torch.equal(gi[blk], packs[s_][1][rank * PCAP:rank * PCAP + n, :K].contiguous().view(torch.int32)):
                fails.append(f"prefill T={Ts}: ids from rank {s_} differ")
        send, meta, slot = packs[rank]
        pos = torch.where(slot >= 0, slot - torch.arange(world, dtype=torch.int32) * PCAP, slot)
        if not torch.equal(r.slot.cpu(), pos):
            fails.append(f"prefill T={Ts}: slot map differs")
        y = (r.x.float() * (rank + 1)).to(torch.bfloat16)
        out = pipc.combine(y, r)
        torch.cuda.synchronize()
        back = torch.cat([(send[d * PCAP:(d + 1) * PCAP].float() * (d + 1)).to(torch.bfloat16) for d in range(world)])
        if not torch.equal(out.cpu(), ref.ep_combine(back, slot)):
            fails.append(f"prefill T={Ts}: combined output differs")
    if pipc.error():
        fails.append(f"prefill device error word {pipc.error()}")
    pipc.close()

# 3. timing: one decode-sized exchange (dispatch + wait + return + combine), expert step elided
if "--bench" in sys.argv:
    for T in (16, 64):
        x, ids, w, slots = (t.to(dev) for t in inputs(rank, T, 300))
        for _ in range(10):
            exchange(x, ids, w, slots, T)
        torch.cuda.synchronize()
        dist.barrier()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            exchange(x, ids, w, slots, T)
        torch.cuda.synchronize()
        if rank == 0:
            print(f"EP IPC exchange ep={world} T={T} H={H} k={K}: {(time.perf_counter() - t0) / n * 1e6:.1f} us",
                  flush=True)

ipc.close()
print(f"rank {rank}: EP IPC world={world} -> {'PASS' if not fails else 'FAIL ' + '; '.join(fails[:6])}", flush=True)
dist.destroy_process_group()
sys.exit(0 if not fails else 1)
