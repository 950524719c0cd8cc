"""Communication probe: measure the collectives the partitioner prices, on the node the job
runs on, before the plan is chosen (SURVEY.md §2.7 A7 "calibrated with measured kernel and
collective times", §7.3 risk 7).

`probe_comm(world)` is collective over the world group (every rank calls it). It times, with
all groups of a size running at once — exactly the contention a dp x tp layout sees:
  * RCCL all-reduce over groups of 2, 4, ... world ranks (message sizes 16 KiB .. 32 MiB);
  * the IPC all-reduce kernel (parallel/custom_allreduce.py), one-shot and two-shot, over
    the same group sizes (up to its 8 MiB buffer);
  * the butterfly all-reduce (parallel/butterfly.py: recursive halving + doubling over
    point-to-point transfers) over the same power-of-two groups (BFLY_PROBE_BUTTERFLY: its
    pairwise steps open a point-to-point communicator per rank pair on first use, so it is
    timed on request, not on every job start);
  * RCCL send/recv between rank pairs (pipeline boundary hops);
  * RCCL all-to-all over the world (EP dispatch).
Each timing is the median of several back-to-back calls, then the MAX over ranks, so every
rank holds the same table and the (deterministic) partition search picks the same plan on
every rank. The table feeds `Hardware.with_comm_table` (partition/hw.py); the cost model
interpolates it log-log instead of using guessed latencies. Nothing runs on 1 rank.
"""
from __future__ import annotations

import logging
import statistics
import time
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger("butterfly_amd.probe")

AR_SIZES = (16 << 10, 256 << 10, 1 << 20, 4 << 20, 8 << 20, 32 << 20)
P2P_SIZES = (64 << 10, 1 << 20, 16 << 20)
A2A_SIZES = (256 << 10, 4 << 20)


def _time(fn, iters: int, device) -> float:
    """Median seconds of one call (each call synchronised; a warm-up call first)."""
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)  # noqa: E731
    fn()
    sync()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        sync()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def _groups_of(world: int, n: int) -> list:
    return [list(range(i, i + n)) for i in range(0, world, n)]


def probe_comm(world: int, device: Optional[torch.device] = None, iters: int = 8,
               custom_ar: bool = True, butterfly: Optional[bool] = None) -> dict:
    """Run the probe (collective); returns {"all_reduce": {impl: {n: [[bytes, s], ...]}},
    "p2p": [[bytes, s], ...], "all_to_all": {n: [[bytes, s], ...]}, "seconds": wall}."""
    if world <= 1 or not dist.is_initialized():
        return {}
    if device is None:
        if dist.get_backend() != "nccl":
            return {}
        device = torch.device("cuda", torch.cuda.current_device())
    custom_ar = custom_ar and device.type == "cuda"
    if butterfly is None:
        from ..utils import flags

        butterfly = flags.get("BFLY_PROBE_BUTTERFLY")
    t_start = time.perf_counter()
    rank = dist.get_rank()
    sizes_n = [n for n in (2, 4, 8, 16) if n <= world and world % n == 0]
    ar: dict = {"rccl": {}, "oneshot": {}, "twoshot": {}, "butterfly": {}}
    keys = []          # (kind, impl, n, bytes) in a fixed order on every rank
    vals = []
    for n in sizes_n:
        pgs = [dist.new_group(g) if n < world else dist.group.WORLD for g in _groups_of(world, n)]
        mine = pgs[rank // n]
        for nb in AR_SIZES:
            t = torch.ones(nb // 2, dtype=torch.bfloat16, device=device)
            keys.append(("ar", "rccl", n, nb))
            vals.append(_time(lambda: dist.all_reduce(t, group=mine), iters, device))
        if custom_ar and n in (2, 4, 8):
            from .custom_allreduce import CustomAllReduce

            car = CustomAllReduce(_groups_of(world, n)[rank // n], rank % n, mine, max_bytes=8 << 20, device=device)
            for two in (False, True):
                for nb in AR_SIZES:
                    rows = max(1, nb // (2 * 8192))
                    ok = car.ok and rows * 8192 * 2 <= car.cap and not (two and n < 4)
                    keys.append(("ar", "twoshot" if two else "oneshot", n, nb))
                    if not ok:
                        vals.append(-1.0)
                        continue
                    t = torch.ones(rows, 8192, dtype=torch.bfloat16, device=device)
                    vals.append(_time(lambda: car.all_reduce_(t, two_shot=two), iters, device))
            car.close()
        if butterfly and n & (n - 1) == 0:
            from .butterfly import butterfly_all_reduce_

            grp = _groups_of(world, n)[rank // n]
            for nb in AR_SIZES:
                t = torch.ones(nb // 2, dtype=torch.bfloat16, device=device)
                keys.append(("ar", "butterfly", n, nb))
                vals.append(_time(lambda: butterfly_all_reduce_(t, grp, mine), iters, device))
    # pipeline hops: even ranks send to odd ranks (all pairs at once)
    peer = rank ^ 1
    for nb in P2P_SIZES:
        t = torch.ones(nb // 2, dtype=torch.bfloat16, device=device)

        def hop():
            if rank % 2 == 0:
                dist.send(t, peer)
            else:
                dist.recv(t, peer)
        keys.append(("p2p", "rccl", 2, nb))
        vals.append(_time(hop, iters, device) if peer < world else -1.0)
    for nb in A2A_SIZES:
        x = torch.ones(nb // 2, dtype=torch.bfloat16, device=device)
        y = torch.empty_like(x)
        keys.append(("a2a", "rccl", world, nb))
        vals.append(_time(lambda: dist.all_to_all_single(y, x), iters, device))
    # one table on every rank: the max over ranks of every entry
    v = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    vals = v.tolist()
    out: dict = {"all_reduce": ar, "p2p": [], "all_to_all": {}, "world": world}
    for (kind, impl, n, nb), s in zip(keys, vals):
        if s < 0:
            continue
        if kind == "ar":
            ar[impl].setdefault(n, []).append([nb, s])
        elif kind == "p2p":
            out["p2p"].append([nb, s])
        else:
            out["all_to_all"].setdefault(n, []).append([nb, s])
    out["seconds"] = time.perf_counter() - t_start
    if rank == 0:
        log.info("comm probe (%d ranks) took %.1f s", world, out["seconds"])
    return out


def ar_policy(table: dict) -> dict:
    """Per group size n: which all-reduce implementation to run by message size, read off the
    measurements: {"twoshot_min": bytes from which two-shot beats one-shot (inf: never),
    "ipc_max": largest message for which the IPC kernel beats RCCL (0: never),
    "butterfly": [lo, hi] message sizes on which the butterfly beats whatever else would run
    (the longest such run of measured sizes; None: never)}."""
    out = {}
    ar = (table or {}).get("all_reduce") or {}
    get = lambda impl, n: {int(b): t for b, t in ((ar.get(impl) or {}).get(n) or (ar.get(impl) or {}).get(str(n)) or [])}  # noqa: E731
    for n in sorted({int(k) for d in ar.values() for k in d}):
        rc, one, two = get("rccl", n), get("oneshot", n), get("twoshot", n)
        sizes = sorted(set(one) | set(two))
        two_min = float("inf")
        for s in reversed(sizes):          # two-shot from the smallest size on which it keeps winning
            if s in two and s in one and two[s] < one[s]:
                two_min = s
            else:
                break
        ipc_max = 0
        for s in sizes:                    # IPC while it beats RCCL, from small messages up
            ipc = two.get(s) if s >= two_min else one.get(s)
            if ipc is None or (s in rc and rc[s] < ipc):
                break
            ipc_max = s
        bf = get("butterfly", n)
        run, best = [], []
        for s in sorted(set(rc) | set(bf)):
            other = [v for v in (rc.get(s), (two.get(s) if s >= two_min else one.get(s)) if s <= ipc_max else None)
                     if v is not None]
            if s in bf and other and bf[s] < min(other):
                run.append(s)
                best = run if len(run) > len(best) else best
            else:
                run = []
        out[n] = {"twoshot_min": two_min, "ipc_max": ipc_max, "butterfly": [best[0], best[-1]] if best else None}
    return out


def apply_policy(policy: dict, tp: int) -> dict:
    """Set the runtime's all-reduce routing for a TP group of `tp` ranks from the measured
    policy (environment flags read when the communicator is built). Returns what was set."""
    import os

    pol = policy.get(tp) or policy.get(str(tp))
    if not pol:
        return {}
    env = {}
    if pol["ipc_max"] <= 0:
        env["BFLY_CUSTOM_AR"] = "0"
    else:
        env["BFLY_CUSTOM_AR_MAX_BYTES"] = str(int(pol["ipc_max"]))
        env["BFLY_CUSTOM_AR_2SHOT_BYTES"] = "0" if pol["twoshot_min"] == float("inf") else str(int(pol["twoshot_min"]))
    if pol.get("butterfly"):
        lo, hi = pol["butterfly"]
        env["BFLY_AR_BUTTERFLY"] = f"{int(tp)}@{int(lo)}:{int(hi)}"   # measured for groups of tp ranks
    os.environ.update(env)
    return env


def summarize(table: dict) -> dict:
    """Compact per-size microseconds for the benchmark JSON."""
    if not table:
        return {}
    us = lambda pts: {f"{nb >> 10}KiB": round(s * 1e6, 1) for nb, s in pts}  # noqa: E731
    return {"all_reduce": {impl: {str(n): us(p) for n, p in d.items()} for impl, d in table["all_reduce"].items()},
            "p2p": us(table["p2p"]), "all_to_all": {str(n): us(p) for n, p in table["all_to_all"].items()},
            "probe_seconds": round(table.get("seconds", 0.0), 2),
            "ar_policy": {str(n): {k: (None if v == float("inf") else v) for k, v in d.items()}
                          for n, d in ar_policy(table).items()}}
