#!/usr/bin/env python3
"""Time the EP step agreement (engine._ep_agree -> Communicator.all_reduce_max_int on the gloo
control plane: three host integers, MAX) at 2 / 4 / 8 ranks on CPU — the per-step host
round trip every expert-parallel rank makes. With the asynchronous engine
the host schedules step k+1 while the device runs step k, so this is hidden when it is well
below the step time (Mixtral 8x7B EP decode: ~18 ms per step).

Both paths: the gloo all-reduce, and the node-local shared-memory control plane
(parallel/shm_ctrl.py, BFLY_SHM_CTRL) that replaces it when the group's ranks share a host.
Also times the same agreement with the ranks' arrival skewed by a random 0-200 us of host work
(a rank's scheduling is not perfectly aligned with its peers'), since the all-reduce ends at
the last arrival.

usage: python tools/ctrl_plane_probe.py [--worlds 2,4,8] [--iters 2000]
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _probe(rank, world, iters):
    import torch
    import torch.distributed as dist

    from butterfly_amd.parallel.shm_ctrl import ShmCtrl

    g = dist.new_group(list(range(world)), backend="gloo")
    shm = ShmCtrl(list(range(world)), rank, g, "probe")
    vals = [rank, rank & 1, 1]

    def gloo_max():
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        return [int(v) for v in t.tolist()]

    def shm_max():
        return shm.max(vals)

    out = {}
    rng = random.Random(rank)
    for name, fn in (("gloo", gloo_max), ("shm", shm_max)):
        for _ in range(50):
            assert fn() == [world - 1, 1 if world > 1 else 0, 1]
        for skew in (0, 200):
            ts = []
            for _ in range(iters):
                if skew:
                    end = time.perf_counter() + rng.uniform(0, skew) * 1e-6
                    while time.perf_counter() < end:
                        pass
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e6)
            ts.sort()
            out[(name, skew)] = (statistics.median(ts), ts[int(0.99 * len(ts)) - 1])
    dist.barrier(group=g)
    shm.close()
    return out


def main():
    from tests.dist_utils import run_world

    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args()
    for w in (int(x) for x in a.worlds.split(",")):
        res = run_world(_probe, w, a.iters, timeout=600)
        for name in ("gloo", "shm"):
            for skew in (0, 200):
                p50 = max(x[(name, skew)][0] for x in res)
                p99 = max(x[(name, skew)][1] for x in res)
                print(json.dumps({"path": name, "ranks": w, "arrival_skew_us": f"0-{skew}", "p50_us": round(p50, 1),
                                  "p99_us": round(p99, 1)}), flush=True)


if __name__ == "__main__":
    main()
