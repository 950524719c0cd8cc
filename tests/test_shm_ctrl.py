"""Node-local shared-memory control plane (parallel/shm_ctrl.py): element-wise max of host
integers over 2 / 4 ranks, many back-to-back calls with changing values and lengths (the
two-parity slot reuse), equal to the gloo all-reduce; a peer that never arrives raises instead of
hanging; nothing is left in /dev/shm."""
import os

import pytest

from .dist_utils import run_world


def _calls(rank, world, n):
    import random

    import torch
    import torch.distributed as dist

    from butterfly_amd.parallel.shm_ctrl import ShmCtrl

    g = dist.new_group(list(range(world)), backend="gloo")
    shm = ShmCtrl(list(range(world)), rank, g, "t")
    rng = random.Random(rank)
    bad = 0
    for i in range(n):
        k = 1 + i % 5
        vals = [rng.randint(-5, 10**9) for _ in range(k)]
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        bad += shm.max(vals) != t.tolist()
    shm.close()
    return bad


@pytest.mark.parametrize("world", [2, 4])
def test_shm_ctrl_matches_gloo_max(world):
    before = {f for f in os.listdir("/dev/shm") if f.startswith("bfly_ctrl_")}
    assert run_world(_calls, world, 300) == [0] * world
    after = {f for f in os.listdir("/dev/shm") if f.startswith("bfly_ctrl_")}
    assert after <= before


def _late_peer(rank, world):
    import torch.distributed as dist

    from butterfly_amd.parallel.shm_ctrl import ShmCtrl

    g = dist.new_group(list(range(world)), backend="gloo")
    shm = ShmCtrl(list(range(world)), rank, g, "late", timeout_s=0.5)
    shm.max([rank])
    if rank == 0:
        try:
            shm.max([1])               # rank 1 never makes its second call
        except TimeoutError as e:
            return "timeout" if "never reached call 1" in str(e) else str(e)
        return "no timeout"
    return "skipped"


def test_shm_ctrl_missing_peer_times_out():
    assert run_world(_late_peer, 2) == ["timeout", "skipped"]
