"""Butterfly (recursive halving / doubling) all-reduce on gloo ranks: exact sums (integer-valued
f32), identical bits on every rank, odd sizes (segments of 0 or 1 element) and the
non-power-of-two fallback."""
import pytest

from tests.dist_utils import run_world


def _run(rank, world, sizes):
    import torch
    import torch.distributed as dist

    from butterfly_amd.parallel.butterfly import butterfly_all_reduce_

    out = []
    ranks = list(range(world))
    for n in sizes:
        g = torch.Generator().manual_seed(1000 * n + rank)
        x = torch.randint(-50, 50, (n,), generator=g).float()
        want = x.clone()
        dist.all_reduce(want)
        got = butterfly_all_reduce_(x.clone(), ranks)
        out.append((torch.equal(got, want), got.tolist()))
    # a 2-D bf16 activation: same bits on every rank
    h = torch.randn(5, 33, generator=torch.Generator().manual_seed(rank)).to(torch.bfloat16)
    out.append((True, butterfly_all_reduce_(h, ranks).float().flatten().tolist()))
    return out


@pytest.mark.parametrize("world", [2, 4, 3])
def test_butterfly_all_reduce_matches_and_agrees(world):
    sizes = [1, 3, 7, 64, 1000]
    res = run_world(_run, world, sizes)
    for r in range(world):
        for j in range(len(sizes)):
            assert res[r][j][0], (world, r, sizes[j])
    for j in range(len(sizes) + 1):
        assert all(res[r][j][1] == res[0][j][1] for r in range(world))


def _comm_route(rank, world):
    import os

    import torch

    from butterfly_amd.parallel.comm import Communicator
    from butterfly_amd.parallel.mesh import Mesh

    from butterfly_amd.parallel import butterfly as bfm

    calls = []
    orig = bfm.butterfly_all_reduce_
    bfm.butterfly_all_reduce_ = lambda t, *a: (calls.append(t.numel()), orig(t, *a))[1]
    comm = Communicator.from_mesh(Mesh(tp=world))
    os.environ["BFLY_AR_BUTTERFLY"] = "0:4096"
    small = torch.full((8, 16), float(rank + 1))       # 512 B: butterfly
    big = torch.full((64, 64), float(rank + 1))         # 16 KiB: the group's all-reduce
    comm.all_reduce_(small)
    comm.all_reduce_(big)
    os.environ.pop("BFLY_AR_BUTTERFLY")
    s = world * (world + 1) / 2
    return bool((small == s).all()) and bool((big == s).all()) and calls == [8 * 16]


def test_communicator_routes_probed_sizes_to_butterfly():
    assert all(run_world(_comm_route, 4))
