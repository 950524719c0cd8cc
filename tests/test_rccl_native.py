"""Native RCCL communicator (csrc/bindings/rccl_comm.cpp, parallel/rccl.py).

CPU: the library's id / version entry points, and the per-axis split plan (colors and keys)
against the mesh's torch groups. GPU: a one-rank communicator through every collective, a
split, the async-error poll and hipGraph capture (RCCL refuses two ranks on one device, so
multi-rank runs need a multi-GPU node; the split plan is what the CPU test pins)."""
import pytest
import torch

from butterfly_amd import ops
from butterfly_amd.parallel.mesh import Mesh
from butterfly_amd.utils import flags


def _lib_or_skip():
    if not ops.load_library():
        pytest.skip("butterfly_amd/_C.so not built")


def test_unique_id_and_version():
    _lib_or_skip()
    from butterfly_amd.parallel import rccl

    a, b = torch.ops.bfly.rccl_unique_id(), torch.ops.bfly.rccl_unique_id()
    assert a.dtype == torch.uint8 and a.numel() == 128
    assert not torch.equal(a, b)           # fresh bootstrap ids
    v = rccl.version()
    assert v >= 22000, v                   # NCCL-API 2.20+ (ncclCommSplit)


def test_flag_registered_on_by_default(monkeypatch):
    monkeypatch.delenv("BFLY_NATIVE_RCCL", raising=False)
    assert flags.get("BFLY_NATIVE_RCCL") is True


class _RecordingWorld:
    """Stands in for the world RcclComm: records every split call (a collective, so every
    rank must issue the same sequence of calls)."""

    def __init__(self):
        self.calls = []

    def split(self, color, key, ranks=None):
        self.calls.append((color, key, tuple(ranks)))
        return ("comm", color, key)


@pytest.mark.parametrize("dp,pp,tp", [(1, 1, 8), (2, 1, 4), (4, 1, 2), (2, 2, 2), (1, 8, 1), (8, 1, 1)])
def test_split_plan_matches_mesh_groups(dp, pp, tp):
    from butterfly_amd.parallel.rccl import split_mesh

    mesh = Mesh(dp=dp, pp=pp, tp=tp)
    n = dp * pp * tp
    per_rank = []
    for rank in range(n):
        w = _RecordingWorld()
        got = split_mesh(w, mesh, rank)
        per_rank.append(w.calls)
        for axis, (_, color, key) in got.items():
            group = mesh.all_groups(axis)[color]
            assert rank in group and group[key] == rank
        # exactly the multi-rank axes, in a fixed order
        assert sorted(got) == sorted(a for a in ("tp", "pp", "dp") if len(mesh.all_groups(a)[0]) > 1)
    # same number of collective split calls on every rank, and ranks sharing a color share a group
    assert len({len(c) for c in per_rank}) == 1
    for i in range(len(per_rank[0])):
        by_color = {}
        for rank in range(n):
            color, key, ranks = per_rank[rank][i]
            by_color.setdefault(color, set()).add(ranks)
        assert all(len(v) == 1 for v in by_color.values())


@pytest.mark.gpu
def test_single_rank_communicator_collectives_and_graph():
    _lib_or_skip()
    from butterfly_amd.parallel.rccl import RcclComm

    uid = torch.ops.bfly.rccl_unique_id()
    c = RcclComm.create(uid, 1, 0)
    try:
        assert c.info() == (0, 1, torch.cuda.current_device())
        x = torch.randn(4096, device="cuda").to(torch.bfloat16)
        ref = x.clone()
        c.all_reduce_(x)
        assert torch.equal(x, ref)
        m = torch.tensor([3, -7, 5], dtype=torch.int32, device="cuda")
        c.all_reduce_(m, "max")
        assert m.tolist() == [3, -7, 5]
        out = torch.empty_like(x)
        assert torch.equal(c.all_gather(x, out), ref)
        out.zero_()
        assert torch.equal(c.reduce_scatter(x, out), ref)
        out.zero_()
        assert torch.equal(c.all_to_all(x, out), ref)
        c.broadcast_(x, 0)
        assert torch.equal(x, ref)
        # point-to-point to itself inside one group call
        r = torch.empty_like(x)
        RcclComm.group_start()
        c.send(x, 0)
        c.recv(r, 0)
        RcclComm.group_end()
        assert torch.equal(r, ref)
        sub = c.split(0, 0, [0])
        assert sub is not None and sub.info()[1] == 1
        none = c.split(-1, 0)
        assert none is None
        assert c.async_error() == 0 and sub.async_error() == 0
        # stream-ordered: capture an all-reduce between two kernels in a hipGraph and replay
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        y = torch.zeros(1024, device="cuda")
        with torch.cuda.stream(s):
            y.add_(1.0)
            sub.all_reduce_(y)
            y.mul_(2.0)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y.add_(1.0)
            sub.all_reduce_(y)
            y.mul_(2.0)
        y.zero_()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        assert torch.allclose(y, torch.full_like(y, 6.0))
        del g
        torch.cuda.synchronize()
        assert sub.close() == "clean"
    finally:
        assert c.close() in ("clean", "released")


@pytest.mark.gpu
def test_abort_all_and_error_poller():
    """The failure path: the async-error poller sees a healthy communicator as healthy, and
    abort_all takes every live communicator down (a later close of one is a no-op)."""
    _lib_or_skip()
    from butterfly_amd.parallel import rccl
    from butterfly_amd.utils import health

    c = rccl.RcclComm.create(torch.ops.bfly.rccl_unique_id(), 1, 0)
    sub = c.split(0, 0, [0])
    assert rccl.abort_all in health._abort_hooks
    live = rccl.live_handles()
    assert c.handle in live and sub.handle in live
    assert rccl.async_errors() is None
    fired = []
    p = rccl.start_error_poller(period=0.05, on_failure=fired.append)
    x = torch.ones(1 << 16, device="cuda")
    c.all_reduce_(x)
    torch.cuda.synchronize()
    import time
    time.sleep(0.3)
    p.stop()
    assert fired == [] and p.failed is None
    assert rccl.abort_all() >= 2
    assert c.handle not in rccl.live_handles() and sub.handle not in rccl.live_handles()
    sub.close()
    c.close()        # already aborted: no-op
    with pytest.raises(RuntimeError):
        c.all_reduce_(x)


_INIT_HANG = """
import time, torch
from butterfly_amd import ops
assert ops.load_library()
from butterfly_amd.parallel.rccl import RcclComm, live_handles
t0 = time.monotonic()
try:
    RcclComm.create(torch.ops.bfly.rccl_unique_id(), 2, 0, timeout=4.0)   # rank 1 never joins
    print("NO-TIMEOUT")
except TimeoutError as e:
    print(f"TIMEOUT after {time.monotonic() - t0:.1f}s live={live_handles()}: {e}")
"""


@pytest.mark.gpu
def test_init_deadline_aborts_instead_of_hanging():
    """A communicator whose peer never joins (a 2-rank init with rank 1 absent) ends through the
    non-blocking init's deadline: TimeoutError after ~4 s, the half-built communicator aborted,
    nothing left in the handle table, the process exits normally (no watchdog os._exit)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _INIT_HANG], cwd=root, capture_output=True, text=True, timeout=90)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    line = next((ln for ln in r.stdout.splitlines() if ln.startswith("TIMEOUT")), None)
    assert line is not None, out[-3000:]
    took = float(line.split()[2].rstrip("s"))
    assert 3.5 <= took < 30, line
    assert "live=[]" in line, line


@pytest.mark.gpu
@pytest.mark.parametrize("n,spec", [(2, "tp2"), (4, "dp2xtp2"), (8, "dp4xtp2")])
def test_native_rccl_matches_torch_multi_gpu(n, spec):
    """Native world + split communicators vs torch.distributed RCCL, one GPU per rank."""
    import os
    import subprocess
    import sys

    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs (RCCL refuses two ranks on one device)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", str(n), "--", sys.executable,
                        os.path.join(root, "tools", "rccl_native_check.py"), spec],
                       cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") >= n
