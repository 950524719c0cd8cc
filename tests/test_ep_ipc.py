"""Byte-minimal EP dispatch (parallel/ep_ipc.py): the loopback emulation of the IPC protocol
(ranks as threads, shared CPU buffers) against the fixed-capacity all-to-all path — received
rows, expert ids / weights, combined outputs bitwise, and fewer link bytes; and a whole
expert-parallel MoE engine with the IPC path on and off."""
import pytest
import torch

from butterfly_amd.parallel.fake import FakeWorld
from butterfly_amd.parallel.mesh import Mesh

H, K, CAP, EL = 64, 2, 16, 2


def _inputs(r, T, ep):
    g = torch.Generator().manual_seed(31 * r + T)
    x = torch.randn(T, H, generator=g).to(torch.bfloat16)
    ids = torch.randint(-1, ep * EL, (T, K), generator=g, dtype=torch.int32)
    w = torch.rand(T, K, generator=g)
    slots = torch.arange(T, dtype=torch.int32)
    if T > 2:
        slots[1] = -1                          # graph padding row
    return x, ids, w, slots


@pytest.mark.parametrize("ep", [2, 4])
def test_loopback_dispatch_matches_all_to_all(ep):
    torch.set_num_threads(1)
    mesh = Mesh(dp=ep, ep=ep)
    world = FakeWorld(mesh, timeout_s=60)

    def run(r, comm):
        me = comm.rank_in("ep")
        assert comm.enable_ep_ipc(CAP, H, K)
        res = []
        for T in (1, 9, CAP):
            x, ids, w, slots = _inputs(me, T, ep)
            got = []
            for use_ipc in (True, False):
                saved = comm.ep_ipc
                if not use_ipc:
                    comm.ep_ipc = None
                rt = comm.ep_dispatch(x, ids, w, slots, EL, CAP)
                y = (rt.x.float() * (me + 1)).to(torch.bfloat16)     # the expert rank's "FFN"
                got.append((rt, comm.ep_combine(y, rt)))
                comm.ep_ipc = saved
            (ri, oi), (ra, oa) = got
            assert ri.path == "loopback" and ra.path == "a2a"
            assert torch.equal(oi, oa), (T, (oi.float() - oa.float()).abs().max())
            # ids / weights of every row; the rows each source actually routed here
            assert torch.equal(ri.ids, ra.ids) and torch.equal(ri.w, ra.w)
            routed = ra.ids.ge(0).any(1)
            assert torch.equal(ri.x[routed], ra.x[routed])
            res.append(comm.ep_ipc.stats())
        return res

    stats = world.run(run)
    a2a_bytes = sum(b for _, op, _, _, b in world.log if op == "all_to_all")
    ipc_bytes = sum(s[-1]["bytes_out"] + s[-1]["bytes_back"] for s in stats)
    assert 0 < ipc_bytes < a2a_bytes


@pytest.mark.parametrize("ipc", ["1", "0"])
def test_expert_parallel_engine_ipc_on_off(ipc, monkeypatch):
    from tests.test_fake_comm import PROMPTS, _gen

    torch.set_num_threads(1)
    monkeypatch.setenv("BFLY_EP_IPC", ipc)
    mesh = Mesh(dp=2, ep=2)
    world = FakeWorld(mesh, timeout_s=60)
    halves = [PROMPTS[:3], PROMPTS[3:]]
    outs = world.run(lambda r, c: (_gen("mixtral-tiny", mesh, c, halves[mesh.coord(r).dp]), c.ep_ipc))
    assert outs[0][0] == _gen("mixtral-tiny", Mesh(), None, halves[0])
    assert outs[1][0] == _gen("mixtral-tiny", Mesh(), None, halves[1])
    assert (outs[0][1] is not None) == (ipc == "1")
    if ipc == "1":
        assert outs[0][1].stats()["rows_out"] > 0


@pytest.mark.parametrize("ep", [2, 4])
def test_prefill_ipc_moe_equals_all_to_all(ep):
    """The EP prefill MoE layer over the IPC exchange (device scan route, block-count-bounded
    receiver; loopback emulation) is bitwise the host-split all-to-all path, with different
    token counts per rank (one rank idle)."""
    from butterfly_amd import ops
    from butterfly_amd.config import ModelConfig
    from butterfly_amd.models import Shard, build_model

    torch.set_num_threads(1)
    mesh = Mesh(dp=ep, ep=ep)
    world = FakeWorld(mesh, timeout_s=60)
    cfg = ModelConfig.from_preset("mixtral-tiny")

    def run(r, comm):
        me = comm.rank_in("ep")
        m = build_model(cfg, Shard(ep_rank=me, ep_size=ep), device="cpu", dtype=torch.float32, comm=comm)
        m.init_random(0)
        assert comm.enable_ep_ipc_prefill(64, cfg.hidden_size, cfg.experts_per_token)
        T = 0 if me == ep - 1 else 9 + 5 * me
        x = torch.randn(T, cfg.hidden_size, generator=torch.Generator().manual_seed(me))
        _, ids, w = ops.moe_route(x, m.p["l0.router_w"], cfg.experts_per_token)
        a = m._moe_ipc_prefill("l0.", x, ids, w, comm.ep_ipc_prefill)
        b = m._moe_alltoall("l0.", x, ids, w)
        return torch.equal(a, b) and a.shape == (T, cfg.hidden_size)

    assert all(world.run(run))


def test_ipc_fallback_conforms_to_the_program():
    """with the IPC exchange set up, the step program lists ep_dispatch /
    ep_return; a call beyond the IPC capacity takes the all-to-all fallback on every EP rank,
    which must pass the program check (BFLY_PROGRAM_CHECK) as that same dispatch / return."""
    from butterfly_amd.partition.schedule import Instr

    torch.set_num_threads(1)
    ep = 2
    mesh = Mesh(dp=ep, ep=ep)
    world = FakeWorld(mesh, timeout_s=60)

    def run(r, comm):
        me = comm.rank_in("ep")
        assert comm.enable_ep_ipc(CAP, H, K)
        grp = tuple(comm.groups["ep"].ranks)
        prog = [Instr("ep_dispatch", grp), Instr("ep_return", grp)]
        x, ids, w, slots = _inputs(me, 2 * CAP, ep)       # more rows than the IPC capacity
        with comm.expect(prog):
            rt = comm.ep_dispatch(x, ids, w, slots, EL, 2 * CAP)
            out = comm.ep_combine(rt.x, rt)
        return rt.path, out.shape

    for path, shape in world.run(run):
        assert path == "a2a" and shape == (2 * CAP, H)
