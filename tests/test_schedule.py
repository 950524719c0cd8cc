"""Communication schedule (partition/schedule.py): the per-rank decode-step programs derived from
a plan are mutually consistent for every factorisation, a broken program is caught, and the
program matches what the engine actually issues (replayed through the loopback backend)."""
import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams
from butterfly_amd.parallel.fake import FakeWorld
from butterfly_amd.parallel.mesh import Mesh
from butterfly_amd.partition import partition
from butterfly_amd.partition.schedule import Instr, check_programs, link_bytes, programs
from butterfly_amd.partition.search import factorizations


@pytest.mark.parametrize("preset", ["llama3-70b", "llama3-8b", "mixtral-8x7b"])
def test_programs_consistent_for_every_factorisation(preset):
    cfg = ModelConfig.from_preset(preset)
    for n in (2, 4, 8):
        for dp, tp, pp in factorizations(n):
            strat = {"dp": dp, "tp": tp, "pp": pp}
            if cfg.is_moe and dp > 1 and tp == 1 and pp == 1:
                strat["ep"] = dp
            try:
                plan = partition(cfg, n, strat)
            except ValueError:
                continue   # infeasible (heads / memory)
            progs = programs(plan, 64)
            check_programs(progs)
            lb = link_bytes(plan, progs)
            if plan.tp > 1 or plan.pp > 1 or plan.ep > 1:
                assert lb and all(v > 0 for v in lb.values())
            # every rank's program covers exactly its stage's layers
            for r, p in progs.items():
                a, b = plan.stages[plan.mesh.coord(r).pp]
                layers = {i.note.split(":")[0] for i in p.instrs if i.op == "compute" and i.note.startswith("layer")}
                assert layers == {f"layer {k}" for k in range(a, b)}


def test_check_programs_catches_mismatch():
    plan = partition(ModelConfig.from_preset("llama3-70b"), 8, {"tp": 2, "pp": 4})
    progs = programs(plan, 16)
    check_programs(progs)
    # rank 3 drops one TP all-reduce: its partner would wait forever
    p3 = progs[3]
    k = next(i for i, ins in enumerate(p3.instrs) if ins.op == "all_reduce")
    del p3.instrs[k]
    with pytest.raises(ValueError, match="group"):
        check_programs(progs)
    # a send without the matching recv size
    progs = programs(plan, 16)
    p0 = progs[0]
    k = next(i for i, ins in enumerate(p0.instrs) if ins.op == "send")
    p0.instrs[k] = Instr("send", p0.instrs[k].group, 1, "comm")
    with pytest.raises(ValueError, match="p2p"):
        check_programs(progs)


PROMPTS = [[3, 14, 15, 92, 65], [35, 89, 79, 32, 38, 46, 26], [43, 7], [38, 32, 79, 50, 28, 84]]


def _decode_window(rank, comm, preset, mesh, stages):
    """Prefill everything, then bracket exactly one decode step by two barriers."""
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu", stage_layers=stages)
    for p in PROMPTS:
        eng.add_request(p, SamplingParams(max_tokens=40, ignore_eos=True))
    groups = mesh.pp if eng.async_pp else 1
    streak = 0
    while eng.scheduler.num_waiting > 0 or streak < groups + 1:
        out = eng.step()
        streak = streak + 1 if out.kind == "decode" else 0
    comm.barrier()
    out = eng.step()
    comm.barrier()
    return out.kind, eng.async_pp, eng.ep_ipc


@pytest.mark.parametrize("pp_async", ["1", "0"])
@pytest.mark.parametrize("preset,kw", [("llama-tiny", dict(tp=2)), ("llama-tiny", dict(pp=2)),
                                       ("llama-tiny", dict(tp=2, pp=2)), ("mixtral-tiny", dict(dp=2, ep=2)),
                                       ("mixtral-tiny", dict(tp=2))])
def test_program_matches_engine(preset, kw, pp_async, monkeypatch):
    monkeypatch.setenv("BFLY_PP_ASYNC", pp_async)
    torch.set_num_threads(1)
    cfg = ModelConfig.from_preset(preset)
    n = kw.get("dp", 1) * kw.get("tp", 1) * kw.get("pp", 1)
    plan = partition(cfg, n, kw, batch_per_gpu=4 * n // kw.get("dp", 1))
    mesh = plan.mesh
    world = FakeWorld(mesh, timeout_s=60)
    outs = world.run(lambda r, c: _decode_window(r, c, preset, mesh, plan.stages))
    assert all(k == "decode" for k, _, _ in outs)
    if outs[0][1]:   # asynchronous pipeline: a step is one tick carrying one request group
        tokens, mb = len(PROMPTS) // mesh.pp, 1
    else:            # synchronous: the whole batch in pp microbatches
        tokens, mb = len(PROMPTS), mesh.pp
    for r in range(mesh.world_size):
        mine = [(op, grp, nb) for rk, op, grp, shape, nb in world.log if rk == r]
        bars = [i for i, e in enumerate(mine) if e[0] == "barrier"]
        got = [e for e in mine[bars[-2] + 1: bars[-1]]]
        want = [i for i in programs(plan, tokens, mb, dtype_bytes=4, ep_ipc=outs[r][2])[r].comm()
                if i.op != "recv"]   # CPU: fp32
        # the loopback log names broadcasts by source ("broadcast<src>") and records sends
        assert [("broadcast" if op.startswith("broadcast") else op, grp) for op, grp, _ in got] == \
            [(i.op, i.group) for i in want], (r, got, [(i.op, i.group) for i in want])
        for (op, _, nb), i in zip(got, want):
            # every payload, EP dispatch / sampling gather / broadcast included; the IPC EP
            # exchange logs its rendezvous (the program carries the routed-bytes bound)
            if op in ("ep_dispatch", "ep_return"):
                continue
            assert nb == i.nbytes, (r, op, nb, i)


def _generate_prepost(rank, comm, preset, mesh, stages):
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu", stage_layers=stages)
    rids = [eng.add_request(p, SamplingParams(max_tokens=3 + 2 * i, ignore_eos=True)) for i, p in enumerate(PROMPTS)]
    while eng.has_unfinished():
        eng.step()
    return [eng.requests[r].output for r in rids], eng.metrics.counters.get("pp_preposted_recvs", 0), eng._prepost


@pytest.mark.parametrize("preset,kw", [("llama-tiny", dict(pp=2)), ("llama-tiny", dict(tp=2, pp=2)),
                                       ("llama-small", dict(pp=4))])
def test_async_pipeline_preposted_receives(preset, kw, monkeypatch):
    """Overlap executor (engine._prepost_recv): every non-first stage posts the boundary receive
    of the group arriving next tick at the end of the current tick, into one of two persistent
    buffers. On the loopback backend (its irecv completes on the spot, so a receive posted
    too early or out of order would hang or mismatch shapes) the tokens must equal the
    single-process engine's and almost every stage tick must have used a pre-posted receive."""
    monkeypatch.setenv("BFLY_PP_ASYNC", "1")
    monkeypatch.setenv("BFLY_PP_PREPOST", "1")
    torch.set_num_threads(1)
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    single = LLMEngine(cfg, Mesh(), ecfg, device="cpu")
    rids = [single.add_request(p, SamplingParams(max_tokens=3 + 2 * i, ignore_eos=True)) for i, p in enumerate(PROMPTS)]
    while single.has_unfinished():
        single.step()
    want = [single.requests[r].output for r in rids]
    n = kw.get("tp", 1) * kw["pp"]
    plan = partition(cfg, n, kw, batch_per_gpu=8)
    mesh = plan.mesh
    world = FakeWorld(mesh, timeout_s=60)
    outs = world.run(lambda r, c: _generate_prepost(r, c, preset, mesh, plan.stages))
    for r, (toks, used, on) in enumerate(outs):
        assert toks == want
        first = mesh.coord(r).pp == 0
        assert on == (not first)
        if not first:
            assert used > 0


def test_native_pp_program_puts_recv_in_graph_and_send_on_send_stream():
    """With native RCCL pipeline edges the boundary receive is the decode graph's first node
    and the send leaves from the send stream, both moving the whole graph bucket; the programs
    stay pairwise consistent."""
    from butterfly_amd.partition import schedule as sch
    from butterfly_amd.partition.plan import PartitionPlan  # noqa: F401
    from butterfly_amd.partition import partition
    from butterfly_amd.config import ModelConfig

    plan = partition(ModelConfig.from_preset("llama-tiny"), 4, {"tp": 2, "pp": 2}, batch_per_gpu=8, ctx=128)
    progs = sch.programs(plan, 6, native_pp=True, bucket=8)
    sch.check_programs(progs)
    h = plan.model.hidden_size
    for r, p in progs.items():
        c = plan.mesh.coord(r)
        p2p = [i for i in p.comm() if i.op in ("send", "recv")]
        assert len(p2p) == 1
        i = p2p[0]
        assert i.nbytes == 8 * h * 2
        assert (i.op, i.stream) == (("recv", "graph") if c.pp == 1 else ("send", "send"))


@pytest.mark.parametrize("pp_async", ["1", "0"])
@pytest.mark.parametrize("kw", [dict(pp=2), dict(tp=2, pp=2), dict(tp=2)])
def test_engine_executes_rank_program(kw, pp_async, monkeypatch):
    """The rank program drives the engine: every boundary receive, stage run,
    send, sampling and id broadcast the engine performs is an instruction of
    schedule.exec_program, executed in the program's order with the program's peers."""
    from butterfly_amd.engine.engine import LLMEngine as Eng
    from butterfly_amd.partition.schedule import exec_program

    monkeypatch.setenv("BFLY_PP_ASYNC", pp_async)
    torch.set_num_threads(1)
    n = kw.get("tp", 1) * kw.get("pp", 1)
    plan = partition(ModelConfig.from_preset("llama-tiny"), n, kw, batch_per_gpu=4)
    mesh = plan.mesh
    ran: dict = {}
    orig = Eng._execute

    def spy(ops, recv, run, send, sample, broadcast=None):
        import threading

        ran.setdefault(threading.current_thread().name, []).append(list(ops))
        return orig(ops, recv, run, send, sample, broadcast)

    monkeypatch.setattr(Eng, "_execute", staticmethod(spy))
    world = FakeWorld(mesh, timeout_s=60)
    outs = world.run(lambda r, c: _decode_window(r, c, "llama-tiny", mesh, plan.stages))
    assert all(k == "decode" for k, _, _ in outs)
    if mesh.pp == 1 and pp_async == "0":
        assert not ran        # synchronous single stage: the stage run and sampling need no program walk
        return
    assert len(ran) == mesh.world_size
    progs = {(m, nat): {r: exec_program(plan, r, m, nat) for r in range(n)} for m in (1, mesh.pp) for nat in (False,)}
    for calls in ran.values():
        for ops in calls:
            assert any(ops == p[r] for p in progs.values() for r in p), ops
    # sends and receives go to the program's peers: next / previous stage
    for r in range(n):
        for ins in exec_program(plan, r, 1):
            if ins.exec == "send":
                assert ins.group == (r, mesh.next_stage(r))
            if ins.exec == "recv":
                assert ins.group == (mesh.prev_stage(r), r)


def _generate_checked(rank, comm, preset, mesh, stages):
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu", stage_layers=stages)
    assert eng.runner.conform is not None
    rids = [eng.add_request(p, SamplingParams(max_tokens=3 + 2 * i, ignore_eos=True)) for i, p in enumerate(PROMPTS)]
    while eng.has_unfinished():
        eng.step()
    return [eng.requests[r].output for r in rids]


@pytest.mark.parametrize("pp_async", ["1", "0"])
@pytest.mark.parametrize("preset,kw", [("llama-tiny", dict(tp=2)), ("llama-tiny", dict(tp=2, pp=2)),
                                       ("mixtral-tiny", dict(dp=2, ep=2)), ("mixtral-tiny", dict(tp=2))])
def test_program_enforced_on_every_decode_step(preset, kw, pp_async, monkeypatch):
    """BFLY_PROGRAM_CHECK: every collective the model code issues in a decode step is checked
    against the rank program's next instruction before it is issued (op, group, payload) and
    the step must issue all of them. A whole generation passes on every layout, with the tokens
    of the single-process engine."""
    monkeypatch.setenv("BFLY_PP_ASYNC", pp_async)
    monkeypatch.setenv("BFLY_PROGRAM_CHECK", "1")
    torch.set_num_threads(1)
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    single = LLMEngine(cfg, Mesh(), ecfg, device="cpu")
    rids = [single.add_request(p, SamplingParams(max_tokens=3 + 2 * i, ignore_eos=True)) for i, p in enumerate(PROMPTS)]
    while single.has_unfinished():
        single.step()
    want = [single.requests[r].output for r in rids]
    n = kw.get("dp", 1) * kw.get("tp", 1) * kw.get("pp", 1)
    plan = partition(cfg, n, kw, batch_per_gpu=4 * n // kw.get("dp", 1))
    world = FakeWorld(plan.mesh, timeout_s=60)
    outs = world.run(lambda r, c: _generate_checked(r, c, preset, plan.mesh, plan.stages))
    assert all(o == want for o in outs)


def test_program_check_raises_before_a_divergent_collective():
    from butterfly_amd.parallel.comm import Communicator, GroupHandle, ProgramMismatch

    g = GroupHandle([0, 1], None, 0)
    c = Communicator(Mesh(), 0, {"tp": g, "ep": g, "pp": g, "dp": g, "world": g})
    prog = [Instr("all_reduce", (0, 1), 64, note="layer 0 attention output"),
            Instr("all_reduce", (0, 1), 64, note="layer 0 FFN output")]
    with c.expect(prog):
        c._conform("all_reduce", "tp", 64)
        c._conform("all_reduce", "tp", 64)
    with pytest.raises(ProgramMismatch, match="about to issue all_to_all"):
        with c.expect(prog):
            c._conform("all_to_all", "tp", 64)
    with pytest.raises(ProgramMismatch, match="instruction 1 is all_reduce"):
        with c.expect(prog):
            c._conform("all_reduce", "tp", 64)
            c._conform("all_reduce", "tp", 128)      # wrong payload
    with pytest.raises(ProgramMismatch, match="not issued"):
        with c.expect(prog):
            c._conform("all_reduce", "tp", 64)
    with pytest.raises(ProgramMismatch, match="after the step program's last"):
        with c.expect(prog[:1]):
            c._conform("all_reduce", "tp", 64)
            c._conform("all_reduce", "tp", 64)
    assert c._expect is None


def _diverging_rank(rank, comm, preset, mesh, stages):
    """Rank 1's program has an extra EP all-to-all in front of the first all-reduce: its model
    code no longer matches the program, and the check must stop it before the collective."""
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu", stage_layers=stages)
    if rank == 1:
        real = eng.runner.conform
        eng.runner.conform = lambda rows: [Instr("all_to_all", (0, 1), 64, note="injected")] + real(rows)
    for p in PROMPTS:
        eng.add_request(p, SamplingParams(max_tokens=4, ignore_eos=True))
    while eng.has_unfinished():
        eng.step()


def test_program_check_stops_a_diverging_rank(monkeypatch):
    monkeypatch.setenv("BFLY_PROGRAM_CHECK", "1")
    torch.set_num_threads(1)
    cfg = ModelConfig.from_preset("llama-tiny")
    plan = partition(cfg, 2, dict(tp=2), batch_per_gpu=8)
    world = FakeWorld(plan.mesh, timeout_s=5)
    with pytest.raises(RuntimeError, match="rank 1 failed: ProgramMismatch.*about to issue all_reduce"):
        world.run(lambda r, c: _diverging_rank(r, c, "llama-tiny", plan.mesh, plan.stages))
