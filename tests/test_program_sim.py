"""Rank-program simulator (csrc/runtime/program_sim.h via partition.schedule.simulate): the
programs of every layout the partitioner produces run to the end against each other, also
under strict rendezvous point-to-point semantics; programs that are consistent per group and
per pair but wait on each other ACROSS groups are reported as a deadlock with every blocked
rank named (the per-group comparison alone passes them)."""
import pytest

from butterfly_amd.config import ModelConfig
from butterfly_amd.partition.schedule import Instr, RankProgram, check_programs, programs, simulate
from butterfly_amd.partition.search import partition


def _progs(spec: dict) -> dict:
    """{rank: [(op, group, nbytes[, stream])]} -> RankPrograms."""
    out = {}
    for r, ins in spec.items():
        out[r] = RankProgram(r, 1, [Instr(i[0], tuple(i[1]), i[2], i[3] if len(i) > 3 else "compute") for i in ins])
    return out


@pytest.mark.parametrize("model,n,strategy", [
    ("llama3-70b", 2, {"pp": 2}), ("llama3-70b", 8, {"pp": 8}), ("llama3-70b", 8, {"tp": 2, "pp": 4}),
    ("llama3-70b", 8, {"dp": 2, "tp": 4}), ("llama3-70b", 8, {"tp": 8}), ("mixtral-8x7b", 8, {"ep": 8}),
])
@pytest.mark.parametrize("microbatches", [1, 4])
@pytest.mark.parametrize("native_pp", [False, True])
def test_every_layout_runs_to_the_end(model, n, strategy, microbatches, native_pp):
    plan = partition(ModelConfig.from_preset(model), n, strategy)
    progs = programs(plan, 64, microbatches=microbatches, native_pp=native_pp)
    check_programs(progs)                                  # includes the buffered simulation
    strict = simulate(progs, rendezvous=True)
    assert strict["ok"], strict
    assert strict["completed"] == sum(len(p.comm()) for p in progs.values())


def test_cross_group_cycle_is_a_deadlock():
    # every group's members issue the same collectives in the same order, yet rank 0 waits in
    # A for rank 1, rank 1 in C for rank 2, rank 2 in B for rank 0
    A, B, C = (0, 1), (0, 2), (1, 2)
    progs = _progs({0: [("all_reduce", A, 64), ("all_reduce", B, 64)],
                    1: [("all_reduce", C, 64), ("all_reduce", A, 64)],
                    2: [("all_reduce", B, 64), ("all_reduce", C, 64)]})
    sim = simulate(progs)
    assert not sim["ok"] and not sim["error"]
    assert sorted(b[0] for b in sim["blocked"]) == [0, 1, 2]
    with pytest.raises(ValueError, match="deadlock"):
        check_programs(progs)


def test_point_to_point_semantics():
    head_to_head = {0: [("send", (0, 1), 8, "comm"), ("recv", (1, 0), 8, "comm")],
                    1: [("send", (1, 0), 8, "comm"), ("recv", (0, 1), 8, "comm")]}
    assert simulate(_progs(head_to_head))["ok"]                       # buffered sends
    stuck = simulate(_progs(head_to_head), rendezvous=True)           # RCCL-style rendezvous
    assert not stuck["ok"] and [b[0] for b in stuck["blocked"]] == [0, 1]
    side = {r: [(op, g, n, "send" if op == "send" else "comm") for op, g, n, _ in ins]
            for r, ins in head_to_head.items()}
    assert simulate(_progs(side), rendezvous=True)["ok"]              # side-stream sends never block
    bad = simulate(_progs({0: [("send", (0, 1), 8)], 1: [("recv", (0, 1), 16)]}))
    assert not bad["ok"] and "16B" in bad["error"]


def test_collective_mismatch_is_an_error():
    sim = simulate(_progs({0: [("all_reduce", (0, 1), 64)], 1: [("all_gather", (0, 1), 64)]}))
    assert not sim["ok"] and "rank" in sim["error"]
