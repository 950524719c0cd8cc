"""Partitioning API: plan validity properties, JSON round trip, objective behaviour."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from butterfly_amd.config import ModelConfig
from butterfly_amd.models.shard import local_dims
from butterfly_amd.partition import PartitionPlan, factorizations, partition


@settings(max_examples=30, deadline=None)
@given(st.sampled_from(["llama3-70b", "llama3-8b", "mixtral-8x7b", "gpt2-small", "llama-tiny"]),
       st.sampled_from([1, 2, 4, 8]), st.sampled_from(["throughput", "latency"]))
def test_plans_are_valid(preset, n, objective):
    cfg = ModelConfig.from_preset(preset)
    try:
        plan = partition(cfg, n, objective=objective, batch_per_gpu=16, ctx=512)
    except ValueError:
        return  # no feasible layout (e.g. model too big) is a legal answer
    plan.validate()
    assert plan.dp * plan.tp * plan.pp == n
    layers = [l for a, b in plan.stages for l in range(a, b)]
    assert layers == list(range(cfg.num_layers))            # every layer exactly once, in order
    assert cfg.num_heads % plan.tp == 0
    for r in range(n):
        local_dims(cfg, plan.shard(r))
        assert plan.weight_bytes[r] <= 288e9                  # fits one MI355X
    back = PartitionPlan.from_json(plan.to_json())
    assert back.to_dict() == plan.to_dict()


def test_fixed_strategy_and_70b_single_gpu_fits():
    p = partition("llama3-70b", 8, {"tp": 2, "pp": 4})
    assert (p.tp, p.pp, p.dp) == (2, 4, 1) and len(p.stages) == 4
    one = partition("llama3-70b", 1)
    assert one.weight_bytes[0] > 140e9 and one.weight_bytes[0] < 288e9


def test_factorizations():
    assert sorted(factorizations(4)) == sorted([(4, 1, 1), (2, 2, 1), (2, 1, 2), (1, 4, 1), (1, 2, 2), (1, 1, 4)])


def test_invalid_plan_rejected():
    p = partition("llama-tiny", 2, {"pp": 2})
    d = p.to_dict()
    d["stages"] = [[0, 1], [0, 2]]
    with pytest.raises(ValueError):
        PartitionPlan.from_dict(d)


def test_mixtral_expert_parallel_candidate():
    p = partition("mixtral-8x7b", 8, {"dp": 8, "ep": 8})
    assert p.ep == 8 and p.shard(3).ep_rank == 3


def test_expert_parallel_with_pipeline_stages():
    """EP x PP (round 6): an explicit ep2 x pp2 request is a valid plan whose stage ranks share
    their EP groups per stage; its rank programs (one microbatch per tick) are consistent, and
    the synchronous multi-microbatch program is refused."""
    import pytest as _pt

    from butterfly_amd.partition.schedule import check_programs, programs, rank_program

    p = partition("mixtral-8x7b", 4, {"dp": 2, "ep": 2, "pp": 2})
    assert p.ep == 2 and p.pp == 2
    mesh = p.mesh
    assert mesh.dp_group(mesh.rank(0, 1, 0)) == [mesh.rank(0, 1, 0), mesh.rank(1, 1, 0)]
    check_programs(programs(p, 8, microbatches=1, ep_ipc=True))
    with _pt.raises(ValueError):
        rank_program(p, 0, 8, microbatches=2)


@settings(max_examples=25, deadline=None)
@given(st.sampled_from(["llama3-70b", "llama3-8b", "mixtral-8x7b"]), st.sampled_from([2, 4, 8]),
       st.sampled_from([8, 32, 64]), st.sampled_from(["throughput", "latency"]))
def test_choice_minimises_busiest_link_among_near_best(preset, n, bpg, objective):
    """Link-aware selection: of every feasible layout whose objective is within 2 % of the best,
    the chosen plan has the fewest bytes per token on its busiest xGMI link."""
    from butterfly_amd.partition.search import _tp_ok, evaluate

    cfg = ModelConfig.from_preset(preset)
    try:
        chosen = partition(cfg, n, objective=objective, batch_per_gpu=bpg, ctx=1024)
    except ValueError:
        return
    plans = []
    for dp, tp, pp in factorizations(n):
        if not _tp_ok(cfg, tp) or pp > cfg.num_layers:
            continue
        for ep in ([1, dp] if cfg.is_moe and dp > 1 and tp == 1 and pp == 1 and cfg.num_experts % dp == 0 else [1]):
            try:
                p = evaluate(cfg, dp, tp, pp, ep, batch_per_gpu=bpg, ctx=1024, objective=objective)
            except ValueError:
                p = None
            if p is not None:
                plans.append(p)
    score = (lambda p: p.estimate["tokens_per_second"]) if objective == "throughput" else \
        (lambda p: -p.estimate["token_latency_seconds"])
    best = max(score(p) for p in plans)
    near = [p for p in plans if score(p) >= best - abs(best) * 0.02]
    assert chosen.estimate["max_link_bytes_per_token"] == min(p.estimate["max_link_bytes_per_token"] for p in near)
    assert score(chosen) >= best - abs(best) * 0.02


def test_measured_comm_table_drives_allreduce_cost():
    """With a probe table attached, all-reduce prices come from it (log-log interpolation of the
    implementation the runtime would pick), not from the default constants."""
    from butterfly_amd.partition.costmodel import CostModel, interp_loglog
    from butterfly_amd.partition.hw import MI355X

    tab = {"all_reduce": {"rccl": {8: [[1 << 20, 100e-6], [8 << 20, 400e-6]]},
                          "oneshot": {8: [[16 << 10, 10e-6], [1 << 20, 30e-6]]},
                          "twoshot": {"8": [[1 << 20, 20e-6], [8 << 20, 50e-6]]}},
           "p2p": [[1 << 20, 15e-6]]}
    cm = CostModel(ModelConfig.from_preset("llama3-70b"), MI355X.with_comm_table(tab))
    assert cm.allreduce(16 << 10, 8) == pytest.approx(10e-6)            # one-shot below 512 KiB
    assert cm.allreduce(8 << 20, 8) == pytest.approx(50e-6)             # two-shot from 512 KiB
    assert cm.allreduce(32 << 20, 8) > 400e-6                           # RCCL beyond the IPC buffer
    assert cm.p2p(1 << 20) == pytest.approx(15e-6)
    assert interp_loglog([[1, 1.0], [100, 100.0]], 10) == pytest.approx(10.0)
