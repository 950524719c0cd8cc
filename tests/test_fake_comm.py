"""In-process loopback backend (parallel/fake.py): the parallel engine programs run as threads
and the backend checks that every rank issues the same collectives in the same order and that
every recv matches a send — the ordering checker of SURVEY.md §5.2."""
import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams
from butterfly_amd.parallel.fake import CommOrderError, FakeWorld
from butterfly_amd.parallel.mesh import Mesh

PROMPTS = [[3, 14, 15, 92, 65], [35, 89, 79, 32, 38, 46, 26], [43], [38, 32, 79, 50, 28, 84]]


def _gen(preset, mesh, comm, prompts, n=5):
    cfg = ModelConfig.from_preset(preset)
    ecfg = EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048, use_graphs=False, seed=5)
    eng = LLMEngine(cfg, mesh, ecfg, comm=comm, device="cpu")
    return eng.generate(prompts, SamplingParams(max_tokens=n, ignore_eos=True))


@pytest.mark.parametrize("preset,kw", [("llama-tiny", dict(tp=2)), ("llama-tiny", dict(pp=2)),
                                       ("llama-tiny", dict(tp=2, pp=2)), ("mixtral-tiny", dict(tp=2)),
                                       ("llama-small", dict(pp=4))])
def test_fake_world_matches_single(preset, kw):
    torch.set_num_threads(1)
    mesh = Mesh(**kw)
    world = FakeWorld(mesh, timeout_s=60)
    ref = _gen(preset, Mesh(), None, PROMPTS)
    outs = world.run(lambda r, c: _gen(preset, mesh, c, PROMPTS))
    assert all(o == ref for o in outs)
    ops = {op for _, op, _, _, _ in world.log}
    assert ("all_reduce" in ops) == (mesh.tp > 1) and ("send" in ops) == (mesh.pp > 1)


def test_fake_world_expert_parallel():
    torch.set_num_threads(1)
    mesh = Mesh(dp=2, ep=2)
    world = FakeWorld(mesh, timeout_s=60)
    halves = [PROMPTS[:3], PROMPTS[3:]]
    outs = world.run(lambda r, c: _gen("mixtral-tiny", mesh, c, halves[mesh.coord(r).dp]))
    assert outs[0] == _gen("mixtral-tiny", Mesh(), None, halves[0])
    assert outs[1] == _gen("mixtral-tiny", Mesh(), None, halves[1])


def test_order_checker_flags_mismatched_collectives():
    world = FakeWorld(Mesh(tp=2), timeout_s=5)

    def prog(rank, comm):
        x = torch.ones(4 if rank == 0 else 5)
        comm.all_reduce_(x, "tp")

    with pytest.raises(RuntimeError, match="CommOrderError|issued"):
        world.run(prog)


def test_order_checker_flags_unmatched_recv():
    world = FakeWorld(Mesh(pp=2), timeout_s=1)

    def prog(rank, comm):
        if rank == 1:
            comm.recv(torch.empty(3), 0)      # rank 0 never sends

    with pytest.raises(RuntimeError, match="timed out"):
        world.run(prog)
