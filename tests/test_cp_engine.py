"""Context-parallel prefill inside the serving engine (engine/engine.py `_cp_step`) on
CPU/gloo: data-parallel replicas prefill each other's long prompts together (ring or Ulysses
attention) and the owning replica's cache collects the whole prompt's K/V on the way, then
decodes it alone. Every replica must generate exactly the tokens the single-process engine
generates for its prompts, its K/V pages must all be returned, and the CP steps must really
have run (each replica computed only its chunk of every long prompt)."""
import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams
from butterfly_amd.parallel.mesh import Mesh

from .dist_utils import run_world

LONG_A = [(11 * i + 5) % 900 + 2 for i in range(45)]
LONG_B = [(13 * i + 7) % 800 + 3 for i in range(61)]
LONG_C = [(17 * i + 1) % 700 + 4 for i in range(33)]
SHORT = [[3, 14, 15, 92, 65], [35, 89, 79, 32, 38, 46, 26], [43]]
PER_DP = [[LONG_A, SHORT[0]], [SHORT[1], LONG_B, LONG_C, SHORT[2]]]


def _ecfg(cp_min=0, attn="ring", mixed=True, async_decode=True):
    return EngineConfig(max_batch=8, max_seq_len=160, kv_cache_tokens=2048, use_graphs=False, seed=5,
                        cp_prefill_min_tokens=cp_min, cp_attention=attn, mixed_prefill=mixed,
                        async_decode=async_decode)


def _single(prompts, max_tokens, mixed=True):
    cfg = ModelConfig.from_preset("llama-tiny")
    eng = LLMEngine(cfg, Mesh(), _ecfg(mixed=mixed), device="cpu")
    return eng.generate(prompts, SamplingParams(max_tokens=max_tokens, ignore_eos=True))


def _cp_generate(rank, world, mesh_kw, attn, max_tokens, mixed, async_decode=True):
    from butterfly_amd.parallel.comm import Communicator

    mesh = Mesh(**mesh_kw)
    comm = Communicator.from_mesh(mesh)
    cfg = ModelConfig.from_preset("llama-tiny")
    eng = LLMEngine(cfg, mesh, _ecfg(cp_min=20, attn=attn, mixed=mixed, async_decode=async_decode), comm=comm,
                    device="cpu")
    # CP prefill no longer switches the serving engine to the synchronous one
    assert eng.cp_min == 20 and eng.async_pp == async_decode
    outs = eng.generate(PER_DP[mesh.coord(rank).dp], SamplingParams(max_tokens=max_tokens, ignore_eos=True))
    m = eng.kv.manager
    return outs, eng.metrics.counters.get("cp_prefill_tokens", 0), m.num_free == m.num_blocks


@pytest.mark.parametrize("mesh_kw,world,attn,mixed,async_decode", [
    (dict(dp=2), 2, "ring", True, True),
    (dict(dp=2), 2, "ring", True, False),
    (dict(dp=2), 2, "ulysses", False, True),
    (dict(dp=2, tp=2), 4, "ring", True, True),
])
def test_cp_prefill_engine_matches_single(mesh_kw, world, attn, mixed, async_decode):
    n = 5
    want = [_single(p, n, mixed) for p in PER_DP]
    outs = run_world(_cp_generate, world, mesh_kw, attn, n, mixed, async_decode)
    mesh = Mesh(**mesh_kw)
    long_tokens = len(LONG_A) + len(LONG_B) + len(LONG_C)
    for rank, (got, cp_tokens, all_free) in enumerate(outs):
        assert got == want[mesh.coord(rank).dp]
        assert all_free
        # each replica ran ~half of every long prompt (chunks of 45/61/33 over 2 ranks)
        assert long_tokens // 2 - 2 <= cp_tokens <= long_tokens // 2 + 2, cp_tokens


def test_cp_off_for_single_replica():
    cfg = ModelConfig.from_preset("llama-tiny")
    eng = LLMEngine(cfg, Mesh(), _ecfg(cp_min=20), device="cpu")
    assert eng.cp_min == 0 and not eng.lockstep_dp
