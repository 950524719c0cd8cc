"""The GEMM planner (csrc/kernels/gemm.hip plan_gemm) must only emit plans that have an
instantiated kernel, for every model shape and token count the engine can produce. Runs on
CPU: plan selection and validation are host code (`gemm_check` is a dry run of the launcher)."""
import pytest
import torch

from butterfly_amd import ops
from butterfly_amd.config import ModelConfig
from butterfly_amd.models.shard import Shard, local_dims

pytestmark = pytest.mark.skipif(not ops.load_library(), reason="kernel library not built")


def model_shapes(preset, tp):
    c = ModelConfig.from_preset(preset)
    d = local_dims(c, Shard(tp_rank=0, tp_size=tp, layer_start=0, layer_end=c.num_layers))
    D = c.head_dim
    out = [((d.hq + 2 * d.hkv) * D, c.hidden_size, 1),        # qkv (bias for gpt2)
           (c.hidden_size, d.hq * D, 1),                      # o
           (d.vocab, c.hidden_size, 0)]                       # lm head
    if c.is_moe:
        out += [(2 * c.intermediate_size * d.experts, c.hidden_size, 2),
                (c.hidden_size, c.intermediate_size * d.experts, 0)]
    elif c.act == "silu":
        out += [(2 * d.ffn, c.hidden_size, 2), (c.hidden_size, d.ffn, 0)]
    else:
        out += [(d.ffn, c.hidden_size, 1), (c.hidden_size, d.ffn, 1)]
    return out


@pytest.mark.parametrize("preset,tp", [("llama3-70b", 1), ("llama3-70b", 2), ("llama3-70b", 8),
                                       ("llama3-8b", 1), ("llama3-8b", 4), ("mixtral-8x7b", 1),
                                       ("gpt2-small", 1), ("llama-small", 1), ("llama-tiny", 1)])
def test_every_plan_is_instantiated(preset, tp):
    Ms = list(range(1, 130)) + [160, 192, 255, 256, 300, 512, 1000, 1024, 2048, 4096, 8192, 16384]
    for N, K, epi in model_shapes(preset, tp):
        if N % 128 or K % 64:
            continue     # the op rejects these up front (the model pads to avoid them)
        for M in Ms:
            rc = torch.ops.bfly.gemm_check(M, N, K, epi)
            assert rc == 0, (preset, tp, M, N, K, epi, rc, torch.ops.bfly.gemm_plan(M, N, K))


def test_in_situ_plan_choices_are_in_the_table():
    """Every whole-step (in-situ) A/B choice pinned in tools/gen_gemm_table.py (INSITU) is an
    entry of the generated gemm_tuned.inc with that plan, and plan_gemm returns it (a pinned
    choice that the generator dropped would silently fall back to the sweep's or the heuristic
    plan)."""
    import importlib.util
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("gen_gemm_table", os.path.join(root, "tools", "gen_gemm_table.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    table = {}
    for ln in open(os.path.join(root, "csrc", "kernels", "gemm_tuned.inc")):
        m = re.match(r"\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)\}", ln)
        if m:
            v = [int(x) for x in m.groups()]
            table[tuple(v[:3])] = v[3:]
    kinds = ("skinny", "tile", "big", "dec", "big8", "mid8", "big4", "mid4")
    for (N, K, M), (pl, _) in mod.INSITU.items():
        assert table.get((N, K, M)) == pl, ((N, K, M), table.get((N, K, M)), pl)
        p = ops.gemm_plan(M, N, K)
        got = [kinds.index(p["kind"]), p["mt"], p["nt"], p["wk"], p["bm"], p["bn"], p["splitk"]]
        assert got == pl, ((N, K, M), got, pl)
