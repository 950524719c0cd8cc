"""Model IR (models/ir.py): parameter accounting and the cost model built on it."""
import pytest

from butterfly_amd.config import ModelConfig
from butterfly_amd.models.ir import build_ir
from butterfly_amd.partition.costmodel import CostModel


@pytest.mark.parametrize("preset", ["llama3-8b", "llama3-70b", "mixtral-8x7b", "gpt2-small", "llama-tiny"])
def test_ir_param_count_matches_config(preset):
    c = ModelConfig.from_preset(preset)
    ir = build_ir(c)
    vpad = -(-c.vocab_size // 128) * 128
    pad = (vpad - c.vocab_size) * c.hidden_size * (1 if c.tie_embeddings else 2)
    assert ir.param_elems == c.param_count() + pad


@pytest.mark.parametrize("tp", [2, 4, 8])
def test_ir_tp_shards_partition_the_layer(tp):
    c = ModelConfig.from_preset("llama3-70b")
    full = build_ir(c, 1).layers[0]
    part = build_ir(c, tp).layers[0]
    h = c.hidden_size
    replicated = 2 * h                          # the two norms live on every TP rank
    assert (part.param_elems - replicated) * tp == full.param_elems - replicated
    kinds = [o.collective for o in part.ops if o.kind == "collective"]
    assert kinds == ["all_reduce", "all_reduce"]


def test_ir_moe_ep_ops():
    c = ModelConfig.from_preset("mixtral-8x7b")
    layer = build_ir(c, 1, ep=8).layers[0]
    names = [o.name for o in layer.ops]
    assert names.index("ep_dispatch") < names.index("experts_gate_up") < names.index("ep_combine")
    # routed decode: top-k slot rows per token, split over the local experts (grouped GEMM),
    # dispatched and returned by all-to-all
    g = layer.op("experts_gate_up")
    assert g.m_scale == c.experts_per_token and g.groups == 1 and g.n == 2 * c.intermediate_size
    assert [o.collective for o in layer.ops if o.kind == "collective"] == ["all_to_all", "all_to_all"]
    l2 = build_ir(c, 1, ep=2).layers[0]
    assert l2.op("experts_down").groups == 4


def test_costmodel_decode_is_weight_bound_at_small_batch():
    c = ModelConfig.from_preset("llama3-70b")
    cm = CostModel(c)
    t1 = cm.layer_time(1, 1, 1024, True).seconds
    t64 = cm.layer_time(64, 1, 1024, True).seconds
    w = cm.layer_weight_bytes(1)
    assert t1 >= w / cm.hw.hbm_bw            # never faster than peak HBM streaming
    assert t64 < 2 * t1                         # decode GEMMs stay weight-streaming bound
    assert cm.layer_time(64, 2, 1024, True).comm_bytes == 2 * 2 * 64 * c.hidden_size
