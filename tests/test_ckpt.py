"""Checkpoint format: save under one plan, load under another (resharding), offline reshard,
and HuggingFace import checked against transformers' own forward (parity oracle)."""
import json

import pytest
import torch

from butterfly_amd.ckpt import format as ck
from butterfly_amd.ckpt.hf import convert_hf
from butterfly_amd.config import ModelConfig
from butterfly_amd.engine.batch import make_prefill_batch
from butterfly_amd.models import Shard, build_model
from butterfly_amd.partition import partition


def _globals(m):
    return {lp.name: lp.get().clone() for lp in m.logical_params() if lp.owner}


@pytest.mark.parametrize("preset", ["llama-tiny", "mixtral-tiny", "gpt2-tiny"])
def test_save_tp2_load_tp1_and_pp2(tmp_path, preset):
    cfg = ModelConfig.from_preset(preset)
    ref = build_model(cfg, dtype=torch.float32)
    ref.init_random(seed=9)
    # write as a TP=2 checkpoint (two ranks written sequentially in-process)
    for r in range(2):
        m = build_model(cfg, Shard(tp_rank=r, tp_size=2), dtype=torch.float32)
        m.init_random(seed=9)
        ck._write_rank(m, tmp_path, r, None)
    ck._write_manifest(tmp_path, 2, cfg, {"tp": 2}, "f32")
    man = json.loads((tmp_path / "manifest.json").read_text())
    assert man["format"] == "butterfly-ckpt" and man["version"] == 1
    # load whole (TP=1)
    one = build_model(cfg, dtype=torch.float32)
    ck.load_into(one, tmp_path)
    g_ref, g_one = _globals(ref), _globals(one)
    assert g_ref.keys() == g_one.keys()
    for k in g_ref:
        assert torch.equal(g_ref[k], g_one[k]), k
    # load into a 2-stage pipeline shard
    st = build_model(cfg, Shard(layer_start=1, layer_end=2), dtype=torch.float32)
    ck.load_into(st, tmp_path)
    for lp in st.logical_params():
        if lp.name in g_ref and lp.split_dim is None:
            assert torch.equal(lp.get(), g_ref[lp.name]), lp.name


def test_offline_reshard_roundtrip(tmp_path):
    cfg = ModelConfig.from_preset("llama-tiny")
    m = build_model(cfg, dtype=torch.bfloat16)
    m.init_random(seed=2)
    ck.save(m, tmp_path / "a", dtype=torch.bfloat16)
    plan = partition(cfg, 4, {"tp": 2, "pp": 2}, batch_per_gpu=4, ctx=64)
    ck.reshard(tmp_path / "a", tmp_path / "b", plan)
    man = ck.read_manifest(tmp_path / "b")
    assert man["plan"]["tp"] == 2 and man["plan"]["pp"] == 2
    back = build_model(cfg, dtype=torch.bfloat16)
    ck.load_into(back, tmp_path / "b")
    for k, v in _globals(m).items():
        assert torch.equal(v, _globals(back)[k]), k


def _hf_logits_vs_ours(hf_model, tmp_path, ids):
    hf_model.save_pretrained(tmp_path / "hf", safe_serialization=True)
    cfg = convert_hf(tmp_path / "hf", tmp_path / "ck", dtype=torch.float32)
    ours = build_model(cfg, dtype=torch.float32)
    ck.load_into(ours, tmp_path / "ck")
    with torch.no_grad():
        ref = hf_model(torch.tensor([ids])).logits[0].float()
    fb = make_prefill_batch([ids], [[-1] * len(ids)])
    fb.logits_idx = torch.arange(len(ids))
    got = ours.forward(fb, None)[:, : cfg.vocab_size]
    return got, ref


def test_hf_llama_parity(tmp_path):
    transformers = pytest.importorskip("transformers")
    c = transformers.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                 num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                                 rope_theta=500000.0, max_position_embeddings=256, rms_norm_eps=1e-5)
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(c).eval()
    got, ref = _hf_logits_vs_ours(m, tmp_path, [1, 5, 9, 33, 100, 7, 250])
    assert torch.allclose(got, ref, atol=2e-4, rtol=1e-3), (got - ref).abs().max()


def test_hf_gpt2_parity(tmp_path):
    transformers = pytest.importorskip("transformers")
    c = transformers.GPT2Config(vocab_size=512, n_embd=128, n_layer=2, n_head=2, n_positions=128)
    torch.manual_seed(0)
    m = transformers.GPT2LMHeadModel(c).eval()
    got, ref = _hf_logits_vs_ours(m, tmp_path, [1, 5, 9, 33, 100, 7])
    assert torch.allclose(got, ref, atol=2e-4, rtol=1e-3), (got - ref).abs().max()


def test_hf_mixtral_parity(tmp_path):
    transformers = pytest.importorskip("transformers")
    c = transformers.MixtralConfig(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, head_dim=32,
                                   num_local_experts=4, num_experts_per_tok=2, max_position_embeddings=256)
    torch.manual_seed(0)
    m = transformers.MixtralForCausalLM(c).eval()
    got, ref = _hf_logits_vs_ours(m, tmp_path, [1, 5, 9, 33, 100])
    assert torch.allclose(got, ref, atol=2e-4, rtol=1e-3), (got - ref).abs().max()
