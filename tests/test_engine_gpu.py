"""End-to-end on one MI355X: the HIP-kernel model vs the fp32 reference-op model with the SAME
weights (prefill and paged decode logits), hipGraph replay == eager, and engine generation."""
import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine.batch import make_decode_batch, make_prefill_batch
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams
from butterfly_amd.models import build_model

pytestmark = pytest.mark.gpu


def _pair(preset):
    cfg = ModelConfig.from_preset(preset)
    g = build_model(cfg, device="cuda", dtype=torch.bfloat16)
    g.init_random(seed=7)
    c = build_model(cfg, device="cpu", dtype=torch.float32)
    for k, v in g.p.items():
        c.p[k].copy_(v.float().cpu())
    return cfg, g, c


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("preset", ["llama-small", "mixtral-tiny", "llama-tiny"])
def test_prefill_and_decode_logits_match_reference(preset):
    cfg, g, c = _pair(preset)
    bs = 32
    prompts = [[3, 1, 4, 1, 5, 9, 2, 6] * 9, list(range(1, 40)), [7]]
    tables, slots, nxt = [], [], 0
    for p in prompts:
        nb = (len(p) + 8 + bs - 1) // bs
        tables.append(list(range(nxt, nxt + nb)))
        nxt += nb
        slots.append([tables[-1][j // bs] * bs + j % bs for j in range(len(p))])
    kg = g.allocate_kv_cache(nxt + 1, bs)
    kc = c.allocate_kv_cache(nxt + 1, bs)
    fb = make_prefill_batch(prompts, slots)
    lg = g.forward(fb.to("cuda"), kg)
    lc = c.forward(fb, kc)
    V = cfg.vocab_size
    assert _rel(lg[:, :V], lc[:, :V]) < 2e-2
    toks = [int(t) for t in lc[:, :V].argmax(-1)]
    pos = [len(p) for p in prompts]
    sl = [tables[i][pos[i] // bs] * bs + pos[i] % bs for i in range(len(prompts))]
    mb = max(len(t) for t in tables)
    db = make_decode_batch(toks, pos, sl, tables, mb, mb * bs)
    dg = g.forward(db.to("cuda"), kg)
    dc = c.forward(db, kc)
    assert _rel(dg[:, :V], dc[:, :V]) < 3e-2


def test_engine_graph_replay_matches_eager():
    cfg = ModelConfig.from_preset("llama-small")
    prompts = [[i + 1, 2 * i + 3, 5] * 7 for i in range(6)]
    outs = []
    for graphs in (False, True):
        ecfg = EngineConfig(max_batch=8, max_seq_len=256, kv_cache_tokens=4096, use_graphs=graphs,
                            graph_batch_sizes=[4, 8], seed=11)
        eng = LLMEngine(cfg, engine_cfg=ecfg, device="cuda")
        outs.append(eng.generate(prompts, SamplingParams(max_tokens=12, ignore_eos=True)))
    assert outs[0] == outs[1]


@pytest.mark.parametrize("params", [dict(temperature=0.0), dict(temperature=0.9, seed=5),
                                    dict(temperature=0.7, top_k=20, seed=2)])
def test_graph_sampling_matches_eager(params, monkeypatch):
    """Decode steps whose tokens come from the sampler captured at the end of the hipGraph
    (per-request temperatures / seeds in the graph's static inputs) give the tokens of eager
    steps with the eager sampler; top-k rows fall back to eager sampling of the graph's
    logits. The engine replays exactly one graph per decode step."""
    cfg = ModelConfig.from_preset("llama-small")
    prompts = [[i + 1, 2 * i + 3, 5] * 7 for i in range(6)]
    outs, replays = [], []
    for graphs in (False, True):
        ecfg = EngineConfig(max_batch=8, max_seq_len=256, kv_cache_tokens=4096, use_graphs=graphs,
                            graph_batch_sizes=[8], seed=11)
        eng = LLMEngine(cfg, engine_cfg=ecfg, device="cuda")
        assert eng.async_pp and (eng.runner.sample_fn is not None)
        n = {"replay": 0, "eager_sample": 0}
        orig = torch.cuda.CUDAGraph.replay
        orig_sample = eng._sample_eager

        def count_replay(self, _o=orig):
            n["replay"] += 1
            return _o(self)

        def count_sample(*a, _o=orig_sample):
            n["eager_sample"] += 1
            return _o(*a)

        monkeypatch.setattr(torch.cuda.CUDAGraph, "replay", count_replay)
        monkeypatch.setattr(eng, "_sample_eager", count_sample)
        outs.append(eng.generate(prompts, SamplingParams(max_tokens=12, ignore_eos=True, **params)))
        monkeypatch.setattr(torch.cuda.CUDAGraph, "replay", orig)
        replays.append(dict(n))
    assert outs[0] == outs[1]
    g = replays[1]
    assert g["replay"] > 0
    if params.get("top_k"):
        assert g["eager_sample"] >= g["replay"]     # filtered rows: eager sampling of the logits
    else:
        assert g["eager_sample"] <= 2                # only the prefill steps sample eagerly


def test_engine_temperature_sampling_runs():
    cfg = ModelConfig.from_preset("llama-tiny")
    eng = LLMEngine(cfg, engine_cfg=EngineConfig(max_batch=4, max_seq_len=128, kv_cache_tokens=2048), device="cuda")
    out = eng.generate([[1, 2, 3], [4, 5]], SamplingParams(max_tokens=8, temperature=0.8, seed=3))
    assert all(len(o) == 8 for o in out)
    assert all(0 <= t < cfg.vocab_size for o in out for t in o)


def test_mixed_chunked_step_matches_reference():
    """A mixed step (decode row + a prompt chunk attending to its cached prefix through the
    LSE-merged flash prefill) on the HIP kernels vs the fp32 reference ops."""
    from butterfly_amd.engine.batch import ForwardBatch

    cfg, g, c = _pair("llama-small")
    bs, V = 32, cfg.vocab_size
    A = [(7 * j) % 3000 + 1 for j in range(90)]
    B = [(11 * j) % 3000 + 2 for j in range(20)]
    # cache: A in blocks 0..2, B in blocks 4..5
    sa = [j for j in range(90)]
    sb = [4 * bs + j for j in range(21)]
    kg, kc = g.allocate_kv_cache(8, bs), c.allocate_kv_cache(8, bs)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    # step 1: A[0:40) (not final) + B (final) as plain prefill
    fb1 = ForwardBatch(input_ids=i32(A[:40] + B), positions=i32(list(range(40)) + list(range(20))),
                       slots=i32(sa[:40] + sb[:20]), is_prefill=True, cu_seqlens=i32([0, 40, 60]), max_seqlen=40,
                       logits_idx=torch.tensor([59]))
    l1g, l1c = g.forward(fb1.to("cuda"), kg), c.forward(fb1, kc)
    assert _rel(l1g[:, :V], l1c[:, :V]) < 5e-2      # one bf16 row vs fp32 (wrong would be O(1))
    tok = int(l1c[0, :V].argmax())
    # step 2: decode row for B + chunk A[40:90) with a 40-token cached prefix
    fb2 = ForwardBatch(input_ids=i32([tok] + A[40:]), positions=i32([20] + list(range(40, 90))),
                       slots=i32([sb[20]] + sa[40:]), is_prefill=True, cu_seqlens=i32([0, 50]), max_seqlen=50,
                       block_tables=i32([[4, 5, 0]]), ctx_lens=i32([21]), max_ctx=96,
                       logits_idx=torch.tensor([0, 50]), num_decode=1, prefix_lens=[40], prefix_cu=i32([0, 40]),
                       prefix_tables=i32([[0, 1, 2]]))
    l2g, l2c = g.forward(fb2.to("cuda"), kg), c.forward(fb2, kc)
    assert _rel(l2g[:, :V], l2c[:, :V]) < 5e-2
    # and the chunked prompt's last-token logits equal a whole-prompt prefill's
    kw = c.allocate_kv_cache(8, bs)
    whole = c.forward(ForwardBatch(input_ids=i32(A), positions=i32(list(range(90))), slots=i32(sa), is_prefill=True,
                                   cu_seqlens=i32([0, 90]), max_seqlen=90, logits_idx=torch.tensor([89])), kw)
    assert _rel(l2c[1:2, :V], whole[:, :V]) < 1e-4


def test_engine_fp8_kv_cache():
    """FP8 KV cache end to end (HIP rope/append + decode attention, hipGraphs, mixed prefill):
    the engine runs, and the first token (from the prefill, which reads no cache) matches
    the bf16-cache engine's. Decode logits are compared at model level below."""
    cfg = ModelConfig.from_preset("llama-small")
    prompts = [[i + 1, 2 * i + 3, 5] * 9 for i in range(5)]
    outs = {}
    for kvd in ("auto", "fp8"):
        eng = LLMEngine(cfg, engine_cfg=EngineConfig(max_batch=8, max_seq_len=128, kv_cache_tokens=2048,
                                                     kv_cache_dtype=kvd, graph_batch_sizes=[8]))
        assert eng.kv.layers[0][0].dtype == (torch.float8_e4m3fn if kvd == "fp8" else torch.bfloat16)
        outs[kvd] = eng.generate(prompts, SamplingParams(max_tokens=12, ignore_eos=True))
    assert all(len(o) == 12 for o in outs["fp8"])
    assert [o[0] for o in outs["fp8"]] == [o[0] for o in outs["auto"]]


def test_fp8_kv_decode_logits_close_to_bf16():
    cfg = ModelConfig.from_preset("llama-small")
    g = build_model(cfg, device="cuda", dtype=torch.bfloat16)
    g.init_random(seed=7)
    bs = 32
    prompts = [list(range(1, 70)), [3, 1, 4, 1, 5] * 20, [9]]
    tables, slots, nxt = [], [], 0
    for p in prompts:
        nb = (len(p) + 8 + bs - 1) // bs
        tables.append(list(range(nxt, nxt + nb)))
        nxt += nb
        slots.append([tables[-1][j // bs] * bs + j % bs for j in range(len(p))])
    logits = {}
    for dt in (torch.bfloat16, torch.float8_e4m3fn):
        kv = g.allocate_kv_cache(nxt + 1, bs, dt)
        fb = make_prefill_batch(prompts, slots)
        lp = g.forward(fb.to("cuda"), kv)
        toks = [int(t) for t in lp[:, :cfg.vocab_size].argmax(-1)]
        pos = [len(p) for p in prompts]
        sl = [tables[i][pos[i] // bs] * bs + pos[i] % bs for i in range(len(prompts))]
        mb = max(len(t) for t in tables)
        db = make_decode_batch(toks, pos, sl, tables, mb, mb * bs)
        logits[dt] = g.forward(db.to("cuda"), kv)[:, :cfg.vocab_size]
    assert _rel(logits[torch.float8_e4m3fn], logits[torch.bfloat16]) < 0.1


@pytest.mark.parametrize("preset", ["llama-small", "mixtral-tiny"])
def test_poisoned_outputs_change_nothing(preset):
    """Output poisoning (ops.set_poison): with every op output allocated as NaN
    / a negative sentinel, prefill and decode logits are bitwise those of the normal run — no
    kernel leaves an element of its output unwritten."""
    from butterfly_amd import ops

    cfg = ModelConfig.from_preset(preset)
    g = build_model(cfg, device="cuda", dtype=torch.bfloat16)
    g.init_random(seed=7)
    bs = 32
    prompts = [[3, 1, 4, 1, 5, 9, 2, 6] * 9, list(range(1, 40)), [7]]
    outs = []
    for poison in (False, True):
        ops.set_poison(poison)
        try:
            tables, slots, nxt = [], [], 0
            for p in prompts:
                nb = (len(p) + 8 + bs - 1) // bs
                tables.append(list(range(nxt, nxt + nb)))
                nxt += nb
                slots.append([tables[-1][j // bs] * bs + j % bs for j in range(len(p))])
            kg = g.allocate_kv_cache(nxt + 1, bs)
            lg = g.forward(make_prefill_batch(prompts, slots).to("cuda"), kg)
            toks = [int(t) for t in lg[:, :cfg.vocab_size].argmax(-1)]
            pos = [len(p) for p in prompts]
            sl = [tables[i][pos[i] // bs] * bs + pos[i] % bs for i in range(len(prompts))]
            mb = max(len(t) for t in tables)
            dg = g.forward(make_decode_batch(toks, pos, sl, tables, mb, mb * bs).to("cuda"), kg)
            torch.cuda.synchronize()
            outs.append((lg.clone(), dg.clone()))
        finally:
            ops.set_poison(False)
    V = cfg.vocab_size
    for a, b in zip(outs[0], outs[1]):
        assert torch.isfinite(b[:, :V].float()).all()
        assert torch.equal(a[:, :V], b[:, :V])
