"""Engine on CPU: continuous batching + paged KV + scheduler produce the same greedy tokens as
step-by-step full recompute."""
import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine.batch import make_prefill_batch
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams


def _greedy_reference(model, prompt, n):
    toks = list(prompt)
    for _ in range(n):
        fb = make_prefill_batch([toks], [[-1] * len(toks)])
        logits = model.forward(fb, None)
        toks.append(int(logits[0, : model.cfg.vocab_size].argmax()))
    return toks[len(prompt):]


def test_engine_greedy_matches_recompute():
    cfg = ModelConfig.from_preset("llama-tiny")
    ecfg = EngineConfig(max_batch=4, max_seq_len=128, kv_cache_tokens=1024, use_graphs=False)
    eng = LLMEngine(cfg, engine_cfg=ecfg, device="cpu")
    prompts = [[1, 2, 3], [7, 8, 9, 10, 11, 12], [42], [5, 5, 5, 5], [100, 200]]
    outs = eng.generate(prompts, SamplingParams(max_tokens=6))
    for p, o in zip(prompts, outs):
        assert o == _greedy_reference(eng.model, p, 6)


def test_engine_preemption_recovers():
    cfg = ModelConfig.from_preset("llama-tiny")
    # tiny KV cache: 4 blocks of 32 tokens -> forces preemption with 3 long sequences
    ecfg = EngineConfig(max_batch=3, max_seq_len=128, kv_cache_tokens=128, use_graphs=False)
    eng = LLMEngine(cfg, engine_cfg=ecfg, device="cpu")
    prompts = [[i + 1] * 30 for i in range(3)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=20))
    for p, o in zip(prompts, outs):
        assert o == _greedy_reference(eng.model, p, 20)


@pytest.mark.parametrize("budget", [7, 16, 64])
def test_mixed_chunked_prefill_matches_unmixed(budget):
    """Chunked prefill mixed into decode steps (scheduler mixed mode): prompts longer than the
    per-step token budget are prefilled over several steps while earlier requests decode; the
    generated tokens must equal the plain prefill-then-decode engine's."""
    from butterfly_amd.config import EngineConfig, ModelConfig
    from butterfly_amd.engine.engine import LLMEngine
    from butterfly_amd.engine.sampler import SamplingParams

    cfg = ModelConfig.from_preset("llama-tiny")
    prompts = [[(5 * i + 3 * j) % 1000 + 1 for j in range(n)] for i, n in enumerate((45, 3, 20, 33, 1, 9))]

    def run(mixed):
        e = LLMEngine(cfg, engine_cfg=EngineConfig(max_batch=4, max_seq_len=128, max_prefill_tokens=budget,
                                                   kv_cache_tokens=1024, use_graphs=False, seed=2,
                                                   mixed_prefill=mixed), device="cpu")
        kinds = set()
        rids = [e.add_request(p, SamplingParams(max_tokens=6 + i, ignore_eos=True)) for i, p in enumerate(prompts)]
        while e.has_unfinished():
            kinds.add(e.step().kind)
        return [e.requests[r].output for r in rids], kinds

    ref, _ = run(False)
    got, kinds = run(True)
    assert got == ref
    assert "mixed" in kinds


def test_prefix_caching_reuses_pages_and_matches():
    """Requests sharing a long prompt prefix: later ones take the cached pages (prefill starts
    after the shared blocks) and generate exactly what an engine without the cache does —
    also after the first owner finished (its pages parked in the LRU, not freed)."""
    cfg = ModelConfig.from_preset("llama-tiny")
    shared = [(13 * j) % 1000 + 1 for j in range(100)]
    prompts = [shared + [5, 6, 7], shared + [9], shared[:64] + [1, 2, 3, 4], shared + [5, 6, 7, 8]]

    def run(cache):
        e = LLMEngine(cfg, engine_cfg=EngineConfig(max_batch=4, max_seq_len=256, max_prefill_tokens=64,
                                                   kv_cache_tokens=2048, use_graphs=False, seed=4,
                                                   prefix_caching=cache), device="cpu")
        first = e.add_request(prompts[0], SamplingParams(max_tokens=5, ignore_eos=True))
        while e.has_unfinished():
            e.step()
        rids = [e.add_request(p, SamplingParams(max_tokens=5, ignore_eos=True)) for p in prompts[1:]]
        while e.has_unfinished():
            e.step()
        return [e.requests[r].output for r in [first] + rids], e.scheduler.prefix_hit_tokens

    ref, hits0 = run(False)
    got, hits = run(True)
    assert got == ref
    assert hits0 == 0 and hits >= 3 * 64      # three later prompts reuse >= 2 blocks of 32


def test_fp8_kv_cache_engine_cpu():
    """kv_cache_dtype="fp8": float8_e4m3fn pages (a quarter of the fp32 CPU bytes), the engine
    runs prefill, mixed steps and decode through them."""

    cfg = ModelConfig.from_preset("llama-tiny")
    base = dict(max_batch=4, max_seq_len=96, kv_cache_tokens=512, use_graphs=False)
    e8 = LLMEngine(cfg, engine_cfg=EngineConfig(kv_cache_dtype="fp8", **base), device="cpu")
    e32 = LLMEngine(cfg, engine_cfg=EngineConfig(**base), device="cpu")
    assert e8.kv.layers[0][0].dtype == torch.float8_e4m3fn
    assert e8.kv.bytes() * 4 == e32.kv.bytes()
    prompts = [[3, 1, 4, 1, 5, 9, 2, 6] * 3, [7, 7, 2]]
    out = e8.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
    assert [len(o) for o in out] == [6, 6]
    with pytest.raises(ValueError):
        LLMEngine(cfg, engine_cfg=EngineConfig(kv_cache_dtype="int4", **base), device="cpu")


def test_nan_fault_fails_the_step(monkeypatch):
    """BFLY_FAULT=rank:step:nan poisons that step's logits; the engine's non-finite check
    turns it into an error instead of emitting tokens (SURVEY.md §5.3 fault injection)."""
    monkeypatch.setenv("BFLY_FAULT", "0:2:nan")
    cfg = ModelConfig.from_preset("llama-tiny")
    ecfg = EngineConfig(max_batch=2, max_seq_len=64, kv_cache_tokens=256, use_graphs=False)
    eng = LLMEngine(cfg, engine_cfg=ecfg, device="cpu")
    eng.add_request([1, 2, 3], SamplingParams(max_tokens=8))
    eng.step()
    eng.step()
    with pytest.raises(RuntimeError, match="non-finite"):
        # the overlapped engine reads a step's token values two steps later
        for _ in range(3 if eng.async_pp else 1):
            eng.step()
