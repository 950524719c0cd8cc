"""Python API + HTTP server (single process, CPU reference path)."""
import threading

import pytest

from butterfly_amd import SamplingParams
from butterfly_amd.config import EngineConfig


def _llm():
    from butterfly_amd.api import LLM

    return LLM("llama-tiny", engine_config=EngineConfig(max_batch=4, max_seq_len=128, kv_cache_tokens=1024, use_graphs=False))


def test_llm_generate_text_and_ids():
    llm = _llm()
    outs = llm.generate(["hello", [5, 6, 7]], SamplingParams(max_tokens=5, ignore_eos=True))
    assert len(outs) == 2 and all(len(o.token_ids) == 5 for o in outs)
    assert isinstance(outs[0].text, str) and outs[1].text is None
    assert outs[0].ttft_s is not None and outs[0].finish_reason == "length"
    again = llm.generate([[5, 6, 7]], SamplingParams(max_tokens=5, ignore_eos=True))
    assert again[0].token_ids == outs[1].token_ids


def test_http_completions():
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient

    from butterfly_amd.server import ServingLoop, create_app

    llm = _llm()
    loop = ServingLoop(llm)
    th = threading.Thread(target=loop.run, daemon=True)
    th.start()
    try:
        c = TestClient(create_app(loop))
        assert c.get("/health").json()["status"] == "ok"
        r = c.post("/v1/completions", json={"prompt": [1, 2, 3], "max_tokens": 4}).json()
        assert len(r["choices"][0]["token_ids"]) == 4 and r["usage"]["prompt_tokens"] == 3
        r2 = c.post("/v1/completions", json={"prompt": "hi there", "max_tokens": 3}).json()
        assert isinstance(r2["choices"][0]["text"], str)
        assert "bfly_steps_decode" in c.get("/metrics").text
        # server-sent events: one event per generated token, then the finish event and [DONE]
        import json

        with c.stream("POST", "/v1/completions", json={"prompt": [1, 2, 3], "max_tokens": 4, "stream": True}) as resp:
            events = [ln[len("data: "):] for ln in resp.iter_lines() if ln.startswith("data: ")]
        assert events[-1] == "[DONE]"
        chunks = [json.loads(e)["choices"][0] for e in events[:-1]]
        assert [t for ch in chunks for t in ch["token_ids"]] == r["choices"][0]["token_ids"]
        assert chunks[-1]["finish_reason"] == "length"
    finally:
        loop.stop = True
        th.join(timeout=30)
