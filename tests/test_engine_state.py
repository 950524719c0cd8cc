"""Request-state snapshots (engine/state.py, SURVEY.md §5.4 "resume = reload weights + replay
request state"): an engine interrupted mid-generation and restored into a fresh engine must
produce the same tokens as an uninterrupted run — greedy and seeded temperature sampling, with
the synchronous (mixed chunked prefill) and the overlapped (async decode) step loops."""
import json

import pytest
import torch

from butterfly_amd.config import EngineConfig, ModelConfig
from butterfly_amd.engine import state
from butterfly_amd.engine.engine import LLMEngine
from butterfly_amd.engine.sampler import SamplingParams

PROMPTS = [[(7 * i + 3 * j) % 900 + 1 for j in range(n)] for i, n in enumerate((12, 3, 40, 7, 25))]


def _params(i):
    if i % 2:
        return SamplingParams(max_tokens=5 + 2 * i, temperature=0.8, seed=100 + i, ignore_eos=True)
    return SamplingParams(max_tokens=5 + 2 * i, ignore_eos=True)


def _engine(async_decode, **kw):
    torch.set_num_threads(1)
    cfg = ModelConfig.from_preset("llama-tiny")
    ecfg = EngineConfig(max_batch=4, max_seq_len=128, max_prefill_tokens=32, kv_cache_tokens=2048,
                        use_graphs=False, seed=3, async_decode=async_decode, **kw)
    return LLMEngine(cfg, engine_cfg=ecfg, device="cpu")


def _run_all(eng):
    while eng.has_unfinished():
        eng.step()
    return {r: list(q.output) for r, q in eng.requests.items()}


@pytest.mark.parametrize("async_decode", [False, True])
@pytest.mark.parametrize("stop_after", [3, 9])
def test_resume_matches_uninterrupted(async_decode, stop_after, tmp_path):
    ref = _engine(async_decode)
    for i, p in enumerate(PROMPTS):
        ref.add_request(p, _params(i))
    want = _run_all(ref)

    a = _engine(async_decode)
    for i, p in enumerate(PROMPTS):
        a.add_request(p, _params(i))
    for _ in range(stop_after):
        a.step()
    path = tmp_path / "replica-000.json"
    a.save_state(path)
    snap = json.loads(path.read_text())
    assert snap["format"] == state.FORMAT and len(snap["requests"]) == len(PROMPTS)
    assert any(r["output"] for r in snap["requests"])            # interrupted mid-generation
    assert not all(r["finished"] for r in snap["requests"])

    b = _engine(async_decode)                                     # fresh engine, same weights
    rids = b.restore(state.load(path))
    assert sorted(rids) == sorted(want)
    got = _run_all(b)
    assert got == want
    # ids handed out after a restore do not collide with restored ones
    assert b.add_request([1, 2, 3], SamplingParams(max_tokens=2)) == max(want) + 1


def test_periodic_snapshots_and_api_resume(tmp_path):
    from butterfly_amd.api import LLM

    eng = _engine(False, snapshot_dir=str(tmp_path), snapshot_every=2)
    for i, p in enumerate(PROMPTS):
        eng.add_request(p, _params(i))
    for _ in range(4):
        eng.step()
    snap = state.load(state.replica_path(tmp_path, 0))
    assert snap["steps_done"] == 4 and not list(tmp_path.glob("*.tmp*"))
    ref = _run_all(eng)

    llm = LLM("llama-tiny", plan=None, engine_config=EngineConfig(max_batch=4, max_seq_len=128,
                                                                 max_prefill_tokens=32, kv_cache_tokens=2048,
                                                                 use_graphs=False, seed=3))
    outs = llm.resume(tmp_path)
    assert [o.token_ids for o in outs] == [ref[r] for r in sorted(ref)]
    assert all(o.finish_reason == "length" for o in outs)


def test_restore_rejects_other_model(tmp_path):
    eng = _engine(False)
    eng.add_request([1, 2], SamplingParams(max_tokens=2))
    snap = eng.snapshot()
    snap["model"] = "llama3-70b"
    with pytest.raises(ValueError):
        _engine(False).restore(snap)


def test_launcher_restart_resumes_from_snapshot(tmp_path):
    """Failure -> recovery end to end (CPU, gloo, TP2): rank 1 dies at engine step 7 of the first
    attempt (BFLY_FAULT=1:7:exit), the launcher takes the job down and starts it again
    (--max-restarts 1), and the new job resumes the request state snapshotted every 2 steps.
    Its outputs equal an uninterrupted run's."""
    import os
    import subprocess
    import sys

    def run(extra_env, launch_args, snap):
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        env.update(OMP_NUM_THREADS="2", BFLY_DIST_BACKEND="gloo", BFLY_FORCE_CPU="1", BFLY_HEARTBEAT_S="0",
                   **extra_env)
        cmd = [sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", *launch_args, "--",
               sys.executable, "-m", "butterfly_amd", "generate", "--model", "llama-tiny", "--plan", "tp2",
               "--max-tokens", "12", "--temperature", "0.7", "--seed", "5", "--no-graphs",
               "--prompt", "abc", "--prompt", "hello world", "--prompt", "x"]
        if snap:
            cmd += ["--snapshot-dir", str(snap), "--snapshot-every", "2"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        lines = [l.split("] ", 1)[1] for l in r.stdout.splitlines() if l.startswith("[rank0] {")]
        return [json.loads(l)["token_ids"] for l in lines], r.stdout + r.stderr

    want, _ = run({}, [], None)
    got, log = run({"BFLY_FAULT": "1:7:exit"}, ["--max-restarts", "1"], tmp_path)
    assert "restart 1/1" in log and "resumed 3 requests" in log, log[-3000:]
    assert got == want and len(want) == 3 and all(len(t) == 12 for t in want)


def test_snapshot_job_identity(tmp_path):
    """A restarted job resumes only a snapshot carrying its own job fingerprint (ADVICE r2:
    a stale snapshot of an earlier job in the same directory must never be replayed)."""
    p1 = SamplingParams(max_tokens=4, temperature=0.7, seed=5)
    job_a = state.job_fingerprint("llama-tiny", ["abc", "x"], p1)
    assert job_a == state.job_fingerprint("llama-tiny", ["abc", "x"], SamplingParams(max_tokens=4, temperature=0.7, seed=5))
    assert job_a != state.job_fingerprint("llama-tiny", ["abc", "y"], p1)
    assert job_a != state.job_fingerprint("llama-tiny", ["abc", "x"], SamplingParams(max_tokens=5, temperature=0.7, seed=5))
    eng = _engine(False)
    eng.job_id = job_a
    eng.add_request([1, 2], SamplingParams(max_tokens=2))
    path = state.save(eng, state.replica_path(tmp_path, 0))
    assert state.snapshot_job(path) == job_a
    with pytest.raises(ValueError):
        state.restore(_engine(False), state.load(path), job="some-other-job")
    assert state.restore(_engine(False), state.load(path), job=job_a) == [0]
