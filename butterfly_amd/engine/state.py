"""Engine request-state snapshots: save / resume a serving replica.

Inference has no optimizer state: "resume" is reloading the weights (butterfly-ckpt, ckpt/format.py)
and replaying the request state. A snapshot holds, per data-parallel replica, every request the
engine knows: its prompt, the tokens it has generated so far (values already on the host), its
sampling parameters and its id. Restoring re-admits each unfinished request with prompt + output as
the sequence to prefill and max_tokens - len(output) still to generate, so its KV cache is rebuilt
by the normal (chunked) prefill path. Sampling noise is keyed on (seed or request id, index of the
generated token) (LLMEngine._sample_params), so a resumed request draws the same random numbers for
its next tokens as an uninterrupted run would. Token-identical continuation is guaranteed on the fp32
CPU path (tests/test_engine_state.py); on the GPU the rebuilt KV comes from the bf16 prefill kernels
instead of the decode kernels that wrote it originally, so a greedy near-tie can resolve differently
after a resume (the tokens stay valid samples of the model, not bit-identical replays).

Job identity: `job` (optional) is a fingerprint of what the job was asked to do (model, prompts,
sampling parameters; `job_fingerprint`). A restarted job resumes only a snapshot carrying its own
fingerprint, so a stale snapshot of an earlier, different job in the same directory is never
replayed (cli.py `generate`).

Format `butterfly-engine-state` v1 (JSON): {"format", "version", "model", "job", "dp_rank", "dp_size",
"next_id", "steps_done", "requests": [{"rid", "prompt", "output", "params", "finished",
"finish_reason"}]}. Tokens still in flight in the asynchronous pipeline (sampled, value not yet
on the host) are not part of it: they are recomputed after the resume.

Periodic snapshots: EngineConfig.snapshot_dir + snapshot_every (steps); one rank per replica (tp 0,
stage 0) writes `replica-<dp>.json` atomically (temporary file + rename), so a crash mid-write
leaves the previous snapshot intact.
"""
from __future__ import annotations

import dataclasses
import hashlib
import json
import os
from pathlib import Path
from typing import Optional

FORMAT = "butterfly-engine-state"
VERSION = 1


def snapshot(engine) -> dict:
    reqs = []
    for rid in sorted(engine.requests):
        r = engine.requests[rid]
        reqs.append({"rid": int(rid), "prompt": [int(t) for t in r.prompt],
                     "output": [int(t) for t in r.output],
                     "params": dataclasses.asdict(r.params),
                     "finished": bool(r.finished), "finish_reason": r.finish_reason})
    nxt = max(engine.requests, default=-1) + 1
    return {"format": FORMAT, "version": VERSION, "model": engine.cfg.name,
            "job": getattr(engine, "job_id", None),
            "dp_rank": int(engine.coord.dp), "dp_size": int(engine.mesh.dp),
            "next_id": int(nxt), "steps_done": int(engine.steps_done), "requests": reqs}


def job_fingerprint(model: str, prompts: list, params) -> str:
    """Stable id of a generation job: model name, prompts (token ids or text) and sampling
    parameters (a SamplingParams or a dict)."""
    p = dataclasses.asdict(params) if dataclasses.is_dataclass(params) else dict(params or {})
    blob = json.dumps({"model": model, "prompts": [list(x) if not isinstance(x, str) else x for x in prompts],
                       "params": p}, sort_keys=True)
    return hashlib.sha256(blob.encode()).hexdigest()[:32]


def restore(engine, state: dict, job: Optional[str] = None) -> list:
    """Re-admit a snapshot's requests into a fresh engine; returns the restored request ids.
    `job`: refuse a snapshot written by a different job (its fingerprint differs or is absent)."""
    from .engine import Request
    from .sampler import SamplingParams

    if state.get("format") != FORMAT or int(state.get("version", 0)) != VERSION:
        raise ValueError(f"not a {FORMAT} v{VERSION} snapshot")
    if state.get("model") != engine.cfg.name:
        raise ValueError(f"snapshot is of model {state.get('model')!r}, engine runs {engine.cfg.name!r}")
    if job is not None and state.get("job") != job:
        raise ValueError(f"snapshot belongs to job {state.get('job')!r}, not {job!r}")
    if engine.requests:
        raise RuntimeError("restore() needs an engine without requests")
    rids = []
    for r in state["requests"]:
        rid = int(r["rid"])
        params = SamplingParams(**r["params"])
        prompt, output = list(r["prompt"]), list(r["output"])
        done = bool(r["finished"]) or len(output) >= params.max_tokens
        if not output and not done:
            engine.add_request(prompt, params, rid=rid)        # never started: the normal path
        else:
            req = Request(rid, prompt, params, output=output, n_gen=len(output), finished=done,
                          finish_reason=r.get("finish_reason") or ("length" if done else None),
                          sched_done=done)
            engine.requests[rid] = req
            if not done:
                engine._admit_resumed(req)
        rids.append(rid)
    engine.reset_ids(int(state.get("next_id", max(rids, default=-1) + 1)))
    return rids


def save(engine, path) -> Path:
    """Write the snapshot atomically (temporary file in the same directory, then rename)."""
    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    tmp = p.with_name(p.name + f".tmp{os.getpid()}")
    with open(tmp, "w") as f:
        json.dump(snapshot(engine), f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, p)
    return p


def load(path) -> dict:
    with open(path) as f:
        return json.load(f)


def replica_path(directory, dp_rank: int) -> Path:
    return Path(directory) / f"replica-{dp_rank:03d}.json"


def snapshot_job(path) -> Optional[str]:
    """The job fingerprint stored in a snapshot file (None if absent or unreadable)."""
    try:
        return load(path).get("job")
    except (OSError, ValueError):
        return None


def maybe_periodic(engine) -> Optional[Path]:
    """Called after every engine step: write this replica's snapshot every `snapshot_every`
    steps (one writer per replica)."""
    e = engine.ecfg
    if not e.snapshot_dir or e.snapshot_every <= 0 or engine.steps_done % e.snapshot_every:
        return None
    if engine.coord.tp != 0 or engine.coord.pp != 0:
        return None
    return save(engine, replica_path(e.snapshot_dir, engine.coord.dp))
