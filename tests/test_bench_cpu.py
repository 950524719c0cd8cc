"""bench.py's multi-rank contract on CPU/gloo (2 ranks): the driver launches it once per rank
and parses rank 0's single JSON line. Exercises the PP (asynchronous pipeline), TP and DP
paths of the benchmark loop — token counting, the cross-rank max of the elapsed time, the
reported parallelism — on the tiny Llama config."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("plan", ["pp2", "tp2", "dp2"])
def test_bench_two_ranks(plan):
    env = dict(os.environ, OMP_NUM_THREADS="2", BFLY_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--",
                        sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "llama-tiny",
                        "--plan", plan, "--steps", "6", "--warmup", "2", "--batch-per-gpu", "4",
                        "--prompt-len", "16"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    lines = [l.split("] ", 1)[1] for l in r.stdout.splitlines() if l.startswith("[rank0] {")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == plan
    assert res["value"] > 0 and res["ms_per_step"] > 0 and res["scaling"] == "weak"
    assert res["config"]["global_batch"] == 8
    if plan == "pp2":
        assert res["config"]["pp_async_groups"] == 2


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` from a bare shell (no WORLD_SIZE): bench.py launches its own
    ranks, relays exactly one JSON line and reports the world the collectives saw."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2", BFLY_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "llama-tiny",
                        "--plan", "tp2", "--steps", "4", "--warmup", "1", "--batch-per-gpu", "4",
                        "--prompt-len", "16"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_size"] == 2 and res["rccl_ranks_seen"] == 2
    assert res["backend"] == "gloo" and res["plan"]["tp"] == 2


def test_bench_self_launch_failure_propagates():
    """A failing rank makes the self-launched job exit non-zero (no JSON line)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2", BFLY_DIST_BACKEND="gloo", BFLY_FAULT="1:0:exit", BFLY_COMM_TIMEOUT_S="60")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "llama-tiny",
                        "--plan", "tp2", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "2",
                        "--prompt-len", "8"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_baseline_config_1():
    """BASELINE config 1 (GPT-2 small, 2-stage layer split on CPU/gloo) is one flag."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--baseline-config", "1", "--steps", "2",
                        "--warmup", "1", "--batch-per-gpu", "2", "--prompt-len", "8"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert res["config"]["model"] == "GPT-2-small" and res["plan"]["pp"] == 2 and res["dtype"] == "fp32"


def test_peer_exit_fails_survivor_within_timeout():
    """Ranks started without our launcher (as torchrun would): rank 1 exits at step 1; rank 0
    must terminate non-zero by itself (collective error or BFLY_COMM_TIMEOUT_S), not hang."""
    import socket
    import time

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, OMP_NUM_THREADS="2", BFLY_DIST_BACKEND="gloo", BFLY_FAULT="1:3:exit",
                   BFLY_COMM_TIMEOUT_S="30", RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model",
                                       "llama-tiny", "--plan", "tp2", "--steps", "4", "--warmup", "1",
                                       "--batch-per-gpu", "2", "--prompt-len", "8"], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    try:
        rc0 = procs[0].wait(timeout=120)
        rc1 = procs[1].wait(timeout=30)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rc1 == 13 and rc0 != 0
    assert time.time() - t0 < 120


def test_launch_honours_plan_placement(tmp_path):
    """`launch --plan` binds rank r to GPU placement[r] through LOCAL_RANK (the device index
    init_distributed and the RCCL communicator use); the launcher never touches the GPU."""
    import subprocess
    import sys

    from butterfly_amd.config import ModelConfig
    from butterfly_amd.partition import partition

    plan = partition(ModelConfig.from_preset("llama-tiny"), 2, {"tp": 2})
    plan.placement = [1, 0]
    pf = tmp_path / "plan.json"
    pf.write_text(plan.to_json())
    prog = "import os; print('R', os.environ['RANK'], 'L', os.environ['LOCAL_RANK'])"
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--plan", str(pf), "--",
                        sys.executable, "-c", prog], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = sorted(l.split("] ", 1)[1] for l in r.stdout.splitlines() if "] R " in l)
    assert got == ["R 0 L 1", "R 1 L 0"], r.stdout
