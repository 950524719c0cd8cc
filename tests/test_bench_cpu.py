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
