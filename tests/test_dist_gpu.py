"""Sharded layouts on ONE MI355X: ranks share cuda:0 over gloo (RCCL refuses two ranks on one
device) and run their TP / PP / EP shards through the HIP kernels; generated tokens and
prefill logits must match a single-process run of the same partition-independent weights
(tools/gpu_dist_check.py). The EP case exercises the routed (sparse) MoE prefill path."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("layout,extra,env", [("tp2", [], {}), ("pp2", [], {}), ("dp2xep2", [], {}),
                                              ("pp2", ["-", "graphs"], {}),
                                              ("tp2", [], {"BFLY_SEQ_PARALLEL": "1",
                                                           "BFLY_SEQ_PARALLEL_MIN_TOKENS": "1"})])
def test_sharded_layout_on_one_gpu(layout, extra, env):
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--",
                        sys.executable, os.path.join(ROOT, "tools", "gpu_dist_check.py"), layout] + extra,
                       cwd=ROOT, env=dict(os.environ, **env), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") == 2, r.stdout[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("plan", ["tp2", "pp2"])
def test_bench_two_ranks_on_one_gpu(plan):
    """bench.py's multi-rank path on the GPU (ranks share cuda:0 over gloo): hipGraph decode,
    the IPC all-reduce (tp2) / asynchronous pipeline (pp2), rank 0's JSON line."""
    import json

    env = dict(os.environ, BFLY_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--",
                        sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "llama-small",
                        "--plan", plan, "--steps", "8", "--warmup", "2", "--batch-per-gpu", "8",
                        "--prompt-len", "64"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    lines = [l.split("] ", 1)[1] for l in r.stdout.splitlines() if l.startswith("[rank0] {")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["config"]["parallelism"] == plan and res["value"] > 0 and res["dtype"] == "bf16"


@pytest.mark.gpu
@pytest.mark.parametrize("n,attn,mode", [(2, "ring", "-"), (3, "ring", "-"), (2, "ulysses", "-"),
                                         (2, "ring", "engine"), (2, "ulysses", "engine")])
def test_context_parallel_prefill_on_one_gpu(n, attn, mode):
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", str(n), "--",
                        sys.executable, os.path.join(ROOT, "tools", "gpu_cp_check.py"), "-", attn, mode],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") == n, r.stdout[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_tp_production_dims_on_one_gpu(n):
    """the real TP decode path at production dimensions (Llama-3-70B layers at
    full width, 64 sequences per GPU: 128 / 256 rows, the mid-M shard plans, split-K slabs
    deferred into the IPC all-reduce with fused add + RMSNorm), ranks sharing cuda:0: logits
    against an fp32 reference model, graph replay bitwise against eager
    (tools/gpu_tp_fullsize.py)."""
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", str(n), "--",
                        sys.executable, os.path.join(ROOT, "tools", "gpu_tp_fullsize.py")],
                       cwd=ROOT, env=dict(os.environ, BFLY_IPC_SHARED_DEVICE="1"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-3000:]
    assert r.stdout.count("PASS") == n, r.stdout[-4000:]
