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
@pytest.mark.parametrize("layout,extra", [("tp2", []), ("pp2", []), ("dp2xep2", []),
                                          ("pp2", ["-", "graphs"])])
def test_sharded_layout_on_one_gpu(layout, extra):
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--",
                        sys.executable, os.path.join(ROOT, "tools", "gpu_dist_check.py"), layout] + extra,
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") == 2, r.stdout[-4000:]
