"""IPC all-reduce (one-shot and two-shot) on the GPU: 2, 4 and 8 ranks sharing one MI355X (gloo only carries
the hipIpc handle exchange; the reduction runs through csrc/kernels/allreduce.hip)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8])
def test_custom_allreduce_shared_gpu(n):
    # 8 ranks on one GPU: the fused one-shot kernel cannot keep 8 x 128 workgroups resident
    # (see tools/car_check.py); everything else, two-shot fused included, is checked
    env = dict(os.environ, BFLY_CAR_SHARED="1", BFLY_CAR_PLAIN_ONE_SHOT="1" if n == 8 else "0")
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", str(n), "--",
                        sys.executable, os.path.join(ROOT, "tools", "car_check.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") == n, r.stdout[-4000:]


@pytest.mark.gpu
def test_tp2_model_with_custom_allreduce():
    env = dict(os.environ, BFLY_CUSTOM_AR="1")
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--",
                        sys.executable, os.path.join(ROOT, "tools", "gpu_dist_check.py"), "tp2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") == 2, r.stdout[-4000:]
