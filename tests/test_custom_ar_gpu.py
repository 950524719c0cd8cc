"""One-shot IPC all-reduce on the GPU: 2 and 4 ranks sharing one MI355X (gloo only carries
the hipIpc handle exchange; the reduction runs through csrc/kernels/allreduce.hip)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_custom_allreduce_shared_gpu(n):
    env = dict(os.environ, BFLY_CAR_SHARED="1")
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
