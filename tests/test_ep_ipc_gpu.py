"""Byte-minimal EP dispatch over peer IPC buffers on the GPU: 2, 4 and 8 ranks sharing one
MI355X (gloo carries only the hipIpc handle exchange and the reference data; the exchange runs
through csrc/kernels/ep_ipc.hip), bitwise against the all-to-all layout, eager and replayed
from a hipGraph (tools/ep_ipc_check.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8])
def test_ep_ipc_shared_gpu(n):
    env = dict(os.environ, BFLY_CAR_SHARED="1")
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", str(n), "--",
                        sys.executable, os.path.join(ROOT, "tools", "ep_ipc_check.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert r.stdout.count("PASS") == n, r.stdout[-4000:]
