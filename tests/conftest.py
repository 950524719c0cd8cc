import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the multi-rank GPU tests run their ranks on ONE device: let the IPC all-reduce / EP exchange
# run there (production refuses shared-GPU IPC groups: parallel/custom_allreduce.py)
os.environ.setdefault("BFLY_IPC_SHARED_DEVICE", "1")
# every multi-rank engine in the suites runs its decode steps with the rank program enforced
# on the in-stage collectives (comm.Communicator.expect): a divergence fails the test by name
os.environ.setdefault("BFLY_PROGRAM_CHECK", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
