"""Multi-GPU preflight (parallel/preflight.py) on CPU / gloo ranks: every outcome is voted, so
an injected failure on ONE rank switches the feature off on EVERY rank; a failed mandatory
check ends the job on every rank; a hung check ends the job with exit code 75 within its
deadline, naming the rank and the check (the launcher takes the rest down)."""
import os
import subprocess
import sys
import time

import pytest

from tests.dist_utils import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _preflight(rank, world, inject):
    os.environ["BFLY_PREFLIGHT_INJECT"] = inject
    os.environ["BFLY_PREFLIGHT_TIMEOUT_S"] = "60"
    from butterfly_amd.parallel.preflight import PreflightError, run_preflight

    try:
        rep = run_preflight(apply=False)
    except PreflightError as e:
        return {"error": str(e)}
    return rep.summary()


def test_clean_run_passes_mandatory_checks_and_skips_gpu_ones():
    for s in run_world(_preflight, 2, ""):
        c = s["checks"]
        assert c["world_collectives"] is True and c["p2p_all_pairs"] is True and c["subgroups"] is None
        for k in ("comm_stream_recv", "graph_collective", "native_rccl", "pp_edge_graph", "native_a2a_graph",
                  "custom_ar", "ep_ipc"):
            assert c[k] is None, (k, c)
        assert s["disabled"] == [] and s["env"] == {} and s["allow_tp"] is True


def test_four_ranks_cover_every_pair_and_subgroups():
    for s in run_world(_preflight, 4, ""):
        assert s["checks"]["p2p_all_pairs"] is True and s["checks"]["subgroups"] is True


@pytest.mark.parametrize("inject,feature,env", [
    ("custom_ar:fail:1", "custom_ar", {"BFLY_CUSTOM_AR": "0"}),
    ("custom_ar:raise:0", "custom_ar", {"BFLY_CUSTOM_AR": "0"}),
    ("comm_stream_recv:fail:0", "pp_prepost", {"BFLY_PP_PREPOST": "0"}),
    ("native_rccl:raise:1", "native_rccl", {"BFLY_NATIVE_RCCL": "0"}),
    ("pp_edge_graph:fail:1", "pp_native_edges", {"BFLY_PP_NATIVE_EDGES": "0"}),
    ("pp_edge_graph:raise:0", "pp_native_edges", {"BFLY_PP_NATIVE_EDGES": "0"}),
    ("native_a2a_graph:raise:0", "native_a2a", {"BFLY_NATIVE_A2A": "0"}),
    ("ep_ipc:fail:1", "ep_ipc", {"BFLY_EP_IPC": "0"}),
    ("ep_ipc:raise:0", "ep_ipc", {"BFLY_EP_IPC": "0"}),
])
def test_one_rank_failure_disables_feature_everywhere(inject, feature, env):
    res = run_world(_preflight, 2, inject)
    for s in res:
        assert feature in s["disabled"], s
        for k, v in env.items():
            assert s["env"][k] == v
    assert res[0]["env"] == res[1]["env"]


def test_each_new_check_fails_alone():
    """A pipeline-edge failure turns off only the native edges: native RCCL itself, the
    all-to-all and the IPC paths stay as they were."""
    for s in run_world(_preflight, 4, "pp_edge_graph:fail:2"):
        assert s["disabled"] == ["pp_native_edges"] and s["env"] == {"BFLY_PP_NATIVE_EDGES": "0"}, s
        assert s["checks"]["native_a2a_graph"] is None and s["checks"]["ep_ipc"] is None


def _ensure_twice(rank, world):
    from butterfly_amd.parallel import preflight

    assert preflight.last_report() is None
    a = preflight.ensure_preflight()
    b = preflight.ensure_preflight()          # already ran in this process: no second run
    return a is b and a is not None and preflight.last_report() is a


def test_ensure_preflight_runs_once_per_process():
    assert run_world(_ensure_twice, 2) == [True, True]


def test_capture_failure_without_native_rccl_disables_graphs():
    for s in run_world(_preflight, 2, "graph_collective:raise:0,native_rccl:fail:1"):
        assert s["checks"]["graph_collective"] is False and s["checks"]["native_rccl"] is False
        assert "hipgraph_decode" in s["disabled"] and s["env"]["BFLY_DISABLE_GRAPHS"] == "1"


@pytest.mark.parametrize("check", ["world_collectives", "p2p_all_pairs"])
def test_mandatory_failure_ends_job_on_every_rank(check):
    for s in run_world(_preflight, 2, f"{check}:fail:1"):
        assert "error" in s and check in s["error"]


@pytest.mark.parametrize("check", ["custom_ar", "pp_edge_graph", "ep_ipc"])
def test_hung_check_exits_75_naming_rank_and_check(check):
    """Rank 1 never returns from a check: both ranks' watchdogs fire within the deadline
    (rank 0 is blocked in the check's vote), the job exits 75 and stderr names rank 1 and
    the check."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2", BFLY_DIST_BACKEND="gloo", BFLY_PREFLIGHT_INJECT=f"{check}:hang:1",
               BFLY_PREFLIGHT_TIMEOUT_S="5", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-m", "butterfly_amd", "launch", "-n", "2", "--",
                        sys.executable, "-m", "butterfly_amd.parallel.preflight"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    took = time.monotonic() - t0
    log = r.stdout + r.stderr
    assert r.returncode == 75, log[-3000:]
    assert f"PREFLIGHT-HANG rank=1 check={check}" in log, log[-3000:]
    assert took < 120, took


def test_watchdog_runs_abort_hooks_before_exit(monkeypatch):
    """A hung check most often sits in a collective: the watchdog aborts the native RCCL
    communicators (the registered abort hooks) before it exits."""
    from butterfly_amd.parallel.preflight import HANG_EXIT_CODE, _Watchdog
    from butterfly_amd.utils import health

    order = []
    monkeypatch.setattr(health, "_abort_hooks", [lambda: order.append("abort")])
    wd = _Watchdog(rank=3, exit_fn=lambda code: order.append(("exit", code)))
    wd.arm("native_rccl", 0.05)
    deadline = time.monotonic() + 10
    while len(order) < 2 and time.monotonic() < deadline:
        time.sleep(0.02)
    wd.close()
    assert order == ["abort", ("exit", HANG_EXIT_CODE)]
