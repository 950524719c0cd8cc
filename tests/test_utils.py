"""Observability / health utilities."""
import json
import time

import torch.distributed as dist

from butterfly_amd.utils import flags
from butterfly_amd.utils.health import FaultInjector, HealthMonitor, StepWatchdog
from butterfly_amd.utils.metrics import Metrics, percentile

from .dist_utils import free_port


def test_metrics_export():
    m = Metrics()
    for v in (1.0, 2.0, 3.0, 4.0):
        m.observe("lat", v)
    m.inc("tokens", 10)
    s = m.summary()
    assert s["histograms"]["lat"]["p50"] == 2.5 and s["counters"]["tokens"] == 10
    assert 'bfly_lat{quantile="0.50"} 2.5' in m.to_prometheus()
    json.loads(m.to_json())
    assert percentile([], 50) != percentile([], 50)  # nan


def test_flags_registry(monkeypatch):
    monkeypatch.setenv("BFLY_DISABLE_GRAPHS", "1")
    assert flags.get("BFLY_DISABLE_GRAPHS") is True
    assert "BFLY_FAULT" in flags.dump()


def test_fault_injector_parse():
    f = FaultInjector("1:3:nan")
    assert f.maybe_inject(0, 3) is None and f.maybe_inject(1, 2) is None
    assert f.maybe_inject(1, 3) == "nan"


def test_watchdog_fires():
    hits = []
    w = StepWatchdog(0.05, on_failure=hits.append)
    w.arm("step 7")
    time.sleep(0.2)
    assert hits and "step 7" in hits[0]
    w.arm()
    w.disarm()


def test_health_monitor_detects_dead_rank():
    store = dist.TCPStore("127.0.0.1", free_port(), 2, True, wait_for_workers=False)
    failures = []
    mon = HealthMonitor(store, rank=0, world=2, period=0.05, timeout=0.2, on_failure=failures.append)
    store.set("bfly/hb/1", repr(time.time() - 10))     # rank 1 went silent 10 s ago
    mon.start()
    time.sleep(0.5)
    mon.stop()
    assert failures and "rank 1" in failures[0]


def test_error_poller_fires_once_on_first_error():
    import time

    from butterfly_amd.utils.health import ErrorPoller

    answers = [None, None, "comm 3 async error 6", "again"]
    hits = []
    p = ErrorPoller(lambda: answers.pop(0) if answers else None, period=0.02, on_failure=hits.append).start()
    deadline = time.time() + 5
    while not hits and time.time() < deadline:
        time.sleep(0.01)
    p.stop()
    assert hits == ["comm 3 async error 6"] and p.failed == hits[0]
    assert answers == ["again"]          # the thread stops after the first failure


def test_abort_hooks_run_bounded(monkeypatch):
    import threading
    import time

    from butterfly_amd.utils import health

    monkeypatch.setattr(health, "_abort_hooks", [])
    ran = []
    block = threading.Event()
    health.register_abort_hook(lambda: ran.append("a"))
    health.register_abort_hook(lambda: block.wait(30))      # an abort that hangs
    t0 = time.time()
    health.run_abort_hooks(timeout=0.3)
    assert ran == ["a"] and time.time() - t0 < 5
    block.set()
    f = health._abort_hooks[0]
    health.register_abort_hook(f)                            # idempotent
    assert len(health._abort_hooks) == 2


def test_default_failure_runs_abort_hooks_before_exit(monkeypatch):
    from butterfly_amd.utils import health

    order = []
    monkeypatch.setattr(health, "_abort_hooks", [lambda: order.append("abort")])
    monkeypatch.setattr(health.os, "_exit", lambda code: order.append(("exit", code)))
    health._default_failure("test")
    assert order == ["abort", ("exit", 75)]


def test_custom_all_reduce_routing_choice():
    """parallel/custom_allreduce.choose_routing: IPC up to the largest size of the winning
    prefix, two-shot from the smallest size where it wins through the routed range."""
    from butterfly_amd.parallel.custom_allreduce import choose_routing

    inf = float("inf")
    sizes = [32 << 10, 128 << 10, 512 << 10, 2 << 20, 8 << 20]
    # IPC wins everywhere; two-shot wins from 512 KiB on
    t = [[5, 7, 20], [8, 9, 24], [20, 15, 35], [60, 40, 70], [200, 120, 150]]
    assert choose_routing(sizes, t) == (8 << 20, 512 << 10)
    # RCCL wins from 2 MiB on: route only up to 512 KiB; two-shot never (groups of 2)
    t = [[5, inf, 20], [8, inf, 24], [20, inf, 35], [80, inf, 70], [300, inf, 150]]
    assert choose_routing(sizes, t) == (512 << 10, 0)
    # RCCL faster at the smallest size: never route to IPC
    assert choose_routing(sizes, [[30, inf, 20]] + t[1:]) == (0, 0)
