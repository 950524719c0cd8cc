"""Metrics registry ("Observability and metrics", /root/reference/CLAUDE.md:42).

Counters, gauges and histograms (exact sample lists; these are per-process serving metrics,
not a TSDB) with JSON and Prometheus text export. The engine records every step (kind, batch,
seconds); the API/server layer records TTFT / TPOT / end-to-end latency per request.
"""
from __future__ import annotations

import json
import threading
import time
from collections import defaultdict


def percentile(xs, q: float) -> float:
    if not xs:
        return float("nan")
    s = sorted(xs)
    k = (len(s) - 1) * q / 100.0
    lo = int(k)
    hi = min(lo + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


class Metrics:
    def __init__(self, max_samples: int = 100_000):
        self._lock = threading.Lock()
        self.counters: dict[str, float] = defaultdict(float)
        self.gauges: dict[str, float] = {}
        self.hist: dict[str, list] = defaultdict(list)
        self.max_samples = max_samples
        self.t_start = time.time()

    def inc(self, name: str, v: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += v

    def set(self, name: str, v: float) -> None:
        with self._lock:
            self.gauges[name] = v

    def observe(self, name: str, v: float) -> None:
        with self._lock:
            h = self.hist[name]
            h.append(v)
            if len(h) > self.max_samples:
                del h[: len(h) - self.max_samples]

    def observe_step(self, kind: str, batch: int, seconds: float) -> None:
        self.inc(f"steps_{kind}")
        self.inc(f"tokens_{kind}", batch)
        self.observe(f"step_seconds_{kind}", seconds)

    def summary(self) -> dict:
        with self._lock:
            out = {"counters": dict(self.counters), "gauges": dict(self.gauges), "histograms": {}}
            for k, v in self.hist.items():
                out["histograms"][k] = {"count": len(v), "p50": percentile(v, 50), "p90": percentile(v, 90),
                                        "p99": percentile(v, 99), "mean": sum(v) / len(v) if v else float("nan")}
            return out

    def to_json(self) -> str:
        return json.dumps(self.summary(), indent=2, sort_keys=True)

    def to_prometheus(self, prefix: str = "bfly_") -> str:
        s = self.summary()
        lines = []
        for k, v in sorted(s["counters"].items()):
            lines += [f"# TYPE {prefix}{k} counter", f"{prefix}{k} {v}"]
        for k, v in sorted(s["gauges"].items()):
            lines += [f"# TYPE {prefix}{k} gauge", f"{prefix}{k} {v}"]
        for k, h in sorted(s["histograms"].items()):
            lines.append(f"# TYPE {prefix}{k} summary")
            for q in ("p50", "p90", "p99"):
                lines.append(f'{prefix}{k}{{quantile="0.{q[1:]}"}} {h[q]}')
            lines.append(f"{prefix}{k}_count {h['count']}")
        return "\n".join(lines) + "\n"
