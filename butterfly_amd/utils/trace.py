"""Tracing: roctx ranges for rocprofv3 and a chrome-trace timeline.

* `range(name)` — context manager that pushes/pops a roctx range (libroctx64, loaded with
  ctypes; a no-op when the library is absent or BFLY_ROCTX is off) and records a complete
  event in the process's chrome-trace buffer when BFLY_TRACE is set.
* `Tracer.dump(path)` writes {"traceEvents": [...]} loadable in chrome://tracing / Perfetto,
  one lane per rank (pid = rank).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time

from . import flags

_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if not flags.get("BFLY_ROCTX"):
        return None
    # rocprofv3 (rocprofiler-sdk) records the SDK's roctx; the legacy libroctx64 is for rocprof v1/v2
    for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "libroctx64.so",
                 "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


class Tracer:
    def __init__(self):
        self.events: list = []
        self.lock = threading.Lock()
        self.enabled = bool(flags.get("BFLY_TRACE"))
        self.pid = int(os.environ.get("RANK", "0"))
        self.t0 = time.perf_counter()

    def add(self, name: str, start: float, end: float, **args) -> None:
        if not self.enabled:
            return
        with self.lock:
            self.events.append({"name": name, "ph": "X", "pid": self.pid, "tid": threading.get_ident() % 100000,
                                "ts": (start - self.t0) * 1e6, "dur": (end - start) * 1e6, "args": args})

    def dump(self, path: str | None = None) -> str | None:
        path = path or flags.get("BFLY_TRACE")
        if not path or not self.events:
            return None
        if "{rank}" in path:
            path = path.format(rank=self.pid)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)
        return path


TRACER = Tracer()
if TRACER.enabled:
    import atexit

    atexit.register(TRACER.dump)     # BFLY_TRACE=path (may contain {rank}): written at exit


@contextlib.contextmanager
def range(name: str, **args):  # noqa: A001 - mirrors roctx naming
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t = time.perf_counter()
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
        TRACER.add(name, t, time.perf_counter(), **args)
