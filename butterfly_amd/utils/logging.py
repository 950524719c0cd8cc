"""Rank-tagged structured logging.

`get_logger(name)` returns a logger whose records carry the process's distributed rank; with
BFLY_LOG_JSON=1 records are emitted as one JSON object per line (for log collectors).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

from . import flags

_configured = False


def _rank() -> int:
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", "0"))


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.rank = _rank()
        return True


class _JsonFormatter(logging.Formatter):
    def format(self, record):
        d = {"ts": round(time.time(), 6), "level": record.levelname, "rank": getattr(record, "rank", 0),
             "logger": record.name, "msg": record.getMessage()}
        if record.exc_info:
            d["exc"] = self.formatException(record.exc_info)
        return json.dumps(d)


def get_logger(name: str = "butterfly") -> logging.Logger:
    global _configured
    if not _configured:
        root = logging.getLogger("butterfly")
        h = logging.StreamHandler(sys.stderr)
        h.addFilter(_RankFilter())
        if os.environ.get("BFLY_LOG_JSON", "0") == "1":
            h.setFormatter(_JsonFormatter())
        else:
            h.setFormatter(logging.Formatter("[%(asctime)s r%(rank)d %(levelname)s %(name)s] %(message)s", "%H:%M:%S"))
        root.addHandler(h)
        root.setLevel(str(flags.get("BFLY_LOG_LEVEL")).upper())
        root.propagate = False
        _configured = True
    return logging.getLogger(name if name.startswith("butterfly") else f"butterfly.{name}")
