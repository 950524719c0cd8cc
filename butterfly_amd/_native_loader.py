"""Import the host C++ runtime (butterfly_amd._native), building it in-tree if missing."""
from __future__ import annotations

import importlib

_mod = None


def native():
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("butterfly_amd._native")
        except ImportError:
            from . import _build

            _build.build_native(verbose=False)
            _mod = importlib.import_module("butterfly_amd._native")
    return _mod
