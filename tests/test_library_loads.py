"""The built kernel library must load on the CPU build box too (CPU tests that skip when it
is missing would otherwise hide a library that was built but cannot be loaded, e.g. a kernel
template whose host launch stub was never emitted: an undefined symbol at dlopen)."""
import os

import pytest

from butterfly_amd import ops

SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "butterfly_amd", "_C.so")


@pytest.mark.skipif(not os.path.exists(SO), reason="butterfly_amd/_C.so not built")
def test_built_library_loads():
    assert ops.load_library(), ops._load_error
