"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer: the
paged-KV block manager and the scheduler (legacy and mixed/chunked modes) built without
Python into a standalone self-test (csrc/runtime/tests/selftest.cpp) and driven through
randomized request streams with preemption. Host code only: GPU sanitizers are not used."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_runtime_selftest_asan_ubsan(tmp_path):
    exe = tmp_path / "rt_selftest"
    src = os.path.join(ROOT, "csrc", "runtime", "tests", "selftest.cpp")
    b = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", src, "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "runtime selftest: PASS" in r.stdout
