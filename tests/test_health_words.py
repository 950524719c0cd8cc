"""Error-poller semantics on CPU (stubbed native library): ncclInProgress is healthy, IPC health
words count only for IPC paths that went live, and a failed self-test's timeout never reaches
the poller (rccl.py async_errors, custom_allreduce health words)."""
import time

from butterfly_amd.parallel import rccl
from butterfly_amd.parallel.comm import butterfly_ranges
from butterfly_amd.utils.health import ErrorPoller


class StubLib:
    def __init__(self, states=(), words=(0, 0)):
        self.states = dict(states)
        self.words = list(words)
        self.cleared = 0

    def health_words(self):
        return list(self.words)

    def health_clear(self, word=-1):
        self.words = [0 if word in (-1, i) else v for i, v in enumerate(self.words)]
        self.cleared += 1

    def rccl_live(self):
        return list(self.states)

    def rccl_async_error(self, h):
        return self.states[h]


def test_in_progress_is_healthy():
    assert rccl.async_errors(StubLib({1: 0, 2: rccl.NCCL_IN_PROGRESS})) is None
    err = rccl.async_errors(StubLib({1: rccl.NCCL_IN_PROGRESS, 2: 3}))
    assert err is not None and "async error 3" in err


def test_poller_survives_in_progress_communicator():
    lib = StubLib({5: rccl.NCCL_IN_PROGRESS})
    fired = []
    p = ErrorPoller(lambda: rccl.async_errors(lib), period=0.01, on_failure=fired.append).start()
    time.sleep(0.1)
    p.stop()
    assert fired == [] and p.failed is None


def test_health_words_only_for_live_ipc_paths():
    lib = StubLib(words=(1, 0))
    assert rccl.async_errors(lib) is None          # nothing armed: a self-test's leftover
    rccl.health_arm("car")
    try:
        assert "all-reduce" in rccl.async_errors(lib)
        with rccl.health_quiet(lib, word="car"):   # a test of the same word: its vote
            pass
    finally:
        rccl.health_arm("car", False)
    lib.words = [0, 1]
    rccl.health_arm("ep")
    try:
        assert "EP IPC" in rccl.async_errors(lib)
    finally:
        rccl.health_arm("ep", False)


def test_failed_self_test_clears_words_and_poller_survives():
    lib = StubLib()
    fired = []
    rccl.health_arm("car")                         # a live group elsewhere in the process
    p = ErrorPoller(lambda: rccl.async_errors(lib), period=0.005, on_failure=fired.append).start()
    try:
        with rccl.health_quiet(lib) as q:
            lib.words = [1, 0]                     # the self-test's flag wait timed out
            time.sleep(0.05)                       # several poller periods inside the test
            q.failed(True)                         # group voted to fall back to RCCL
        time.sleep(0.05)
    finally:
        p.stop()
        rccl.health_arm("car", False)
    assert lib.cleared == 1 and lib.words == [0, 0]
    assert fired == []


def test_quiet_clears_on_exception():
    lib = StubLib(words=(1, 1))
    try:
        with rccl.health_quiet(lib):
            raise RuntimeError("self-test raised")
    except RuntimeError:
        pass
    assert lib.cleared == 1


def test_butterfly_ranges_keyed_by_group(monkeypatch):
    monkeypatch.setenv("BFLY_AR_BUTTERFLY", "4@1024:65536")
    r = butterfly_ranges()
    assert r == {4: (1024, 65536)}
    monkeypatch.setenv("BFLY_AR_BUTTERFLY", "0:4096")
    r = butterfly_ranges()
    assert r[2] == (0, 4096) and r[8] == (0, 4096)
    monkeypatch.setenv("BFLY_AR_BUTTERFLY", "")
    assert butterfly_ranges() == {}


def test_quiet_is_scoped_to_its_word():
    """an EP self-test neither hides nor wipes a live custom all-reduce timeout."""
    lib = StubLib()
    rccl.health_arm("car")
    try:
        with rccl.health_quiet(lib, word="ep") as q:
            lib.words = [1, 1]                     # a real car timeout + the EP test's own
            assert "all-reduce" in rccl.async_errors(lib)
            q.failed(True)
        assert lib.words == [1, 0]                 # only the EP word was cleared
        assert "all-reduce" in rccl.async_errors(lib)
    finally:
        rccl.health_arm("car", False)


def test_timeout_before_a_test_stays_reported():
    """A live path's timeout already set when a test of the same word starts is sticky."""
    lib = StubLib(words=(1, 0))
    rccl.health_arm("car")
    try:
        with rccl.health_quiet(lib, word="car") as q:
            q.failed(True)                         # the test clears the word...
        assert lib.words == [0, 0]
        assert "all-reduce" in rccl.async_errors(lib)   # ...the earlier failure is kept
    finally:
        rccl.health_arm("car", False)
    assert rccl.async_errors(lib) is None          # path closed: nothing live to report
