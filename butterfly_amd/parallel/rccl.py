"""Native RCCL communicators over csrc/bindings/rccl_comm.cpp.

The world communicator is created from a 128-byte unique id that rank 0 draws and ships over
the control plane (one torch.distributed broadcast); every mesh axis then gets its own
communicator by `ncclCommSplit` of the world one (color = which group of the axis the rank is
in, key = its position), so a rank holds one RCCL communicator per axis without a second
bootstrap. The data-path collectives are single stream-ordered RCCL calls on torch's current
stream: no work objects, watchdog events or allocator stream records, so they capture into
the decode hipGraph like the kernels around them.

Enabled whenever the backend is RCCL (BFLY_NATIVE_RCCL, default on; parallel/comm.py routes all-reduce / all-gather /
reduce-scatter / all-to-all of groups larger than one rank here). RCCL refuses two ranks on
one device, so on a one-GPU box only nranks = 1 communicators can be exercised; the multi-rank
path needs a multi-GPU node.

Communicators are NON-BLOCKING: init and split poll RCCL's background setup
against BFLY_RCCL_INIT_TIMEOUT_S and raise TimeoutError (after aborting the half-built
communicator) when a peer never joins; `close()` is a bounded ncclCommFinalize + destroy that
falls back to an abort, so teardown never wedges. Graphs that captured a communicator's kernels
must be dropped before it is closed (LLMEngine.close orders this).
"""
from __future__ import annotations

import threading
from typing import Optional

import torch
import torch.distributed as dist

_OPS = {"sum": 0, "max": 1, "min": 2, "prod": 3}


def _lib():
    from .. import ops

    if not ops.load_library():
        raise RuntimeError(f"native RCCL needs butterfly_amd/_C.so: {ops._load_error}")
    return torch.ops.bfly


def _timeout(name: str, value: Optional[float]) -> float:
    from ..utils import flags

    return float(flags.get(name) if value is None else value)


def _call(fn, *args):
    """Native call; a deadline expiry (message 'RCCL-TIMEOUT') becomes TimeoutError."""
    try:
        return fn(*args)
    except RuntimeError as e:
        if "RCCL-TIMEOUT" in str(e):
            raise TimeoutError(str(e).split("\n")[0]) from None
        raise


def version() -> int:
    """RCCL version code of the library torch loaded (e.g. 22606 = 2.26.6)."""
    return int(_lib().rccl_version())


class RcclComm:
    """One RCCL communicator (a handle into the native table) and the global ranks it spans."""

    def __init__(self, handle: int, ranks: list):
        self.handle = int(handle)
        self.ranks = list(ranks)
        self._closed = False

    # -- construction ---------------------------------------------------------------------
    @classmethod
    def create(cls, uid: torch.Tensor, nranks: int, rank: int, ranks: Optional[list] = None,
               timeout: Optional[float] = None) -> "RcclComm":
        """Non-blocking ncclCommInitRankConfig on the current device with an id every member
        already holds, polled until ready; TimeoutError after `timeout` seconds
        (BFLY_RCCL_INIT_TIMEOUT_S) with the communicator aborted."""
        lib = _lib()
        lib.rccl_set_call_timeout(float(_timeout("BFLY_COMM_TIMEOUT_S", None)))
        h = _call(lib.rccl_init, uid.cpu().contiguous(), nranks, rank, _timeout("BFLY_RCCL_INIT_TIMEOUT_S", timeout))
        # the failure paths (health._default_failure, the preflight's hang exit) abort every
        # native communicator before the process exits
        from ..utils.health import register_abort_hook
        register_abort_hook(abort_all)
        return cls(h, ranks if ranks is not None else list(range(nranks)))

    @classmethod
    def world(cls, pg=None, timeout: Optional[float] = None) -> "RcclComm":
        """Collective over the torch.distributed world (or `pg`): rank 0's id is broadcast on
        the existing process group, then every rank joins."""
        lib = _lib()
        n, r = dist.get_world_size(pg), dist.get_rank(pg)
        uid = lib.rccl_unique_id() if r == 0 else torch.zeros(128, dtype=torch.uint8)
        dev = "cuda" if dist.get_backend(pg) == "nccl" else "cpu"
        t = uid.to(dev)
        dist.broadcast(t, dist.get_global_rank(pg, 0) if pg is not None else 0, group=pg)
        return cls.create(t.cpu(), n, r, timeout=timeout)

    def split(self, color: int, key: int, ranks: Optional[list] = None,
              timeout: Optional[float] = None) -> Optional["RcclComm"]:
        """ncclCommSplit (collective over this communicator): ranks passing the same color form
        one communicator ordered by key; color < 0 leaves the rank out (returns None). Bounded
        like `create`."""
        h = _call(_lib().rccl_split, self.handle, int(color), int(key), _timeout("BFLY_RCCL_INIT_TIMEOUT_S", timeout))
        return None if h < 0 else RcclComm(h, ranks if ranks is not None else [])

    # -- queries ----------------------------------------------------------------------------
    def info(self) -> tuple:
        """(rank in communicator, size, device ordinal)."""
        r, n, d = _lib().rccl_info(self.handle)
        return int(r), int(n), int(d)

    @property
    def size(self) -> int:
        return self.info()[1]

    def async_error(self) -> int:
        """0 when healthy, else the ncclResult_t of an asynchronous failure."""
        return int(_lib().rccl_async_error(self.handle))

    # -- collectives (stream-ordered on torch's current stream) -----------------------------
    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        _lib().rccl_all_reduce(self.handle, t, _OPS[op])
        return t

    def all_gather(self, t: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        _lib().rccl_all_gather(self.handle, t.contiguous(), out)
        return out

    def reduce_scatter(self, t: torch.Tensor, out: torch.Tensor, op: str = "sum") -> torch.Tensor:
        _lib().rccl_reduce_scatter(self.handle, t.contiguous(), out, _OPS[op])
        return out

    def all_to_all(self, t: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        _lib().rccl_all_to_all(self.handle, t.contiguous(), out)
        return out

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        _lib().rccl_broadcast(self.handle, t, int(root))
        return t

    def send(self, t: torch.Tensor, peer: int) -> None:
        _lib().rccl_send(self.handle, t.contiguous(), int(peer))

    def recv(self, t: torch.Tensor, peer: int) -> torch.Tensor:
        _lib().rccl_recv(self.handle, t, int(peer))
        return t

    @staticmethod
    def group_start() -> None:
        _lib().rccl_group_start()

    @staticmethod
    def group_end() -> None:
        _lib().rccl_group_end()

    def close(self, abort: bool = False, timeout: Optional[float] = None) -> str:
        """Tear down: 'clean' (finalize + destroy within `timeout`, BFLY_RCCL_CLOSE_TIMEOUT_S),
        'aborted' (requested, or the finalize outlived its deadline) or 'released' (already
        gone, e.g. taken down by abort_all). Never blocks past the deadline."""
        if self._closed:
            return "released"
        self._closed = True
        rc = int(_lib().rccl_release(self.handle, abort, _timeout("BFLY_RCCL_CLOSE_TIMEOUT_S", timeout)))
        return {1: "clean", 0: "aborted"}.get(rc, "released")


def live_handles() -> list:
    """Handles of every live native communicator in this process."""
    return [int(h) for h in _lib().rccl_live()]


def abort_all() -> int:
    """ncclCommAbort every live communicator (safe from any thread, also while another thread
    is blocked in a collective): the failure-path hook. Returns how many were aborted."""
    return int(_lib().rccl_abort_all())


# ncclResult_t values that mean "no failure": ncclSuccess, and ncclInProgress, which a
# NON-BLOCKING communicator reports while an operation (a collective's lazy connection setup,
# a split, a group end) is still being set up in RCCL's background thread
NCCL_SUCCESS, NCCL_IN_PROGRESS = 0, 7
HEALTHY_STATES = (NCCL_SUCCESS, NCCL_IN_PROGRESS)


# Host-mapped IPC health words (custom all-reduce, EP IPC) are acted on only for IPC paths
# that went LIVE (passed their self-test and route traffic): a flag-wait timeout inside a
# self-test, autotune or preflight check is a vote to fall back, not a failure of the job.
# Quiet and clear are scoped to the word under test ("car" or "ep"), so an EP self-test never
# hides or wipes a custom all-reduce timeout and vice versa; a word that was already set for a
# live path when a test on it began is kept (sticky) and still reported.
_health_lock = threading.Lock()
_health_live = {"car": 0, "ep": 0}     # live IPC objects per word
_health_quiet = {"car": 0, "ep": 0}    # self-tests / autotunes in progress, per word
_health_sticky = {"car": False, "ep": False}   # live timeouts seen at a test's start
_WORD_INDEX = {"car": 0, "ep": 1}      # bfly::kHealthCar / kHealthEp


def health_arm(word: str, on: bool = True) -> None:
    """An IPC object of `word` ("car" / "ep") went live (on) or was closed (off)."""
    with _health_lock:
        _health_live[word] = max(0, _health_live[word] + (1 if on else -1))
        if _health_live[word] == 0:
            _health_sticky[word] = False


class health_quiet:
    """Context of a collective self-test / autotune of the `word` IPC path ("car" or "ep"):
    the poller ignores that word while it runs, and a test that ends in a fallback
    (`failed(True)` or an exception) clears that word only."""

    def __init__(self, lib=None, word: str = "car"):
        if word not in _WORD_INDEX:
            raise ValueError(f"unknown health word {word!r}")
        self.lib, self.word, self.fallback = lib, word, False

    def failed(self, fallback: bool = True) -> None:
        self.fallback = fallback

    def __enter__(self):
        lib = self.lib or _lib()
        w = self.word
        with _health_lock:
            # a timeout of a live path of this word that happened before the test began is a
            # real failure: keep it reportable whatever the test does with the word
            if _health_live[w] and int(lib.health_words()[_WORD_INDEX[w]]):
                _health_sticky[w] = True
            _health_quiet[w] += 1
        return self

    def __exit__(self, et, ev, tb):
        try:
            if self.fallback or et is not None:
                (self.lib or _lib()).health_clear(_WORD_INDEX[self.word])
        finally:
            with _health_lock:
                _health_quiet[self.word] -= 1
        return False


def async_errors(lib=None) -> Optional[str]:
    """None when every live communicator is healthy and no live IPC path's flag wait timed out,
    else a description of the first failure (the ErrorPoller check). The IPC kernels' timeouts
    are read from host-mapped health words (plain loads: safe while the stream is stuck).
    `lib`: the op namespace to query (tests pass a stub)."""
    lib = _lib() if lib is None else lib
    with _health_lock:
        quiet = dict(_health_quiet)
        live = dict(_health_live)
        sticky = dict(_health_sticky)
    words = dict(zip(("car", "ep"), (int(v) for v in lib.health_words())))
    what = {"car": "custom all-reduce peer wait timed out (health word)",
            "ep": "EP IPC dispatch peer wait timed out (health word)"}
    for w in ("car", "ep"):
        if live[w] and (sticky[w] or (words[w] and quiet[w] == 0)):
            return what[w]
    for h in lib.rccl_live():
        try:
            err = int(lib.rccl_async_error(h))
        except RuntimeError:   # released between the listing and the query
            continue
        if err not in HEALTHY_STATES:
            return f"RCCL communicator {int(h)} async error {err}"
    return None


def start_error_poller(period: Optional[float] = None, on_failure=None):
    """Daemon thread polling `async_errors` every BFLY_RCCL_POLL_S seconds (0 = off): a peer
    that died or a network error is acted on within a second even while the main thread is
    stuck inside a collective; the failure handler aborts every communicator and exits 75."""
    from ..utils import flags
    from ..utils.health import ErrorPoller

    period = flags.get("BFLY_RCCL_POLL_S") if period is None else period
    return ErrorPoller(async_errors, period=period, on_failure=on_failure, name="bfly-rccl-poll").start()


def pp_edges(world: RcclComm, mesh, rank: int, force: bool = False) -> tuple:
    """Two-rank communicators for this rank's pipeline edges (collective: every rank calls it
    with the same mesh): (to the next stage, from the previous stage), each None at the ends.
    Edge s -> s+1 of a pipeline gets its own communicator (sender = rank 0, receiver = rank 1),
    split from `world` in two calls (even edges, then odd ones: a rank sits on at most one edge
    of each parity). Separate communicators per direction keep a stage's receive (captured in
    its decode graph) and its send (eager, on the send stream) on different RCCL objects.
    The connections are set up here with one tiny transfer per edge, so no later (captured)
    transfer has to run a connection handshake."""
    from ..utils import flags

    if mesh.pp <= 1 or not (force or flags.get("BFLY_PP_NATIVE_EDGES")):
        return None, None
    groups = mesh.all_groups("pp")
    g = next(i for i, grp in enumerate(groups) if rank in grp)
    s = groups[g].index(rank)
    pp = mesh.pp
    send = recv = None
    for parity in (0, 1):
        if s % 2 == parity and s + 1 < pp:
            c = world.split(g * pp + s, 0, [rank, groups[g][s + 1]])
            send = c
        elif s % 2 != parity and s >= 1:
            c = world.split(g * pp + s - 1, 1, [groups[g][s - 1], rank])
            recv = c
        else:
            world.split(-1, 0)
    dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.zeros(16, dtype=torch.float32, device=dev)
    # warm-up in stage order (first edges first) so no pair waits on another
    for parity in (0, 1):
        if send is not None and s % 2 == parity:
            send.send(t, 1)
        if recv is not None and (s - 1) % 2 == parity:
            recv.recv(t, 0)
    torch.cuda.synchronize(dev)
    return send, recv


def split_mesh(world: RcclComm, mesh, rank: int) -> dict:
    """One communicator per mesh axis with more than one rank, split from `world` (collective:
    every rank calls this with the same mesh). Returns {axis: RcclComm}."""
    out = {}
    for axis in ("tp", "pp", "dp"):
        groups = mesh.all_groups(axis)
        if len(groups[0]) <= 1:
            continue
        color = next(i for i, g in enumerate(groups) if rank in g)
        comm = world.split(color, groups[color].index(rank), groups[color])
        if comm is not None:
            out[axis] = comm
    return out
