"""In-process loopback communication backend (SURVEY.md §2.7-B B5, §5.2 "comm-ordering checker").

`FakeWorld(mesh)` hands out one `FakeComm` per rank; the ranks run as threads of one process
and meet in shared memory instead of RCCL/gloo. It implements the same interface as
`parallel.comm.Communicator` (so engines, models and samplers run unchanged) and CHECKS the
communication program while doing so:
  * every collective of a group must be the same op with the same shape/dtype on all ranks
    at the same per-group sequence number — otherwise `CommOrderError` names both calls;
  * every recv must match the next send queued on that (src, dst) pair in shape and dtype;
  * a rank that waits longer than `timeout_s` for its peers raises (a deadlock in the
    program, e.g. mismatched send/recv order between pipeline stages).
`FakeWorld.run(fn)` runs fn(rank, comm) on every rank in threads and returns the results,
re-raising the first failure.
"""
from __future__ import annotations

import threading
from collections import defaultdict, deque
from typing import Callable

import torch

from .comm import Communicator, GroupHandle
from .mesh import Mesh


class CommOrderError(RuntimeError):
    pass


class _Slot:
    def __init__(self, n: int):
        self.contrib: dict = {}
        self.result = None
        self.reads = 0
        self.n = n


class FakeWorld:
    def __init__(self, mesh: Mesh, timeout_s: float = 120.0):
        self.mesh = mesh
        self.n = mesh.world_size
        self.timeout_s = timeout_s
        self.cv = threading.Condition()
        self.slots: dict = {}
        self.seq = defaultdict(int)                 # (group ranks, rank) -> next sequence no.
        self.queues = defaultdict(deque)            # (src, dst) -> deque of tensors
        self.log: list = []                         # (rank, op, group, shape, bytes) in issue order
        self.comms = [FakeComm(self, r) for r in range(self.n)]

    # -- rendezvous ---------------------------------------------------------------------------
    def collective(self, rank: int, ranks: tuple, op: str, t: torch.Tensor, reduce: Callable):
        key_seq = (ranks, rank)
        with self.cv:
            seq = self.seq[key_seq]
            self.seq[key_seq] += 1
            key = (ranks, seq)
            slot = self.slots.get(key)
            if slot is None:
                slot = self.slots[key] = _Slot(len(ranks))
            sig = (op, tuple(t.shape), t.dtype)
            for other, (osig, _) in slot.contrib.items():
                if osig != sig:
                    raise CommOrderError(f"collective #{seq} of group {ranks}: rank {rank} issued {sig}, "
                                         f"rank {other} issued {osig}")
            slot.contrib[rank] = (sig, t.detach().clone())
            self.log.append((rank, op, ranks, tuple(t.shape), t.numel() * t.element_size()))
            if len(slot.contrib) == slot.n:
                slot.result = reduce([slot.contrib[r][1] for r in ranks])
                self.cv.notify_all()
            elif not self.cv.wait_for(lambda: slot.result is not None, self.timeout_s):
                missing = sorted(set(ranks) - set(slot.contrib))
                raise CommOrderError(f"rank {rank}: {op} #{seq} of group {ranks} timed out waiting for {missing}")
            out = slot.result
            slot.reads += 1
            if slot.reads == slot.n:
                del self.slots[key]
            return out

    def send(self, src: int, dst: int, t: torch.Tensor) -> None:
        with self.cv:
            self.queues[(src, dst)].append(t.detach().clone())
            self.log.append((src, "send", (src, dst), tuple(t.shape), t.numel() * t.element_size()))
            self.cv.notify_all()

    def recv(self, src: int, dst: int, like: torch.Tensor) -> torch.Tensor:
        q = self.queues[(src, dst)]
        with self.cv:
            if not self.cv.wait_for(lambda: len(q) > 0, self.timeout_s):
                raise CommOrderError(f"rank {dst}: recv from {src} timed out (no matching send)")
            t = q.popleft()
        if t.shape != like.shape or t.dtype != like.dtype:
            raise CommOrderError(f"rank {dst}: recv {tuple(like.shape)}/{like.dtype} from {src} matched a send "
                                 f"of {tuple(t.shape)}/{t.dtype}")
        return t

    def run(self, fn: Callable, *args) -> list:
        results: list = [None] * self.n
        errors: list = []

        def body(r):
            from .. import ops

            ops.arena_scope(("fake-rank", r))    # per-rank kernel workspaces (ops._Arena)
            try:
                results[r] = fn(r, self.comms[r], *args)
            except BaseException as e:  # noqa: BLE001 — surfaced below
                errors.append((r, e))
                with self.cv:
                    self.cv.notify_all()

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.n)]
        for th in threads:
            th.start()
        for th in threads:
            th.join(self.timeout_s * 4)
        if errors:
            r, e = errors[0]
            raise RuntimeError(f"rank {r} failed: {e!r}") from e
        return results


class _Done:
    def wait(self):
        return None

    def is_completed(self):
        return True


class FakeComm(Communicator):
    def __init__(self, world: FakeWorld, rank: int):
        mesh = world.mesh
        groups = {}
        for axis in ("tp", "pp", "dp"):
            for ranks in mesh.all_groups(axis):
                if rank in ranks:
                    groups[axis] = GroupHandle(list(ranks), "fake" if len(ranks) > 1 else None, ranks.index(rank))
        groups["ep"] = groups["dp"] if mesh.ep > 1 else GroupHandle([rank], None, 0)
        groups["world"] = GroupHandle(list(range(mesh.world_size)), "fake", rank)
        super().__init__(mesh, rank, groups)
        self.world = world

    def _coll(self, group: str, op: str, t: torch.Tensor, reduce: Callable) -> torch.Tensor:
        g = self.groups[group]
        return self.world.collective(self.rank, tuple(g.ranks), op, t, reduce)

    def all_reduce_(self, t, group="tp"):
        if self.groups[group].size == 1:
            return t
        self._conform("all_reduce", group, t.numel() * t.element_size())
        self.stats["calls"] += 1
        self.stats["all_reduce_bytes"] += t.numel() * t.element_size()
        t.copy_(self._coll(group, "all_reduce", t, lambda xs: torch.stack([x.float() for x in xs]).sum(0).to(xs[0].dtype)))
        return t

    def all_reduce_max_(self, t, group="tp"):
        if self.groups[group].size == 1:
            return t
        self.stats["calls"] += 1
        t.copy_(self._coll(group, "all_reduce_max", t, lambda xs: torch.stack(xs).max(0).values))
        return t

    def all_reduce_rms_norm_(self, t, w, eps, residual, group="tp"):
        from .. import ops

        self.all_reduce_(t, group)
        return ops.rms_norm(t, w, eps, residual=residual)

    def all_gather(self, t, group="tp", out=None):
        g = self.groups[group]
        if g.size == 1:
            if out is not None:
                out.copy_(t)
                return out
            return t
        res = self._coll(group, "all_gather", t.contiguous(), lambda xs: torch.cat(xs, 0))
        if out is None:
            return res.clone()
        out.copy_(res)
        return out

    def reduce_scatter(self, t, group="ep", out=None):
        g = self.groups[group]
        if g.size == 1:
            return t
        full = self._coll(group, "reduce_scatter", t.contiguous(),
                          lambda xs: torch.stack([x.float() for x in xs]).sum(0).to(xs[0].dtype))
        n = t.shape[0] // g.size
        part = full[g.rank_in_group * n:(g.rank_in_group + 1) * n]
        if out is None:
            return part.clone()
        out.copy_(part)
        return out

    def all_to_all_v(self, t, send_splits, group="ep"):
        g = self.groups[group]
        if g.size == 1:
            return t, list(send_splits)
        me = g.rank_in_group
        # split sizes meet in a checked collective; the ragged row blocks travel through the
        # (src, dst) queues, so a shape mismatch on either side is reported by recv()
        splits_all = self._coll(group, "a2a_splits", torch.tensor(send_splits, dtype=torch.int64),
                                lambda xs: torch.stack(xs))
        off = 0
        for r, n in enumerate(send_splits):
            self.world.send(self.rank, g.ranks[r], t[off:off + n])
            off += n
        recv_splits = [int(splits_all[r][me]) for r in range(g.size)]
        parts = []
        for r, n in enumerate(recv_splits):
            like = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype)
            parts.append(self.world.recv(g.ranks[r], self.rank, like))
        return torch.cat(parts, 0).to(t.device), recv_splits

    def all_to_all(self, t, group="ep", out=None):
        g = self.groups[group]
        if g.size == 1:
            if out is not None:
                out.copy_(t)
                return out
            return t
        self._conform("all_to_all", group, t.numel() * t.element_size())
        me, n = g.rank_in_group, g.size
        self.stats["calls"] += 1
        allx = self._coll(group, "all_to_all", t.contiguous(), lambda xs: torch.stack(xs))
        res = torch.cat([allx[r].chunk(n, 0)[me] for r in range(n)], 0)
        if out is None:
            return res.clone()
        out.copy_(res)
        return out

    def all_reduce_max_int(self, values, group="world"):
        g = self.groups[group]
        if g.size == 1:
            return list(values)
        t = torch.tensor(values, dtype=torch.int64)
        return [int(v) for v in self._coll(group, "max_int", t, lambda xs: torch.stack(xs).max(0).values)]

    def broadcast_(self, t, src_in_group=0, group="world"):
        g = self.groups[group]
        if g.size == 1:
            return t
        src = src_in_group
        t.copy_(self._coll(group, f"broadcast{src}", t, lambda xs: xs[src].clone()))
        return t

    def barrier(self, group="world"):
        g = self.groups[group]
        if g.size > 1:
            self._coll(group, "barrier", torch.zeros(1), lambda xs: xs[0])

    def send(self, t, dst):
        self.stats["send_bytes"] += t.numel() * t.element_size()
        self.world.send(self.rank, dst, t)

    def recv(self, t, src):
        self.stats["recv_bytes"] += t.numel() * t.element_size()
        t.copy_(self.world.recv(src, self.rank, t))
        return t

    def isend(self, t, dst):
        self.send(t, dst)
        return _Done()

    def irecv(self, t, src):
        self.recv(t, src)
        return _Done()

    def prepost_ok(self) -> bool:
        # the loopback irecv completes on the spot; posting it a tick early still exercises
        # the engine's pre-post ordering (the matching send happened earlier in that tick)
        return True

    def enable_ep_ipc(self, capmax: int, hidden: int, top_k: int) -> bool:
        """The IPC dispatch's protocol in shared CPU memory (parallel/ep_ipc.EpLoopback)."""
        if self.groups["ep"].size not in (2, 4, 8):
            return False
        from .ep_ipc import EpLoopback

        self.ep_ipc = EpLoopback(self, capmax, hidden, top_k)
        return True

    def enable_ep_ipc_prefill(self, capmax: int, hidden: int, top_k: int) -> bool:
        """The prefill-sized IPC exchange, emulated on its own shared buffers."""
        if self.groups["ep"].size not in (2, 4, 8):
            return False
        from .ep_ipc import EpLoopback

        self.ep_ipc_prefill = EpLoopback(self, capmax, hidden, top_k, name="ep_ipc_prefill")
        return True

    def check_health(self):
        return None
