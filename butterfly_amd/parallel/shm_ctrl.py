"""Node-local control plane: the max of a few host integers over a group whose ranks share one
host, through a POSIX shared-memory segment instead of a gloo all-reduce.

Every expert-parallel step starts with an agreement over the EP group (engine._ep_agree: padded
rows, any prefill, any work), and lockstep data-parallel engines agree on liveness each step
(has_unfinished_global). On gloo that is a TCP round trip through the store's sockets: 0.4-0.9
ms at 2-8 ranks on the build box, with multi-millisecond p99s (profiles/r6_ctrl_plane_probe.jsonl).
The asynchronous engine hides it behind the device's step as long as it stays well below the
step, but it is pure host latency on every rank, every step.

Here each rank owns two slots (one per step parity) of [sequence, v0 .. v{W-1}] int64 words in
one segment. A call writes its values, then publishes the sequence number (x86 stores are not
reordered with each other, and the sequence write is the last one); it then polls the peers'
slots of the same parity until each carries the same sequence, and takes the element-wise max.
Two parities are enough: a rank can only start call k+2 after every peer has published call
k+1, which each peer does only after it finished reading call k.

Bounded: a peer that never arrives (died, diverged) raises after BFLY_COMM_TIMEOUT_S instead of
spinning forever. The segment is created by the group's first rank, its name broadcast over the
group's gloo process group, and unlinked as soon as every rank has mapped it (nothing is left in
/dev/shm however the job ends); close() unmaps.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np

WORDS = 16                    # values per call (a call may pass fewer)
_SLOT = 1 + WORDS             # [seq, values...]


class ShmCtrl:
    def __init__(self, ranks: list, rank_in_group: int, pg, tag: str, timeout_s: float = 300.0):
        import torch.distributed as dist
        from multiprocessing import shared_memory

        self.n, self.me = len(ranks), rank_in_group
        self.timeout_s = timeout_s
        self.calls = 0
        size = self.n * 2 * _SLOT * 8
        name = [None]
        self._owner = rank_in_group == 0
        if self._owner:
            nm = f"bfly_ctrl_{os.getpid()}_{tag}"
            self._shm = shared_memory.SharedMemory(name=nm, create=True, size=size)
            np.ndarray((size // 8,), dtype=np.int64, buffer=self._shm.buf)[:] = -1
            name[0] = nm
        dist.broadcast_object_list(name, src=ranks[0], group=pg)
        if not self._owner:
            self._shm = shared_memory.SharedMemory(name=name[0], create=False)
            try:   # attaching processes must not unlink the owner's segment at exit
                from multiprocessing import resource_tracker

                resource_tracker.unregister(self._shm._name, "shared_memory")
            except Exception:
                pass
        self.name = name[0]
        self._a = np.ndarray((self.n, 2, _SLOT), dtype=np.int64, buffer=self._shm.buf)
        dist.barrier(group=pg)     # every rank attached before the first call
        if self._owner:
            # the name is no longer needed: unlinked now, the mappings stay valid, and nothing
            # is left in /dev/shm however the job ends
            self._shm.unlink()

    def max(self, values: list) -> list:
        """Element-wise max of `values` (<= WORDS integers) over the group; collective."""
        k = len(values)
        if k > WORDS:
            raise ValueError(f"at most {WORDS} values per call")
        seq = self.calls
        self.calls += 1
        par = seq & 1
        mine = self._a[self.me, par]
        mine[1:1 + k] = values
        mine[0] = seq                      # publish last
        out = list(values)
        pending = [r for r in range(self.n) if r != self.me]
        t0 = time.perf_counter()
        spins = 0
        while pending:
            rest = []
            for r in pending:
                slot = self._a[r, par]
                if slot[0] == seq:
                    vals = slot[1:1 + k]
                    for i in range(k):
                        if vals[i] > out[i]:
                            out[i] = int(vals[i])
                else:
                    rest.append(r)
            pending = rest
            if pending:
                spins += 1
                if spins > 64:
                    time.sleep(0)          # peers are late: yield the CPU
                    if time.perf_counter() - t0 > self.timeout_s:
                        raise TimeoutError(f"shared-memory control plane: ranks {pending} of the group "
                                           f"never reached call {seq} ({self.timeout_s:.0f}s)")
        return [int(v) for v in out]

    def close(self) -> None:
        if self._shm is None:
            return
        self._a = None
        try:
            self._shm.close()
        except BufferError:
            pass
        self._shm = None


def same_host(pg, ranks: list) -> bool:
    """Every rank of the group runs on this host (collective over `pg`)."""
    import socket

    import torch.distributed as dist

    hosts = [None] * len(ranks)
    dist.all_gather_object(hosts, socket.gethostname(), group=pg)
    return len(set(hosts)) == 1


def make(ranks: list, rank_in_group: int, pg, tag: str, timeout_s: Optional[float] = None) -> Optional[ShmCtrl]:
    """A ShmCtrl for the group when its ranks share this host, else None (collective)."""
    from ..utils import flags

    if len(ranks) < 2 or pg is None or not same_host(pg, ranks):
        return None
    t = flags.get("BFLY_COMM_TIMEOUT_S") if timeout_s is None else timeout_s
    return ShmCtrl(ranks, rank_in_group, pg, tag, timeout_s=float(t) if t and t > 0 else 300.0)
