"""Communication layer ("Low-overhead inter-node communication for tensor passing",
/root/reference/CLAUDE.md:20).

One process per GPU; collectives go through torch.distributed — backend "nccl" is RCCL on
ROCm (xGMI on MI355X), "gloo" for the CPU plumbing configuration and the control plane.
`Communicator` binds a rank to the process groups of its mesh axes (tp / pp / dp / ep) and
exposes the handful of collectives the rank programs need:

  all_reduce_   TP sum after row-parallel O / down projections (and vocab-parallel embed)
  all_gather    TP sampling (score, id) pairs
  all_to_all    EP token dispatch / return (fixed capacity on decode, graph-capturable)
  all_to_all_v  EP dispatch on prefill steps (variable sizes, host-exchanged splits)
  send / recv   PP stage boundary activations and token feedback
  broadcast_    control-plane metadata

Small TP all-reduces (decode) can be routed to a one-shot peer-to-peer kernel
(parallel/custom_allreduce.py) instead of RCCL; everything else stays on RCCL. On RCCL
(BFLY_NATIVE_RCCL, on by default) the data-path collectives of every multi-rank group go to the rank's own
RCCL communicators (parallel/rccl.py: world init + one ncclCommSplit per mesh axis) instead of
torch's ProcessGroups; control-plane ops (host integers, barriers) stay on torch.
Every op is stream-ordered and allocation-free when given outputs, so it can be captured
in a hipGraph together with the compute kernels.
"""
from __future__ import annotations

import contextlib
import datetime
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from .mesh import Mesh


class ProgramMismatch(RuntimeError):
    """A collective this rank was about to issue is not the next one of its step program."""


class NativeWork:
    """Completion handle of a native RCCL point-to-point transfer issued on a side stream:
    `wait()` makes the CURRENT stream wait for it (torch Work semantics), `event` lets a
    caller order later work on it directly."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)

    def is_completed(self) -> bool:
        return self.event.query()


@dataclass
class GroupHandle:
    ranks: list
    pg: Optional[object]          # torch ProcessGroup, None when size == 1
    rank_in_group: int
    native: Optional[object] = None   # parallel/rccl.RcclComm (BFLY_NATIVE_RCCL) for the data path
    ctrl: Optional[object] = None     # gloo ProcessGroup for host integers when `pg` is RCCL
    shm: Optional[object] = None      # parallel/shm_ctrl.ShmCtrl: node-local host-integer max

    @property
    def size(self) -> int:
        return len(self.ranks)


class Communicator:
    def __init__(self, mesh: Mesh, rank: int, groups: dict[str, GroupHandle]):
        self.mesh = mesh
        self.rank = rank
        self.groups = groups
        self.custom_ar = None            # optional CustomAllReduce for the tp group
        self.ep_ipc = None               # optional byte-minimal EP dispatch (parallel/ep_ipc.py)
        self.ep_ipc_prefill = None       # the same exchange sized for prefill steps (no host sync)
        self.stats = {"all_reduce_bytes": 0, "send_bytes": 0, "recv_bytes": 0, "calls": 0}
        # native RCCL pipeline edges (parallel/rccl.pp_edges): to the next / from the previous
        # stage; sends run on their own stream so a send never blocks the compute stream
        self.pp_native_send = None
        self.pp_native_recv = None
        self._send_stream = None
        self._expect = None              # [instructions, cursor] while a step program is enforced

    # -- construction ---------------------------------------------------------------------
    @classmethod
    def single(cls) -> "Communicator":
        m = Mesh()
        g = GroupHandle([0], None, 0)
        return cls(m, 0, {"tp": g, "pp": g, "dp": g, "ep": g, "world": g})

    @classmethod
    def from_mesh(cls, mesh: Mesh) -> "Communicator":
        """Create every group of the mesh (collective: all ranks must call this)."""
        if mesh.world_size == 1 or not dist.is_initialized():
            if mesh.world_size != 1:
                raise RuntimeError("torch.distributed not initialised for a multi-rank mesh")
            return cls.single()
        rank = dist.get_rank()
        groups: dict[str, GroupHandle] = {}
        for axis in ("tp", "pp", "dp"):
            mine = None
            for ranks in mesh.all_groups(axis):
                pg = dist.new_group(ranks) if len(ranks) > 1 else None
                if rank in ranks:
                    mine = GroupHandle(ranks, pg, ranks.index(rank))
            groups[axis] = mine
        if dist.get_backend() == "nccl" and mesh.dp > 1:
            # control plane of the data-parallel / expert-parallel axis: host integers (EP
            # padding and step-mode agreement, lockstep liveness) over gloo on CPU tensors, so
            # agreeing never waits for the device (an RCCL all-reduce read back with .tolist()
            # would drain the compute stream every step)
            for ranks in mesh.all_groups("dp"):
                cpg = dist.new_group(ranks, backend="gloo")
                if rank in ranks:
                    groups["dp"].ctrl = cpg
        from ..utils import flags

        if mesh.dp > 1 and flags.get("BFLY_SHM_CTRL"):
            # the per-step host agreements of the data-parallel / expert-parallel axis through
            # shared memory when the group's ranks share a host (parallel/shm_ctrl.py); each
            # group sets its own up (group-local collectives on its host-side process group)
            from .shm_ctrl import make

            g = groups["dp"]
            gi = next(i for i, rs in enumerate(mesh.all_groups("dp")) if rank in rs)
            g.shm = make(g.ranks, g.rank_in_group, g.ctrl if g.ctrl is not None else g.pg, f"dp{gi}")
        groups["ep"] = groups["dp"] if mesh.ep > 1 else GroupHandle([rank], None, 0)
        groups["world"] = GroupHandle(list(range(mesh.world_size)), dist.group.WORLD, rank)
        comm = cls(mesh, rank, groups)

        gpu_rccl = dist.get_backend() == "nccl" and torch.cuda.is_available()
        if gpu_rccl and flags.get("BFLY_PREFLIGHT"):
            # every multi-GPU entry point (bench, CLI, LLM, server) gets the bounded-time
            # preflight before the native communicators / IPC paths are switched on: a failed
            # check turns its feature off here on every rank (collective, same point everywhere)
            from .preflight import ensure_preflight

            ensure_preflight()
        if flags.get("BFLY_NATIVE_RCCL") and gpu_rccl:
            comm.enable_native_rccl()
        if flags.get("BFLY_CUSTOM_AR") and mesh.tp > 1 and torch.cuda.is_available():
            comm.enable_custom_all_reduce(flags.get("BFLY_CUSTOM_AR_MAX_BYTES"))
        return comm

    @staticmethod
    def _nccl(g: GroupHandle) -> bool:
        # tensor-form collectives on RCCL; list forms on gloo (also used with GPU tensors
        # when several ranks share one device, which RCCL refuses)
        if g.pg is None:
            return False
        try:
            return dist.get_backend(g.pg) == "nccl"
        except (ValueError, RuntimeError):   # not a torch ProcessGroup (the loopback backend)
            return False

    # -- queries ----------------------------------------------------------------------------
    def size(self, group: str = "tp") -> int:
        return self.groups[group].size

    def rank_in(self, group: str = "tp") -> int:
        return self.groups[group].rank_in_group

    # -- rank-program conformance ----------------------------------------------------------
    @contextlib.contextmanager
    def expect(self, instrs):
        """Enforce a step program on the collectives issued inside the block:
        every one is checked against the program's next instruction BEFORE it is issued (op,
        group, payload), so a rank whose model code diverged from the program raises here,
        naming both, instead of entering a collective its peers never issue (a hang on RCCL).
        At the end of the block every listed instruction must have been issued."""
        prev, self._expect = self._expect, [list(instrs), 0]
        try:
            yield
            todo = self._expect[0][self._expect[1]:]
            if todo:
                raise ProgramMismatch(f"rank {self.rank}: the step ended with {len(todo)} program instruction(s) "
                                      f"not issued, the first: {todo[0].op} {todo[0].group} ({todo[0].note})")
        finally:
            self._expect = prev

    @contextlib.contextmanager
    def _unchecked(self):
        """Collectives issued inside are one program instruction already conformed by the
        caller (e.g. the all-to-all pair standing in for an IPC EP dispatch)."""
        prev, self._expect = self._expect, None
        try:
            yield
        finally:
            self._expect = prev

    def _conform(self, op: str, group: str, nbytes: Optional[int] = None) -> None:
        e = self._expect
        if e is None:
            return
        instrs, i = e
        ranks = tuple(self.groups[group].ranks)
        if i >= len(instrs):
            raise ProgramMismatch(f"rank {self.rank}: {op} on {ranks} ({nbytes} B) issued after the step program's "
                                  f"last instruction")
        ins = instrs[i]
        if ins.op != op or tuple(ins.group) != ranks or (nbytes is not None and ins.nbytes != nbytes):
            raise ProgramMismatch(f"rank {self.rank}: about to issue {op} on {ranks} ({nbytes} B) where the step "
                                  f"program's instruction {i} is {ins.op} on {ins.group} ({ins.nbytes} B, {ins.note})")
        e[1] = i + 1

    # -- collectives --------------------------------------------------------------------------
    def all_reduce_(self, t, group: str = "tp") -> torch.Tensor:
        """In-place sum over the group; returns the reduced tensor. `t` may be a deferred
        split-K GEMM output (ops.Partial): the IPC kernel reduces its slabs while publishing,
        any other path materialises it first."""
        from .. import ops

        g = self.groups[group]
        if g.size == 1:
            return ops.materialize(t)
        nb = t.shape[0] * t.shape[1] * 2 if isinstance(t, ops.Partial) else t.numel() * t.element_size()
        self._conform("all_reduce", group, nb)
        self.stats["calls"] += 1
        self.stats["all_reduce_bytes"] += nb
        if group == "tp" and self.custom_ar is not None and self.custom_ar.should_use(t):
            return self.custom_ar.all_reduce_(t)
        t = ops.materialize(t)
        if self._butterfly_fits(g, t):
            from .butterfly import butterfly_all_reduce_

            return butterfly_all_reduce_(t, g.ranks, g.pg)
        if g.native is not None:
            return g.native.all_reduce_(t)
        dist.all_reduce(t, group=g.pg)
        return t

    def _butterfly_fits(self, g: GroupHandle, t: torch.Tensor) -> bool:
        """The probe routed this message size, for groups of this size, to the butterfly
        all-reduce (BFLY_AR_BUTTERFLY), the group is a power of two and no graph is being
        captured (its point-to-point steps run eagerly). The flag is re-parsed whenever its value
        changes, so an all-reduce issued before the probe sets it does not switch it off."""
        ranges = butterfly_ranges()
        if not ranges or g.size & (g.size - 1) or g.pg is None:
            return False
        rng = ranges.get(g.size)
        if rng is None:
            return False
        if t.is_cuda and torch.cuda.is_current_stream_capturing():
            return False
        lo, hi = rng
        return lo <= t.numel() * t.element_size() <= hi

    def all_reduce_max_(self, t: torch.Tensor, group: str = "tp") -> torch.Tensor:
        """In-place element-wise max over the group (stream-ordered, capturable on RCCL)."""
        g = self.groups[group]
        if g.size == 1:
            return t
        self.stats["calls"] += 1
        if g.native is not None:
            return g.native.all_reduce_(t, "max")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g.pg)
        return t

    def all_reduce_rms_norm_(self, t: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor,
                             group: str = "tp") -> torch.Tensor:
        """residual += all_reduce(t); return rms_norm(residual) * w — one fused kernel on the
        IPC path (the all-reduce feeding every transformer block's add+norm), else RCCL
        all-reduce followed by the fused add+norm kernel."""
        from .. import ops

        g = self.groups[group]
        car = self.custom_ar
        if g.size > 1 and group == "tp" and car is not None and car.should_use(t):
            self._conform("all_reduce", group, t.shape[0] * t.shape[1] * 2)
            self.stats["calls"] += 1
            self.stats["all_reduce_bytes"] += t.shape[0] * t.shape[1] * 2
            return car.all_reduce_rms_norm_(t, w, eps, residual)
        t = self.all_reduce_(t, group)
        return ops.rms_norm(t, w, eps, residual=residual)

    def enable_custom_all_reduce(self, max_bytes: int) -> bool:
        """Set up the one-shot IPC all-reduce for the TP group (collective over the group).
        Returns True when it passed its self-test and will be used."""
        g = self.groups["tp"]
        if g.size not in (2, 4, 8) or not torch.cuda.is_available():
            return False
        import logging

        from ..utils import flags
        from .custom_allreduce import CustomAllReduce

        log = logging.getLogger("butterfly_amd.comm")
        car = CustomAllReduce(g.ranks, g.rank_in_group, g.pg, max_bytes=max_bytes)
        self.custom_ar = car if car.ok else None
        if not car.ok:
            car.close()
            return False
        self._start_poller()
        if flags.get("BFLY_CUSTOM_AR_AUTOTUNE") and (g.native is not None or dist.get_backend(g.pg) == "nccl"):
            # route by measurement on this node (IPC kernel vs RCCL per message size)
            def rccl(t, g=g):
                if g.native is not None:
                    return g.native.all_reduce_(t)
                dist.all_reduce(t, group=g.pg)
                return t

            tuning = car.autotune(g.pg, rccl)
            log.info("custom all-reduce routing: %s", tuning)
            if car.route_bytes <= 0:
                log.info("custom all-reduce: RCCL is faster at every decode size here; keeping RCCL")
                car.close()
                self.custom_ar = None
        return self.custom_ar is not None

    def enable_ep_ipc(self, capmax: int, hidden: int, top_k: int) -> bool:
        """Set up the byte-minimal IPC EP dispatch for the decode MoE layer (collective over the
        EP group; eager, before any graph capture). True when it passed its self-test."""
        g = self.groups["ep"]
        if g.size not in (2, 4, 8) or not torch.cuda.is_available() or g.pg is None:
            return False
        from .ep_ipc import EpIpc

        ipc = EpIpc(g.ranks, g.rank_in_group, g.pg, capmax, hidden, top_k)
        self.ep_ipc = ipc if ipc.ok else None
        if not ipc.ok:
            ipc.close()
        else:
            self._start_poller()
        return self.ep_ipc is not None

    def enable_ep_ipc_prefill(self, capmax: int, hidden: int, top_k: int) -> bool:
        """A second IPC exchange sized for prefill steps (`capmax` tokens per source: the
        engine's prefill budget). Its receive blocks are bounded by device-resident row counts,
        so an EP prefill MoE layer needs no host synchronisation (ep_ipc.EpIpc.dispatch_prefill)."""
        g = self.groups["ep"]
        if g.size not in (2, 4, 8) or not torch.cuda.is_available() or g.pg is None:
            return False
        from .ep_ipc import EpIpc

        ipc = EpIpc(g.ranks, g.rank_in_group, g.pg, capmax, hidden, top_k)
        self.ep_ipc_prefill = ipc if ipc.ok else None
        if not ipc.ok:
            ipc.close()
        else:
            self._start_poller()
        return self.ep_ipc_prefill is not None

    def ep_dispatch(self, x: torch.Tensor, ids: torch.Tensor, w: torch.Tensor, slots, experts_per_rank: int,
                    cap: int):
        """Fixed-capacity EP token dispatch (decode): every token goes once to each EP rank
        owning one of its top-k experts. Returns an ep_ipc.EpRoute: this rank's routed rows,
        their local expert ids / weights, and the slots to combine the returned rows. Byte-
        minimal IPC path when enabled, else ep_pack + two all-to-alls (bitwise the same)."""
        from .. import ops
        from .ep_ipc import EpRoute

        ipc = self.ep_ipc
        if ipc is not None and ipc.fits(x, ids, cap):
            self._conform("ep_dispatch", "ep")   # routed bytes depend on the routing: op and group only
            return ipc.dispatch(x, ids, w, slots, experts_per_rank, cap)
        k = ids.shape[1]
        send, meta, slot = ops.ep_pack(x, ids, w, slots, experts_per_rank, self.size("ep"), cap)
        if ipc is not None:
            # the IPC path is set up (the program lists ep_dispatch) but this call does not fit
            # it (rows beyond its capacity): every EP rank takes this fallback together, and the
            # all-to-all pair IS the program's dispatch step
            self._conform("ep_dispatch", "ep")
            with self._unchecked():
                xr = self.all_to_all(send, "ep")
                mr = self.all_to_all(meta, "ep")
        else:
            xr = self.all_to_all(send, "ep")
            mr = self.all_to_all(meta, "ep")
        return EpRoute(xr, mr[:, :k].contiguous().view(torch.int32), mr[:, k:].contiguous(), slot,
                       x.shape[0], "a2a")

    def ep_combine(self, y: torch.Tensor, route) -> torch.Tensor:
        """Return every routed row's expert output to its source and sum each token's rows (f32,
        fixed rank order)."""
        from .. import ops

        if route.path != "a2a":
            self._conform("ep_return", "ep")
            return self.ep_ipc.combine(y, route)
        if self.ep_ipc is not None:             # the fallback of a listed ep_dispatch (above)
            self._conform("ep_return", "ep")
            with self._unchecked():
                back = self.all_to_all(y, "ep")
            return ops.ep_combine(back, route.slot)
        return ops.ep_combine(self.all_to_all(y, "ep"), route.slot)

    def enable_native_rccl(self) -> dict:
        """Create the rank's native RCCL communicators (collective over the world): the world
        one from a broadcast unique id, then one ncclCommSplit per mesh axis. Returns
        {axis: RcclComm} for the groups that now use them."""
        from .rccl import RcclComm, pp_edges, split_mesh

        world = RcclComm.world()
        natives = split_mesh(world, self.mesh, self.rank)
        for axis, nc in natives.items():
            self.groups[axis].native = nc
        self.groups["world"].native = world
        self.pp_native_send, self.pp_native_recv = pp_edges(world, self.mesh, self.rank)
        self._start_poller()
        return natives

    def _start_poller(self) -> None:
        """One error-poller thread per process (parallel/rccl.async_errors): native RCCL async
        errors and the IPC kernels' host-mapped timeout words, checked every second even while
        the main thread is stuck in a step."""
        if getattr(self, "_rccl_poller", None) is None:
            from .rccl import start_error_poller
            self._rccl_poller = start_error_poller()

    def graph_safe(self) -> bool:
        """True when every collective a decode step issues inside its graph is capturable:
        single-rank groups, RCCL (native or ProcessGroup), or the IPC kernels. A gloo data-path
        collective (ranks sharing one GPU in tests) is not: its host staging would invalidate
        the capture, so such engines decode eagerly."""
        for axis, ipc in (("tp", self.custom_ar), ("ep", self.ep_ipc), ("pp", None)):
            g = self.groups.get(axis)
            if g is None or g.size == 1 or g.native is not None or self._nccl(g) or ipc is not None:
                continue
            if axis == "pp" and not self.native_p2p:
                continue      # pipeline transfers run outside the graph unless on native edges
            return False
        return True

    def capturable(self, group: str) -> bool:
        """A collective over `group` can be captured into a hipGraph (single rank, native RCCL or
        an RCCL ProcessGroup; not gloo, whose host staging invalidates a capture)."""
        g = self.groups.get(group)
        return g is None or g.size == 1 or g.native is not None or self._nccl(g)

    def close(self) -> dict:
        """Tear down this rank's native resources, bounded: the IPC buffers, then the native
        RCCL communicators (edges, axes, world) through their finalize-or-abort close. Graphs
        that captured any of them must be gone first (LLMEngine.close). Returns {name: status}."""
        out = {}
        if getattr(self, "_rccl_poller", None) is not None:
            self._rccl_poller.stop()
            self._rccl_poller = None
        for name in ("custom_ar", "ep_ipc", "ep_ipc_prefill"):
            obj = getattr(self, name)
            if obj is not None:
                obj.close()
                setattr(self, name, None)
                out[name] = "closed"
        comms = [("pp_send", self.pp_native_send), ("pp_recv", self.pp_native_recv)]
        comms += [(k, g.native) for k, g in self.groups.items() if g is not None and g.native is not None]
        seen = set()
        for name, c in comms:
            if c is None or id(c) in seen:
                continue
            seen.add(id(c))
            out[name] = c.close()
        self.pp_native_send = self.pp_native_recv = None
        for g in self.groups.values():
            if g is not None:
                g.native = None
                if g.shm is not None:
                    g.shm.close()
                    g.shm = None
                    out["shm_ctrl"] = "closed"
        return out

    @property
    def native_p2p(self) -> bool:
        """Pipeline boundary transfers run on native RCCL edge communicators."""
        return self.pp_native_send is not None or self.pp_native_recv is not None

    def _edge(self, peer: int, sending: bool):
        if sending:
            return self.pp_native_send if peer == self.mesh.next_stage(self.rank) else None
        return self.pp_native_recv if peer == self.mesh.prev_stage(self.rank) else None

    def send_stream(self, device) -> "torch.cuda.Stream":
        if self._send_stream is None:
            self._send_stream = torch.cuda.Stream(device)
        return self._send_stream

    def recv_native(self, t: torch.Tensor) -> torch.Tensor:
        """Receive from the previous stage on the CURRENT stream (capturable: a stage's decode
        graph starts with it, landing the boundary rows in the graph's static input)."""
        self.pp_native_recv.recv(t, 0)
        return t

    def check_health(self) -> None:
        """Raise if the IPC all-reduce recorded a peer-wait timeout (a rank stopped arriving:
        its results since then are not trustworthy) or a native RCCL communicator reports an
        asynchronous error. Cheap: one 4-byte device read plus host queries."""
        if self.custom_ar is not None and self.custom_ar.error():
            raise RuntimeError(f"rank {self.rank}: custom all-reduce peer wait timed out")
        if self.ep_ipc is not None and self.ep_ipc.error():
            raise RuntimeError(f"rank {self.rank}: EP IPC dispatch peer wait timed out")
        for name, g in self.groups.items():
            if g is not None and g.native is not None:
                err = g.native.async_error()
                if err:
                    raise RuntimeError(f"rank {self.rank}: RCCL communicator '{name}' async error {err}")

    def all_gather(self, t: torch.Tensor, group: str = "tp", out: torch.Tensor | None = None) -> torch.Tensor:
        g = self.groups[group]
        if g.size == 1:
            if out is not None:
                out.copy_(t)
                return out
            return t
        if out is None:
            out = torch.empty((g.size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if g.native is not None:
            return g.native.all_gather(t, out)
        if self._nccl(g):
            dist.all_gather_into_tensor(out, t.contiguous(), group=g.pg)
        else:  # gloo: list form
            dist.all_gather(list(out.chunk(g.size, 0)), t.contiguous(), group=g.pg)
        return out

    def reduce_scatter(self, t: torch.Tensor, group: str = "ep", out: torch.Tensor | None = None) -> torch.Tensor:
        g = self.groups[group]
        if g.size == 1:
            return t
        n = t.shape[0] // g.size
        if out is None:
            out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if g.native is not None:
            return g.native.reduce_scatter(t, out)
        if self._nccl(g):
            dist.reduce_scatter_tensor(out, t.contiguous(), group=g.pg)
        else:  # gloo has no reduce_scatter: all-reduce then slice
            full = t.contiguous().clone()
            dist.all_reduce(full, group=g.pg)
            out.copy_(full[g.rank_in_group * n:(g.rank_in_group + 1) * n])
        return out

    def all_to_all_v(self, t: torch.Tensor, send_splits: list, group: str = "ep") -> tuple:
        """Variable-size all-to-all along dim 0 (EP token dispatch / return): rows
        [sum(send_splits[:r]), +send_splits[r]) go to group rank r. Returns (received rows in
        source-rank order, recv_splits). The split sizes are exchanged first (host sync), so
        this is an eager (prefill) primitive; decode keeps fixed-shape collectives."""
        g = self.groups[group]
        if g.size == 1:
            return t, list(send_splits)
        dev = t.device if self._nccl(g) else torch.device("cpu")
        sc = torch.tensor(send_splits, dtype=torch.int64, device=dev)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=g.pg)
        recv_splits = [int(v) for v in rc.tolist()]
        src = t.contiguous() if self._nccl(g) else t.detach().cpu().contiguous()
        out = torch.empty((sum(recv_splits),) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
        dist.all_to_all_single(out, src, output_split_sizes=recv_splits, input_split_sizes=list(send_splits),
                               group=g.pg)
        self.stats["calls"] += 1
        return out.to(t.device), recv_splits

    def all_to_all(self, t: torch.Tensor, group: str = "ep", out: torch.Tensor | None = None) -> torch.Tensor:
        """Equal-split all-to-all along dim 0: block r of `t` (t.shape[0] / n rows) goes to group
        rank r; block r of the result came from group rank r. Fixed shapes and no host sync,
        so it is stream-ordered and hipGraph-capturable on RCCL (the EP decode dispatch)."""
        from ..utils import flags

        g = self.groups[group]
        if g.size == 1:
            if out is not None:
                out.copy_(t)
                return out
            return t
        self._conform("all_to_all", group, t.numel() * t.element_size())
        if out is None:
            out = torch.empty_like(t)
        self.stats["calls"] += 1
        if g.native is not None and flags.get("BFLY_NATIVE_A2A"):
            return g.native.all_to_all(t, out)
        if self._nccl(g):
            dist.all_to_all_single(out, t.contiguous(), group=g.pg)
            return out
        # gloo: host staging (CPU tensors pass straight through)
        src = t.detach().cpu().contiguous()
        dst = torch.empty_like(src)
        dist.all_to_all_single(dst, src, group=g.pg)
        out.copy_(dst)
        return out

    def all_reduce_max_int(self, values: list, group: str = "world") -> list:
        """Host-side max of a few integers over a group (control plane, e.g. EP padding)."""
        g = self.groups[group]
        if g.size == 1:
            return list(values)
        if g.shm is not None:         # node-local shared memory: a few microseconds, no sockets
            return g.shm.max(values)
        if g.ctrl is not None:        # gloo control plane: no device work, no stream sync
            t = torch.tensor(values, dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g.ctrl)
            return [int(v) for v in t.tolist()]
        dev = "cuda" if dist.get_backend(g.pg) == "nccl" else "cpu"
        t = torch.tensor(values, dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g.pg)
        return [int(v) for v in t.tolist()]

    def prepost_ok(self) -> bool:
        """Receives may be posted ahead of their use (non-blocking, stream-ordered): RCCL."""
        return self._world_nccl()

    def broadcast_ints(self, values: Optional[list], n: int, src_in_group: int, group: str = "dp") -> list:
        """Host list of n integers from one group rank to all (control plane: e.g. the prompt
        of an engine context-parallel step). Device-staged on RCCL, host tensors on gloo."""
        g = self.groups[group]
        if g.size == 1:
            return list(values)
        dev = "cuda" if self._nccl(g) else "cpu"
        t = torch.tensor(values, dtype=torch.int64, device=dev) if g.rank_in_group == src_in_group \
            else torch.empty(n, dtype=torch.int64, device=dev)
        dist.broadcast(t, g.ranks[src_in_group], group=g.pg)
        return [int(v) for v in t.tolist()]

    def _world_nccl(self) -> bool:
        return dist.is_initialized() and dist.get_backend() == "nccl"

    def send(self, t: torch.Tensor, dst: int) -> None:
        self.stats["send_bytes"] += t.numel() * t.element_size()
        nc = self._edge(dst, True)
        if nc is not None:
            nc.send(t.contiguous(), 1)          # stream-ordered on the current stream
            return
        if t.is_cuda and not self._world_nccl():   # gloo point-to-point needs host memory
            dist.send(t.detach().cpu().contiguous(), dst)
            return
        dist.send(t.contiguous(), dst)

    def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
        self.stats["recv_bytes"] += t.numel() * t.element_size()
        nc = self._edge(src, False)
        if nc is not None:
            nc.recv(t, 0)
            return t
        if t.is_cuda and not self._world_nccl():
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src)
            t.copy_(h)
            return t
        dist.recv(t, src)
        return t

    def isend(self, t: torch.Tensor, dst: int):
        self.stats["send_bytes"] += t.numel() * t.element_size()
        nc = self._edge(dst, True)
        if nc is not None:
            # on the send stream, after everything the current stream has queued (the producer);
            # the allocator keeps `t` alive until the send stream is past it
            s = self.send_stream(t.device)
            s.wait_stream(torch.cuda.current_stream(t.device))
            t = t.contiguous()
            with torch.cuda.stream(s):
                nc.send(t, 1)
                ev = torch.cuda.Event()
                ev.record(s)
            t.record_stream(s)
            return NativeWork(ev)
        if t.is_cuda and not self._world_nccl():
            return dist.isend(t.detach().cpu().contiguous(), dst)
        return dist.isend(t.contiguous(), dst)

    def irecv(self, t: torch.Tensor, src: int):
        self.stats["recv_bytes"] += t.numel() * t.element_size()
        nc = self._edge(src, False)
        if nc is not None:
            nc.recv(t, 0)                      # on the current stream (a pre-poster's comm stream)
            ev = torch.cuda.Event()
            ev.record()
            return NativeWork(ev)
        return dist.irecv(t, src)

    def broadcast_(self, t: torch.Tensor, src_in_group: int = 0, group: str = "world") -> torch.Tensor:
        """In-place broadcast from group rank `src_in_group`. On the group's native RCCL
        communicator (the pipeline's per-tick token-id feedback, group "pp") it is ONE
        stream-ordered ncclBroadcast on the current stream: no ProcessGroup work object or
        watchdog per tick, and the ids never leave the device."""
        g = self.groups[group]
        if g.size == 1:
            return t
        self.stats["calls"] += 1
        if g.native is not None and t.is_cuda:
            return g.native.broadcast_(t, src_in_group)   # split keys = group order
        dist.broadcast(t, g.ranks[src_in_group], group=g.pg)
        return t

    def barrier(self, group: str = "world") -> None:
        g = self.groups[group]
        if g.size > 1:
            dist.barrier(group=g.pg)


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from the torchrun environment (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT). Returns (rank, world_size, local_rank). Idempotent; a
    no-op single-process setup when WORLD_SIZE is absent or 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 or dist.is_initialized():
        return (dist.get_rank(), dist.get_world_size(), local) if dist.is_initialized() else (0, 1, 0)
    if backend is None:
        from ..utils import flags

        backend = flags.get("BFLY_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    t = timeout_s or float(os.environ.get("BFLY_COMM_TIMEOUT_S", "600"))
    kwargs = {}
    if backend == "nccl":
        kwargs["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=t), **kwargs)
    return rank, world, local


_bf_cache: tuple = ("", {})


def butterfly_ranges() -> dict:
    """BFLY_AR_BUTTERFLY as {group size: (lo, hi) bytes}. Entries "W@lo:hi" separated by ','
    (what the probe writes: the range it measured for groups of W ranks); a bare "lo:hi"
    applies to every power-of-two group (manual runs)."""
    global _bf_cache
    import os

    raw = os.environ.get("BFLY_AR_BUTTERFLY", "")
    if raw == _bf_cache[0]:
        return _bf_cache[1]
    out: dict = {}
    for ent in filter(None, (e.strip() for e in raw.split(","))):
        size, _, rng = ent.rpartition("@")
        lo, hi = (int(v) for v in rng.split(":"))
        if size:
            out[int(size)] = (lo, hi)
        else:
            for w in (2, 4, 8, 16, 32, 64):
                out.setdefault(w, (lo, hi))
    _bf_cache = (raw, out)
    return out
