"""One-shot IPC all-reduce for the TP group.

Each rank allocates one uncached device buffer, exports it with hipIpcGetMemHandle, and the
group exchanges handles over the (already initialised) process group. The all-reduce itself
is one HIP kernel (csrc/kernels/allreduce.hip): publish own rows, flag every peer, read the
peers' rows directly over xGMI and sum in fixed rank order, so all ranks hold bitwise
identical results. `all_reduce_rms_norm_` additionally fuses the residual add and RMSNorm
that follow every TP all-reduce in the transformer block, removing one kernel and one pass
over the activations per all-reduce.

Only messages up to `max_bytes` (default BFLY_CUSTOM_AR_MAX_BYTES) go here — the decode
all-reduces; larger ones (prefill) stay on RCCL. From `two_shot_bytes` on (groups of 4 or 8)
the kernel runs as reduce-scatter + all-gather over the same buffers: every link then carries
2S/W instead of S bytes, at the price of a second rendezvous. Construction runs a self-test; if the IPC
mapping, the kernel or the flag protocol misbehave on this machine, the instance reports
`ok = False` and the communicator keeps using RCCL.
"""
from __future__ import annotations

import logging

import torch
import torch.distributed as dist

from .. import ops

log = logging.getLogger("butterfly_amd.comm")


def device_identity(index: int) -> str:
    """Physical identity of a GPU (host + PCI domain/bus/device): equal for two ranks exactly
    when they drive the same card, whatever each process's device numbering."""
    import socket

    p = torch.cuda.get_device_properties(index)
    return f"{socket.gethostname()}:{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"


def shared_device_refusal(idents: list, what: str) -> str | None:
    """Reason to refuse an IPC group whose ranks share a GPU, or None. The flag-rendezvous
    kernels spin while they wait for a peer's workgroups; on a shared GPU those spinning
    workgroups of one rank can hold the CU resources a co-resident rank's kernel needs to reach
    the rendezvous (co-residency starvation: the Llama-3-70B tp4 shared-GPU rehearsal stall,
    profiles/r4_tp4_stall/). Tests opt in with BFLY_IPC_SHARED_DEVICE=1."""
    from ..utils import flags

    if len(set(idents)) == len(idents) or flags.get("BFLY_IPC_SHARED_DEVICE"):
        return None
    return (f"{what}: ranks of the group share a GPU ({idents}); spin-waiting IPC kernels can starve "
            "each other's workgroups there, so the group keeps RCCL / the all-to-all "
            "(BFLY_IPC_SHARED_DEVICE=1 allows it for tests)")


def choose_routing(sizes: list, times: list) -> tuple:
    """(route_bytes, two_shot_bytes) from measured times per size (ascending) of [one-shot,
    two-shot, RCCL] (inf = not available): messages go to the IPC kernel up to the largest size
    of the prefix of sizes where its faster variant beats RCCL (0: never), and the two-shot
    variant from the smallest size on which it beats the one-shot one at that and every larger
    routed size (0: never)."""
    route = 0
    for sz, (one, two, rccl) in zip(sizes, times):
        if min(one, two) <= rccl:
            route = sz
        else:
            break
    two_from = 0
    for i in range(len(sizes) - 1, -1, -1):
        if sizes[i] > route:
            continue
        one, two, _ = times[i]
        if two < one:
            two_from = sizes[i]
        else:
            break
    return route, two_from


class CustomAllReduce:
    def __init__(self, ranks: list, rank_in_group: int, pg, max_bytes: int = 8 << 20,
                 device: torch.device | None = None, two_shot_bytes: int | None = None):
        ops.require_library()
        self.world = len(ranks)
        self.rank = rank_in_group
        self.cap = int(max_bytes)
        self.route_bytes = self.cap        # largest message routed here (autotune may lower it)
        self.tuning: dict | None = None
        if two_shot_bytes is None:
            from ..utils import flags

            two_shot_bytes = flags.get("BFLY_CUSTOM_AR_2SHOT_BYTES")
        self.two_shot_bytes = int(two_shot_bytes)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        if self.world not in (2, 4, 8):
            raise ValueError("custom all-reduce supports groups of 2, 4 or 8 ranks")
        L = torch.ops.bfly
        L.health_init()          # host-mapped timeout words, allocated before any capture
        self._ptr = 0
        self._opened = []
        self.bases = []
        self.ok = False
        # every step below is collective: a local failure is voted on, never raised alone
        handle = None
        try:
            self._ptr = L.car_alloc(L.car_buffer_bytes(self.cap))
            handle = bytes(L.car_ipc_handle(self._ptr).tolist())
        except Exception as e:  # noqa: BLE001
            log.warning("custom all-reduce: buffer export failed (%r)", e)
        # the kernel loads peer rows directly: every peer GPU must be reachable over P2P
        # (xGMI). Ranks sharing one device (the 1-GPU test setup) need no peer mapping.
        me = self.device.index if self.device.index is not None else torch.cuda.current_device()
        handles: list = [None] * self.world
        dist.all_gather_object(handles, (handle, me, device_identity(me)), group=pg)
        devs = [d for _, d, _ in handles]
        refusal = shared_device_refusal([i for _, _, i in handles], "custom all-reduce")
        # ranks sharing one GPU (tests): a smaller grid per rank, so the spinning workgroups of the
        # ranks that arrive first cannot hold every CU while a late rank still has to run a
        # one-workgroup-per-CU GEMM before it reaches the rendezvous (seen as a 20 s flag-wait
        # timeout in the 4-rank production-dims test); the same on every rank
        shared = len({i for _, _, i in handles}) < len(handles)
        self.blocks = max(1, 128 // self.world) if shared else 128
        handles = [h for h, _, _ in handles]
        local_ok = all(h is not None for h in handles)
        if refusal:
            log.warning(refusal)
            local_ok = False
        try:
            unreachable = [d for d in devs if d != me and not torch.cuda.can_device_access_peer(me, d)]
        except Exception as e:  # noqa: BLE001
            unreachable = [repr(e)]
        if unreachable:
            log.warning("custom all-reduce: no P2P access from device %d to %s; using RCCL",
                        me, unreachable)
            local_ok = False
        if local_ok:
            try:
                for r, h in enumerate(handles):
                    if r == self.rank:
                        self.bases.append(self._ptr)
                    else:
                        p = L.car_ipc_open(torch.tensor(list(h), dtype=torch.uint8))
                        self._opened.append(p)
                        self.bases.append(p)
            except Exception as e:  # noqa: BLE001
                log.warning("custom all-reduce: opening a peer buffer failed (%r)", e)
                local_ok = False
        self._armed = False
        if self._vote(local_ok, pg):
            from .rccl import health_arm, health_quiet

            with health_quiet(word="car") as q:   # a timeout here is a fallback vote, not a failure
                self.ok = self._self_test(pg)
                q.failed(not self.ok)
            if self.ok:
                health_arm("car")
                self._armed = True

    # ---------------------------------------------------------------------------------------
    def should_use(self, t) -> bool:
        if isinstance(t, ops.Partial):   # split-K slabs: reduced inside the all-reduce kernel
            t = t.out
        return (self.ok and t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2
                and t.is_contiguous() and t.shape[1] % 8 == 0 and t.shape[1] <= 16384
                and t.numel() * 2 <= self.route_bytes and t.data_ptr() % 16 == 0)

    def use_two_shot(self, t: torch.Tensor) -> bool:
        return (self.world >= 4 and 0 < self.two_shot_bytes <= t.numel() * 2
                and (t.shape[1] // 8) % self.world == 0)

    def all_reduce_(self, t, two_shot: bool | None = None) -> torch.Tensor:
        """In place; `t` may be a deferred split-K GEMM output (ops.Partial), whose reduce the
        kernel fuses into its publish step (the result lands in t.out)."""
        if isinstance(t, ops.Partial):
            two = self.use_two_shot(t.out) if two_shot is None else two_shot
            torch.ops.bfly.custom_all_reduce(t.out, t.out, None, None, 0.0, self.bases, self.rank, self.cap,
                                             t.slabs, two, self.blocks)
            return t.out
        two = self.use_two_shot(t) if two_shot is None else two_shot
        torch.ops.bfly.custom_all_reduce(t, t, None, None, 0.0, self.bases, self.rank, self.cap, None, two,
                                         self.blocks)
        return t

    def all_reduce_rms_norm_(self, t, w: torch.Tensor, eps: float,
                             residual: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """residual += all_reduce(t) (bf16), returns rms_norm(residual) * w. `t` may be an
        ops.Partial (split-K slabs reduced in the kernel)."""
        slabs = None
        if isinstance(t, ops.Partial):
            t, slabs = t.out, t.slabs
        if out is None:
            out = torch.empty_like(t)
        torch.ops.bfly.custom_all_reduce(t, out, residual, w, float(eps), self.bases, self.rank, self.cap, slabs,
                                         self.use_two_shot(t), self.blocks)
        return out

    def autotune(self, pg, rccl_all_reduce, sizes=(32 << 10, 128 << 10, 512 << 10, 2 << 20, 8 << 20),
                 iters: int = 20) -> dict:
        """Route by measurement instead of by fixed thresholds: time this kernel (one-shot and,
        for groups of 4 / 8, two-shot) against `rccl_all_reduce` at decode-sized messages, take
        the slowest rank's time per (size, variant) — a MAX all-reduce over the group, so every
        rank decides the same — and set `route_bytes` / `two_shot_bytes` from it
        (`choose_routing`). Collective: every rank of the group calls it, in the same order."""
        from .rccl import health_quiet

        with health_quiet(word="car") as q:
            tuning = self._autotune(pg, rccl_all_reduce, sizes, iters)
            q.failed(self.route_bytes == 0)
        return tuning

    def _autotune(self, pg, rccl_all_reduce, sizes, iters: int) -> dict:
        dev = self.device
        inf = float("inf")
        rows_of = [max(1, sz // (8192 * 2)) for sz in sizes]
        times = []
        for rows in rows_of:
            # every call sums W copies in place: small values, restored before each variant, so
            # the timed data stays finite (W = 8 x 23 calls would overflow bf16 otherwise)
            src = (torch.randn(rows, 8192, device=dev) * 1e-3).to(torch.bfloat16)
            t = src.clone()
            fits = rows * 8192 * 2 <= self.cap
            row = []
            for fn in ((lambda: self.all_reduce_(t, two_shot=False)) if fits else None,
                       (lambda: self.all_reduce_(t, two_shot=True)) if fits and self.world >= 4 else None,
                       lambda: rccl_all_reduce(t)):
                if fn is None:
                    row.append(inf)
                    continue
                t.copy_(src)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize(dev)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(iters):
                    fn()
                b.record()
                torch.cuda.synchronize(dev)
                row.append(a.elapsed_time(b) * 1e3 / iters)
            times.append(row)
        T = torch.tensor([[min(v, 1e30) for v in r] for r in times], dtype=torch.float64)
        T = T.to(dev) if dist.get_backend(pg) == "nccl" else T
        dist.all_reduce(T, op=dist.ReduceOp.MAX, group=pg)
        T = T.cpu().tolist()
        route, two = choose_routing([r * 8192 * 2 for r in rows_of], T)
        self.route_bytes, self.two_shot_bytes = min(route, self.cap), two
        self.tuning = {"sizes": [r * 8192 * 2 for r in rows_of], "us": [[round(v, 1) for v in r] for r in T],
                       "route_bytes": self.route_bytes, "two_shot_bytes": self.two_shot_bytes}
        if not self._vote(self.error() == 0, pg):      # a flag wait timed out somewhere: RCCL
            self.route_bytes = 0
        return self.tuning

    def error(self) -> int:
        """Sticky device error word (non-zero after a flag-wait timeout)."""
        return int(torch.ops.bfly.car_error(self._ptr))

    def clear_error(self) -> None:
        torch.ops.bfly.car_clear_error(self._ptr)

    def _vote(self, good: bool, pg) -> bool:
        """True iff `good` on every rank of the group."""
        flag = torch.tensor([1 if good else 0], dtype=torch.int32,
                            device=self.device if dist.get_backend(pg) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=pg)
        return bool(flag.item())

    def _self_test(self, pg) -> bool:
        """Every call is followed by a group vote on its error word, so a flag wait that timed
        out (peer stores never seen, e.g. no cross-device visibility) costs the spin limit once:
        the group stops together (a rank that went on alone would wait out every later call).
        Every rank runs the same sequence of votes whatever fails locally."""
        good = True
        modes = [False, True] if self.world >= 4 else [False]
        cases = [(rows, dim, two) for rows, dim in ((3, 64), (130, 4096)) for two in modes]
        for rows, dim, two in cases:
            x = torch.arange(rows * dim, device=self.device, dtype=torch.float32).view(rows, dim)
            x = ((x % 17) + self.rank).to(torch.bfloat16)
            want = sum(((x.float() - self.rank) + r) for r in range(self.world)).to(torch.bfloat16)
            y = None
            for _ in range(3):      # exercise both buffer parities
                try:
                    y = x.clone()
                    self.all_reduce_(y, two_shot=two)
                    torch.cuda.synchronize(self.device)
                    call_ok = self.error() == 0
                except Exception as e:  # noqa: BLE001 — any failure means: keep RCCL
                    log.warning("custom all-reduce self-test raised %r", e)
                    call_ok = False
                if not self._vote(call_ok, pg):
                    good = False
                    break
            if not good:
                break
            good = bool(torch.equal(y, want))
            if not self._vote(good, pg):
                good = False
                break
        if not good:
            log.warning("custom all-reduce self-test failed on some rank; using RCCL")
        return good

    def close(self) -> None:
        L = torch.ops.bfly
        if getattr(self, "_armed", False):
            from .rccl import health_arm

            health_arm("car", False)
            self._armed = False
        for p in self._opened:
            L.car_ipc_close(p)
        self._opened = []
        if self._ptr:
            torch.cuda.synchronize(self.device)
            L.car_free(self._ptr)
            self._ptr = 0
        self.ok = False
