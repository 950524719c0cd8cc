"""Feature-flag registry ("Use feature flags for incompatible changes during transition",
/root/reference/CLAUDE.md:81).

Every BFLY_* environment flag the framework reads is declared here once, with its type,
default and meaning; `dump()` prints the effective values at startup so a run's behaviour is
reproducible from its log.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Callable


@dataclass(frozen=True)
class Flag:
    name: str
    default: Any
    parse: Callable[[str], Any]
    help: str


def _bool(s: str) -> bool:
    return s.strip().lower() in ("1", "true", "yes", "on")


FLAGS: dict[str, Flag] = {}


def define(name: str, default, parse, help: str) -> Flag:
    f = Flag(name, default, parse, help)
    FLAGS[name] = f
    return f


define("BFLY_POISON_OUTPUTS", False, _bool, "allocate every op output filled with NaN / a negative sentinel so elements "
       "a kernel leaves unwritten show up (debug; read at import, ops.set_poison at run time)")
define("BFLY_DEBUG_CHECKS", False, _bool, "host-side index checks (one sync each) in ops whose kernels cannot raise, "
       "e.g. gather_rows (read at import)")
define("BFLY_MOE_BIG_TILE", True, _bool, "prefill-scale MoE expert GEMMs (>= 256 routed rows per local expert) on "
       "the 256x256 8-phase tile over the device tile list (read at import)")
define("BFLY_GRAPH_SAMPLING", True, _bool, "a last stage's decode hipGraphs end with the token sampler (per-request "
       "temperatures / seeds staged with the inputs: one replay per step); top-k / top-p rows sample eagerly")
define("BFLY_DISABLE_GRAPHS", False, _bool, "run decode steps eagerly instead of replaying hipGraphs")
define("BFLY_CUSTOM_AR", True, _bool, "use the one-shot IPC all-reduce kernel (self-tested at start-up, "
       "RCCL otherwise) for small TP all-reduces")
define("BFLY_CUSTOM_AR_MAX_BYTES", 8 << 20, int, "largest all-reduce (bytes) routed to the IPC kernel")
define("BFLY_CUSTOM_AR_AUTOTUNE", True, _bool, "time the IPC all-reduce (one- / two-shot) against RCCL at start-up "
       "and route each message size to the faster one (0: the fixed BFLY_CUSTOM_AR_* thresholds)")
define("BFLY_AR_BUTTERFLY", "", str, "\"W@lo:hi[,...]\": all-reduces of lo..hi bytes over a group of W ranks (bare "
       "\"lo:hi\": any power-of-two group) run as the butterfly "
       "(recursive halving + doubling over point-to-point transfers, parallel/butterfly.py), outside graph capture; set by "
       "the start-up probe only where it measured faster than RCCL and the IPC kernel (empty = never)")
define("BFLY_PROBE_BUTTERFLY", False, _bool, "the start-up comm probe also times the butterfly all-reduce (and may "
       "route sizes to it through BFLY_AR_BUTTERFLY)")
define("BFLY_CUSTOM_AR_2SHOT_BYTES", 512 << 10, int, "IPC all-reduces of at least this many bytes over 4 or 8 "
       "ranks run as reduce-scatter + all-gather (2S/W bytes per link instead of S; 0 = always one-shot)")
define("BFLY_GEMM_TUNED", True, _bool, "consult the measured GEMM plan table (0: heuristic plans only; read by the kernel library)")
define("BFLY_GEMM_NT_WEIGHTS", True, _bool, "stream decode GEMM weights with the non-temporal policy (read by the kernel library)")
define("BFLY_GEMM_PLAN", "", str, "force GEMM plans for whole-model A/B runs: \"N,K,Mbucket:kind,mt,nt,wk,bm,bn,sk;...\" "
       "(read by the kernel library)")
define("BFLY_ATTN_XCD", 1, int, "prefill attention: XCD-aware item walk (0: plain order; read by the kernel library)")
define("BFLY_ATTN_TRACE", "", str, "set: the prefill attention kernel stamps its item phases into the LSE buffer "
       "instead of writing results (tools/attn_trace.py; read by the kernel library)")
define("BFLY_KERNEL_LIB", "", str, "path of another build of the kernel library (same-box A/B runs of kernel changes)")
define("BFLY_LOG_JSON", False, _bool, "emit log records as one JSON object per line")
define("BFLY_RESTART", 0, int, "restart attempt of this job (set by `launch --max-restarts`; 0 = first run)")
define("BFLY_ATTN_PAGED_LDS", True, _bool, "paged-prefix prefill attention: the LDS-staged kernel for chunks of "
       "several sequences (0: the register kernel everywhere; read by the kernel library)")
define("BFLY_DEFER_REDUCE", True, _bool, "fuse split-K GEMM reduces into the consuming rope / add+rmsnorm kernels")
define("BFLY_NORM_ROWSCALE", True, _bool, "decode add+RMSNorm split over (row, 1024-column) workgroups that write x * g "
       "and partial sums of squares; the consuming QKV / gate-up GEMM applies the 1/rms row scale in its epilogue "
       "(tp == 1, batches <= BFLY_NORM_ROWSCALE_MAX_ROWS; 0: one-workgroup-per-row add+RMSNorm)")
define("BFLY_NORM_ROWSCALE_MAX_ROWS", 256, int, "largest batch that takes the row-split add+RMSNorm")
define("BFLY_PROGRAM_CHECK", True, _bool, "enforce the rank's step program on every decode step of a multi-rank "
       "engine (world_size > 1): each collective the model issues is checked against the program's next "
       "instruction before it is issued (comm.Communicator.expect); a divergence raises ProgramMismatch instead "
       "of hanging the group. Host-side only, on eager steps and graph warm-up / capture passes: a graph "
       "replay issues nothing from the host, so replayed steps cost nothing")
define("BFLY_PP_PREPOST", True, _bool, "asynchronous pipeline on RCCL: post each stage's boundary receive one tick "
       "early on a dedicated comm stream into one of two persistent buffers (event-guarded reuse)")
define("BFLY_NATIVE_RCCL", True, _bool, "data-path collectives (all-reduce / all-gather / reduce-scatter / "
       "all-to-all) and pipeline edges on the rank's own RCCL communicators (world init + ncclCommSplit "
       "per mesh axis, parallel/rccl.py) instead of torch ProcessGroups, whenever the backend is RCCL "
       "(the multi-GPU preflight turns it off if its native check fails); 0 = torch ProcessGroups")
define("BFLY_PP_NATIVE_EDGES", True, _bool, "with native RCCL: pipeline boundaries on two-rank edge communicators "
       "(receive captured in the stage's decode graph, A/B sends on a side stream); 0 = torch ProcessGroup "
       "send/recv with pre-posted receives (the preflight's pp_edge_graph check turns it off on failure)")
define("BFLY_NATIVE_A2A", True, _bool, "with native RCCL: the EP all-to-all (fixed-capacity decode dispatch) on the "
       "native communicator; 0 = torch ProcessGroup (the preflight's native_a2a_graph check turns it off)")
define("BFLY_RCCL_INIT_TIMEOUT_S", 180.0, float, "deadline of a native RCCL communicator init / split (non-blocking "
       "setup polled by the host); expiry aborts it and raises TimeoutError")
define("BFLY_RCCL_CLOSE_TIMEOUT_S", 30.0, float, "deadline of a native RCCL communicator finalize at teardown; expiry "
       "aborts it instead")
define("BFLY_IPC_SHARED_DEVICE", False, _bool, "allow the IPC all-reduce / EP exchange for groups whose ranks share "
       "one GPU (tests only: spin-waiting workgroups of one rank can starve a co-resident rank's kernels of CUs)")
define("BFLY_SEQ_PARALLEL", False, _bool, "TP prefill with sequence parallelism: the residual stream and the norms are "
       "split by tokens over the TP group (reduce-scatter + all-gather replace each all-reduce)")
define("BFLY_SEQ_PARALLEL_MIN_TOKENS", 256, int, "sequence parallelism only on prefill steps with at least this many tokens")
define("BFLY_MOE_SPARSE", True, _bool, "prefill MoE layers: token-routed grouped expert GEMMs instead of the dense path")
define("BFLY_PACKED_DECODE", True, _bool, "engines whose decode batch is at most 512 rows keep K-tile-blocked copies of "
       "projection weights for the decode GEMMs in the HBM left after the KV cache (BFLY_PACKED_KINDS)")
define("BFLY_PACKED_KINDS", "gu_w,moe_gu_w,qkv_w,o_w", str, "projection kinds packed by BFLY_PACKED_DECODE, in "
       "priority order: a kind is packed whole or not at all, while the HBM lasts (down_w / moe_down_w also "
       "work: whole-step within noise, profiles/r6_packed/kinds_ab.log; o_w runs its own packed plan where one is "
       "tuned, gemm.hip kPackedTuned)")
define("BFLY_MOE_NORM_ROUTE", True, _bool, "MoE layers at tp = 1: the add+RMSNorm over the O projection's split-K "
       "slabs also routes the rows (0: separate moe_route launch)")
define("BFLY_MOE_GATE_EPILOGUE", True, _bool, "dense MoE decode path: the routing weights applied in the gate/up "
       "GEMM's epilogue (0: separate moe_gate_scale pass)")
define("BFLY_EP_DECODE_A2A", True, _bool, "EP MoE on decode (and idle) steps: fixed-capacity all-to-all dispatch with "
       "routed-rows-only expert GEMMs, graph-capturable (0: all-gather + dense local experts + reduce-scatter)")
define("BFLY_EP_IPC", True, _bool, "EP MoE on decode: byte-minimal dispatch / return over peer IPC buffers "
       "(only routed rows travel; self-tested at start-up, else the fixed-capacity all-to-all)")
define("BFLY_EP_IPC_PREFILL", True, _bool, "EP MoE on prefill steps (with BFLY_EP_IPC): the byte-minimal IPC exchange "
       "sized for the prefill budget, routed by a device scan and bounded by device-resident row counts (no host "
       "sync per layer; else the host-split variable all-to-all)")
define("BFLY_EP_ALLTOALL", True, _bool, "EP MoE on prefill steps: dispatch tokens by all-to-all (else all-gather / reduce-scatter)")
define("BFLY_PP_ASYNC", True, _bool, "pipeline parallelism: keep pp decode groups in flight across steps "
       "(one group per stage per tick, no fill/drain bubble) instead of per-step microbatching")
define("BFLY_DIST_BACKEND", "", str, "torch.distributed backend override for init_distributed (default: nccl "
       "= RCCL with a GPU, gloo without; gloo lets several ranks share one GPU in tests)")
define("BFLY_FORCE_CPU", False, _bool, "bench.py: run on the CPU reference path even when a GPU is visible "
       "(BASELINE config 1, the gloo plumbing configuration)")
define("BFLY_RCCL_POLL_S", 1.0, float, "period of the thread polling native RCCL communicators for async errors "
       "(on one: abort every communicator, exit 75); 0 = off")
define("BFLY_SHM_CTRL", True, _bool, "data-parallel / expert-parallel per-step host agreements (EP padding, "
       "lockstep liveness) through a shared-memory segment when the group's ranks share a host, instead of a "
       "gloo all-reduce (parallel/shm_ctrl.py)")
define("BFLY_COMM_TIMEOUT_S", 600.0, float, "collective / process-group timeout in seconds")
define("BFLY_HEARTBEAT_S", 5.0, float, "health heartbeat period (0 disables the watchdog)")
define("BFLY_STEP_TIMEOUT_S", 0.0, float, "engine step watchdog: terminate a rank whose step exceeds this (0 = off)")
define("BFLY_FAULT", "", str, "fault injection 'rank:step:kind' (kind: hang|exit|nan) for tests")
define("BFLY_PREFLIGHT", True, _bool, "multi-rank jobs (bench.py): run the bounded-time multi-GPU preflight "
       "(parallel/preflight.py) before partitioning; failed features fall back, a hang exits 75")
define("BFLY_PREFLIGHT_TIMEOUT_S", 90.0, float, "deadline of each preflight check (seconds)")
define("BFLY_PREFLIGHT_INJECT", "", str, "preflight fault injection 'check:kind[:rank],...' (kind: fail|raise|hang)")
define("BFLY_NAN_CHECK", True, _bool, "check the logits of every sampled step for NaN/Inf and fail the step "
       "(one reduction over the local vocab shard per step)")
define("BFLY_TRACE", "", str, "write a chrome-trace JSON of engine steps to this path")
define("BFLY_ROCTX", False, _bool, "emit roctx ranges (visible in rocprofv3 --marker-trace)")
define("BFLY_LOG_LEVEL", "INFO", str, "log level of the rank-tagged logger")
define("BFLY_OFFLOAD_ARCH", "gfx950", str, "HIP offload architecture for the kernel build")
define("BFLY_HOST_CXX", "/opt/rocm/lib/llvm/bin/clang++", str, "host compiler for the torch bindings")


def get(name: str):
    f = FLAGS[name]
    v = os.environ.get(name)
    return f.default if v is None or v == "" else f.parse(v)


def dump() -> dict:
    return {n: get(n) for n in sorted(FLAGS)}
