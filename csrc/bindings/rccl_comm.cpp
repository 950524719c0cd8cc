// Native RCCL communicator: the rank's communicators as RCCL objects
// owned here rather than torch ProcessGroups, so the data-path collectives are ONE
// stream-ordered RCCL call each (no work objects, no watchdog events, no allocator record
// streams) and capture into the decode hipGraph like the kernels around them.
//
//   rccl_unique_id()                       rank 0 creates the id; the caller ships its 128 bytes
//                                          to the other ranks over the control plane
//   rccl_init(uid, nranks, rank, t)        ncclCommInitRankConfig on the current device -> handle
//   rccl_split(h, color, key, t)           ncclCommSplit: one call per mesh axis (tp / pp / dp)
//                                          from the world communicator; color < 0 -> no group
//   rccl_all_reduce / all_gather / reduce_scatter / all_to_all / broadcast / send / recv
//                                          on torch's current stream, in place or into `out`
//   rccl_group_start / rccl_group_end      batch point-to-point calls (PP fan-out)
//   rccl_async_error(h)                    ncclCommGetAsyncError, polled by the health monitor
//   rccl_release(h, abort, t)              finalize + destroy (bounded) or abort one communicator
//   rccl_live() / rccl_abort_all()         live handles (polled by the async-error watcher);
//                                          abort every one on the failure path
//
// NON-BLOCKING communicators (ncclConfig_t.blocking = 0): init, split and
// finalize run in RCCL's background thread while this thread polls ncclCommGetAsyncError
// against a deadline `t` (seconds). A peer that never joins therefore ends in a named
// TimeoutError-style exception after ncclCommAbort, not in a process that can only be killed.
// Teardown is ncclCommFinalize (flushes the communicator's queued work, polled) followed by
// ncclCommDestroy; a finalize that outlives its deadline is aborted instead and reported, so a
// teardown can never wedge the job. (Destroying a communicator while a hipGraph that captured
// its kernels is alive waits for that graph: callers drop their graphs first.) A collective on
// a non-blocking communicator may return ncclInProgress while RCCL sets up a connection; the
// call then polls to completion of the enqueue (the GPU work itself stays asynchronous).
//
// Handles are indices into a process-wide table (a rank drives a few communicators at most).
// This links the librccl.so torch itself loads, so there is exactly one RCCL in the process.
// On one node every communicator runs over xGMI; RCCL refuses two ranks on one device, which
// is why the one-GPU test box can only run nranks = 1 communicators.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

using at::Tensor;

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define RCCL_CHECK(call)                                                                         \
  do {                                                                                           \
    const ncclResult_t r_ = (call);                                                              \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL: " #call " failed: ", ncclGetErrorString(r_));          \
  } while (0)

std::mutex g_mu;
std::vector<ncclComm_t> g_comms;   // handle -> communicator (nullptr once destroyed)

ncclComm_t comm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "RCCL: bad communicator handle ", h);
  return g_comms[h];
}

int64_t add_comm(ncclComm_t c) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

// Poll a non-blocking communicator until its pending operation (init / split / finalize /
// connection setup) is done. Returns the communicator's state, or ncclInProgress when
// `timeout_s` passed first (<= 0: no deadline).
ncclResult_t wait_ready(ncclComm_t c, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  for (;;) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t r = ncclCommGetAsyncError(c, &st);
    if (r != ncclSuccess) return r;
    if (st != ncclInProgress) return st;
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0 && dt > timeout_s) return ncclInProgress;
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

double g_call_timeout_s = 600.0;   // enqueue deadline of data-path calls (rccl_set_call_timeout)

// A data-path call returned; complete its enqueue if the communicator is still busy.
void finish_call(ncclResult_t r, ncclComm_t c, const char* what) {
  if (r == ncclInProgress) r = wait_ready(c, g_call_timeout_s);
  TORCH_CHECK(r != ncclInProgress, "RCCL: ", what, " did not complete its enqueue within ", g_call_timeout_s, " s");
  TORCH_CHECK(r == ncclSuccess, "RCCL: ", what, " failed: ", ncclGetErrorString(r));
}

#define RCCL_CALL(what, c, call) finish_call((call), (c), what)

ncclConfig_t nonblocking_config() {
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  return cfg;
}

ncclDataType_t dtype_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kFloat8_e4m3fn: return ncclUint8;   // moved, never reduced
    default: TORCH_CHECK(false, "RCCL: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t op_of(int64_t op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclProd;
    default: TORCH_CHECK(false, "RCCL: reduction op must be 0 sum / 1 max / 2 min / 3 prod");
  }
}

void check_dev(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL: ", what, " must be a contiguous GPU tensor");
}

Tensor rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  Tensor out = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), id.internal, NCCL_UNIQUE_ID_BYTES);
  return out;
}

// A pending init / split that failed or outlived its deadline: abort it and raise. The
// message starts with "RCCL-TIMEOUT" for a deadline (parallel/rccl.py maps it to TimeoutError).
void settle_or_abort(ncclComm_t c, ncclResult_t st, double timeout_s, const char* what) {
  if (st == ncclSuccess) return;
  (void)ncclCommAbort(c);
  TORCH_CHECK(st != ncclInProgress, "RCCL-TIMEOUT: ", what, " not complete after ", timeout_s,
              " s (a peer never joined); communicator aborted");
  TORCH_CHECK(false, "RCCL: ", what, " failed: ", ncclGetErrorString(st));
}

int64_t rccl_init(const Tensor& uid, int64_t nranks, int64_t rank, double timeout_s) {
  TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte && uid.numel() == NCCL_UNIQUE_ID_BYTES,
              "rccl_init: uid must be the 128-byte CPU tensor from rccl_unique_id");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "rccl_init: rank out of range");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  ncclConfig_t cfg = nonblocking_config();
  const ncclResult_t r = ncclCommInitRankConfig(&c, (int)nranks, id, (int)rank, &cfg);   // current device
  TORCH_CHECK((r == ncclSuccess || r == ncclInProgress) && c != nullptr, "RCCL: ncclCommInitRankConfig failed: ",
              ncclGetErrorString(r));
  settle_or_abort(c, wait_ready(c, timeout_s), timeout_s, "ncclCommInitRankConfig");
  return add_comm(c);
}

int64_t rccl_split(int64_t h, int64_t color, int64_t key, double timeout_s) {
  ncclComm_t c = comm_of(h), out = nullptr;
  ncclConfig_t cfg = nonblocking_config();
  const ncclResult_t r = ncclCommSplit(c, color < 0 ? NCCL_SPLIT_NOCOLOR : (int)color, (int)key, &out, &cfg);
  TORCH_CHECK(r == ncclSuccess || r == ncclInProgress, "RCCL: ncclCommSplit failed: ", ncclGetErrorString(r));
  // the split runs on the parent too (colour exchange): settle both
  const ncclResult_t sp = wait_ready(c, timeout_s);
  TORCH_CHECK(sp != ncclInProgress, "RCCL-TIMEOUT: ncclCommSplit (parent) not complete after ", timeout_s, " s");
  TORCH_CHECK(sp == ncclSuccess, "RCCL: ncclCommSplit (parent) failed: ", ncclGetErrorString(sp));
  if (out == nullptr) return -1;
  settle_or_abort(out, wait_ready(out, timeout_s), timeout_s, "ncclCommSplit");
  return add_comm(out);
}

void rccl_set_call_timeout(double timeout_s) { g_call_timeout_s = timeout_s; }

std::vector<int64_t> rccl_info(int64_t h) {
  ncclComm_t c = comm_of(h);
  int n = 0, r = 0, dev = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  RCCL_CHECK(ncclCommUserRank(c, &r));
  RCCL_CHECK(ncclCommCuDevice(c, &dev));
  return {r, n, dev};
}

int64_t rccl_version() {
  int v = 0;
  RCCL_CHECK(ncclGetVersion(&v));
  return v;
}

void rccl_all_reduce(int64_t h, Tensor& t, int64_t op) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  ncclComm_t c = comm_of(h);
  RCCL_CALL("ncclAllReduce", c, ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), op_of(op), c, cur_stream()));
}

void rccl_all_gather(int64_t h, const Tensor& inp, Tensor& out) {
  check_dev(inp, "input");
  check_dev(out, "output");
  ncclComm_t c = comm_of(h);
  int n = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  TORCH_CHECK(out.numel() == inp.numel() * n && out.scalar_type() == inp.scalar_type(), "rccl_all_gather: out size");
  c10::DeviceGuard g(inp.device());
  RCCL_CALL("ncclAllGather", c, ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), dtype_of(inp), c, cur_stream()));
}

void rccl_reduce_scatter(int64_t h, const Tensor& inp, Tensor& out, int64_t op) {
  check_dev(inp, "input");
  check_dev(out, "output");
  ncclComm_t c = comm_of(h);
  int n = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  TORCH_CHECK(inp.numel() == out.numel() * n && out.scalar_type() == inp.scalar_type(), "rccl_reduce_scatter: sizes");
  c10::DeviceGuard g(inp.device());
  RCCL_CALL("ncclReduceScatter", c,
            ncclReduceScatter(inp.data_ptr(), out.data_ptr(), out.numel(), dtype_of(inp), op_of(op), c, cur_stream()));
}

// Equal-split all-to-all along dim 0 (the EP decode dispatch): block r of `inp` -> rank r.
void rccl_all_to_all(int64_t h, const Tensor& inp, Tensor& out) {
  check_dev(inp, "input");
  check_dev(out, "output");
  ncclComm_t c = comm_of(h);
  int n = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  TORCH_CHECK(inp.numel() == out.numel() && inp.numel() % n == 0 && out.scalar_type() == inp.scalar_type(),
              "rccl_all_to_all: sizes");
  c10::DeviceGuard g(inp.device());
  RCCL_CALL("ncclAllToAll", c, ncclAllToAll(inp.data_ptr(), out.data_ptr(), inp.numel() / n, dtype_of(inp), c, cur_stream()));
}

void rccl_broadcast(int64_t h, Tensor& t, int64_t root) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  ncclComm_t c = comm_of(h);
  RCCL_CALL("ncclBroadcast", c, ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), (int)root, c, cur_stream()));
}

void rccl_send(int64_t h, const Tensor& t, int64_t peer) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  ncclComm_t c = comm_of(h);
  RCCL_CALL("ncclSend", c, ncclSend(t.data_ptr(), t.numel(), dtype_of(t), (int)peer, c, cur_stream()));
}

void rccl_recv(int64_t h, Tensor& t, int64_t peer) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  ncclComm_t c = comm_of(h);
  RCCL_CALL("ncclRecv", c, ncclRecv(t.data_ptr(), t.numel(), dtype_of(t), (int)peer, c, cur_stream()));
}

void rccl_group_start() { RCCL_CHECK(ncclGroupStart()); }

// On non-blocking communicators ncclGroupEnd may return ncclInProgress: settle every live one.
void rccl_group_end() {
  const ncclResult_t r = ncclGroupEnd();
  TORCH_CHECK(r == ncclSuccess || r == ncclInProgress, "RCCL: ncclGroupEnd failed: ", ncclGetErrorString(r));
  if (r != ncclInProgress) return;
  std::vector<ncclComm_t> live;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (ncclComm_t c : g_comms)
      if (c != nullptr) live.push_back(c);
  }
  for (ncclComm_t c : live) finish_call(ncclInProgress, c, "ncclGroupEnd");
}

// 0 = healthy; otherwise the ncclResult_t of an asynchronous failure (peer gone, timeout).
// The query runs under the table lock (it is a non-blocking flag read), so the poller thread
// can never race a concurrent rccl_release / rccl_abort_all into a destroyed communicator.
int64_t rccl_async_error(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "RCCL: bad communicator handle ", h);
  ncclResult_t st = ncclSuccess;
  RCCL_CHECK(ncclCommGetAsyncError(g_comms[h], &st));
  return (int64_t)st;
}

// Bounded teardown of one communicator. Returns 1 after a clean finalize + destroy, 0 when it
// was aborted (on request, or because the finalize outlived `timeout_s`), -1 when the handle
// was already released.
int64_t rccl_release(int64_t h, bool abort, double timeout_s) {
  ncclComm_t c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size(), "RCCL: bad communicator handle ", h);
    c = g_comms[h];
    g_comms[h] = nullptr;
  }
  if (c == nullptr) return -1;   // already released (or taken down by rccl_abort_all)
  if (!abort) {
    ncclResult_t r = ncclCommFinalize(c);
    if (r == ncclSuccess || r == ncclInProgress) r = wait_ready(c, timeout_s);
    if (r == ncclSuccess) {
      RCCL_CHECK(ncclCommDestroy(c));
      return 1;
    }
  }
  (void)ncclCommAbort(c);
  return 0;
}

// Handles of the live communicators (the async-error watcher polls these from its own thread).
std::vector<int64_t> rccl_live() {
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<int64_t> out;
  for (size_t i = 0; i < g_comms.size(); ++i)
    if (g_comms[i] != nullptr) out.push_back((int64_t)i);
  return out;
}

// Failure path: abort every live communicator. A rank whose peer died sits in a collective (a kernel spinning on a flag that never comes, or a host
// wait on it); ncclCommAbort from another thread sets the abort flag those kernels poll, which
// drains the stream and lets the process exit instead of wedging the GPU. The table entries are
// cleared under the lock and aborted outside it, so a thread blocked in a collective that holds
// a communicator pointer never deadlocks the abort. Errors are ignored: the process is going
// down and every communicator must get its abort. Returns how many were aborted.
int64_t rccl_abort_all() {
  std::vector<ncclComm_t> victims;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& c : g_comms)
      if (c != nullptr) {
        victims.push_back(c);
        c = nullptr;
      }
  }
  for (ncclComm_t c : victims) (void)ncclCommAbort(c);
  return (int64_t)victims.size();
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(bfly, m) {
  m.def("rccl_unique_id() -> Tensor", &rccl_unique_id);
  m.def("rccl_init(Tensor uid, int nranks, int rank, float timeout_s=600.0) -> int", &rccl_init);
  m.def("rccl_split(int comm, int color, int key, float timeout_s=600.0) -> int", &rccl_split);
  m.def("rccl_set_call_timeout(float timeout_s) -> ()", &rccl_set_call_timeout);
  m.def("rccl_info(int comm) -> int[]", &rccl_info);
  m.def("rccl_version() -> int", &rccl_version);
  m.def("rccl_all_reduce(int comm, Tensor(a!) t, int op=0) -> ()", &rccl_all_reduce);
  m.def("rccl_all_gather(int comm, Tensor inp, Tensor(a!) out) -> ()", &rccl_all_gather);
  m.def("rccl_reduce_scatter(int comm, Tensor inp, Tensor(a!) out, int op=0) -> ()", &rccl_reduce_scatter);
  m.def("rccl_all_to_all(int comm, Tensor inp, Tensor(a!) out) -> ()", &rccl_all_to_all);
  m.def("rccl_broadcast(int comm, Tensor(a!) t, int root) -> ()", &rccl_broadcast);
  m.def("rccl_send(int comm, Tensor t, int peer) -> ()", &rccl_send);
  m.def("rccl_recv(int comm, Tensor(a!) t, int peer) -> ()", &rccl_recv);
  m.def("rccl_group_start() -> ()", &rccl_group_start);
  m.def("rccl_group_end() -> ()", &rccl_group_end);
  m.def("rccl_async_error(int comm) -> int", &rccl_async_error);
  m.def("rccl_release(int comm, bool abort=False, float timeout_s=30.0) -> int", &rccl_release);
  m.def("rccl_live() -> int[]", &rccl_live);
  m.def("rccl_abort_all() -> int", &rccl_abort_all);
}
