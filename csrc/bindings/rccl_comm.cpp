// Native RCCL communicator: the rank's communicators as RCCL objects
// owned here rather than torch ProcessGroups, so the data-path collectives are ONE
// stream-ordered RCCL call each (no work objects, no watchdog events, no allocator record
// streams) and capture into the decode hipGraph like the kernels around them.
//
//   rccl_unique_id()                       rank 0 creates the id; the caller ships its 128 bytes
//                                          to the other ranks over the control plane
//   rccl_init(uid, nranks, rank)           ncclCommInitRank on the current device -> handle
//   rccl_split(h, color, key)              ncclCommSplit: one call per mesh axis (tp / pp / dp)
//                                          from the world communicator; color < 0 -> no group
//   rccl_all_reduce / all_gather / reduce_scatter / all_to_all / broadcast / send / recv
//                                          on torch's current stream, in place or into `out`
//   rccl_group_start / rccl_group_end      batch point-to-point calls (PP fan-out)
//   rccl_async_error(h)                    ncclCommGetAsyncError, polled by the health monitor
//   rccl_release(h, abort)                 ncclCommAbort / ncclCommDestroy of one communicator
//   rccl_live() / rccl_abort_all()         live handles (polled by the async-error watcher);
//                                          abort every one on the failure path
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

#include <cstring>
#include <mutex>
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

int64_t rccl_init(const Tensor& uid, int64_t nranks, int64_t rank) {
  TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte && uid.numel() == NCCL_UNIQUE_ID_BYTES,
              "rccl_init: uid must be the 128-byte CPU tensor from rccl_unique_id");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "rccl_init: rank out of range");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  RCCL_CHECK(ncclCommInitRank(&c, (int)nranks, id, (int)rank));   // on the current device
  return add_comm(c);
}

int64_t rccl_split(int64_t h, int64_t color, int64_t key) {
  ncclComm_t c = comm_of(h), out = nullptr;
  RCCL_CHECK(ncclCommSplit(c, color < 0 ? NCCL_SPLIT_NOCOLOR : (int)color, (int)key, &out, nullptr));
  return out == nullptr ? -1 : add_comm(out);
}

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
  RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), op_of(op), comm_of(h), cur_stream()));
}

void rccl_all_gather(int64_t h, const Tensor& inp, Tensor& out) {
  check_dev(inp, "input");
  check_dev(out, "output");
  ncclComm_t c = comm_of(h);
  int n = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  TORCH_CHECK(out.numel() == inp.numel() * n && out.scalar_type() == inp.scalar_type(), "rccl_all_gather: out size");
  c10::DeviceGuard g(inp.device());
  RCCL_CHECK(ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), dtype_of(inp), c, cur_stream()));
}

void rccl_reduce_scatter(int64_t h, const Tensor& inp, Tensor& out, int64_t op) {
  check_dev(inp, "input");
  check_dev(out, "output");
  ncclComm_t c = comm_of(h);
  int n = 0;
  RCCL_CHECK(ncclCommCount(c, &n));
  TORCH_CHECK(inp.numel() == out.numel() * n && out.scalar_type() == inp.scalar_type(), "rccl_reduce_scatter: sizes");
  c10::DeviceGuard g(inp.device());
  RCCL_CHECK(ncclReduceScatter(inp.data_ptr(), out.data_ptr(), out.numel(), dtype_of(inp), op_of(op), c, cur_stream()));
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
  RCCL_CHECK(ncclAllToAll(inp.data_ptr(), out.data_ptr(), inp.numel() / n, dtype_of(inp), c, cur_stream()));
}

void rccl_broadcast(int64_t h, Tensor& t, int64_t root) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  RCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), (int)root, comm_of(h), cur_stream()));
}

void rccl_send(int64_t h, const Tensor& t, int64_t peer) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  RCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), dtype_of(t), (int)peer, comm_of(h), cur_stream()));
}

void rccl_recv(int64_t h, Tensor& t, int64_t peer) {
  check_dev(t, "tensor");
  c10::DeviceGuard g(t.device());
  RCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), dtype_of(t), (int)peer, comm_of(h), cur_stream()));
}

void rccl_group_start() { RCCL_CHECK(ncclGroupStart()); }
void rccl_group_end() { RCCL_CHECK(ncclGroupEnd()); }

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

void rccl_release(int64_t h, bool abort) {
  ncclComm_t c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size(), "RCCL: bad communicator handle ", h);
    c = g_comms[h];
    g_comms[h] = nullptr;
  }
  if (c == nullptr) return;   // already released (or taken down by rccl_abort_all)
  RCCL_CHECK(abort ? ncclCommAbort(c) : ncclCommDestroy(c));
}

// Handles of the live communicators (the async-error watcher polls these from its own thread).
std::vector<int64_t> rccl_live() {
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<int64_t> out;
  for (size_t i = 0; i < g_comms.size(); ++i)
    if (g_comms[i] != nullptr) out.push_back((int64_t)i);
  return out;
}

// Failure path: abort every live communicator. Communicators are created blocking, so a rank
// whose peer died sits in a collective (a kernel spinning on a flag that never comes, or a host
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
  m.def("rccl_init(Tensor uid, int nranks, int rank) -> int", &rccl_init);
  m.def("rccl_split(int comm, int color, int key) -> int", &rccl_split);
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
  m.def("rccl_release(int comm, bool abort=False) -> ()", &rccl_release);
  m.def("rccl_live() -> int[]", &rccl_live);
  m.def("rccl_abort_all() -> int", &rccl_abort_all);
}
