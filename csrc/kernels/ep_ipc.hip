// Byte-minimal expert-parallel token dispatch / return over peer IPC mappings (xGMI), for
// the decode MoE layer.
//
// The all-to-all form (transformer._moe_alltoall_fixed over RCCL) moves ep x cap rows each way
// per layer whatever the routing. Here every rank owns one uncached device buffer (the custom
// all-reduce's allocator, so remote stores are written through and local reads see them),
// mapped by every EP peer through hipIpc handles:
//   [0, 64 KiB)  control: cur epoch, arrival counters, error word, per-source dispatch and
//                return flags, per-source row counts, byte statistics
//   x    [ep][capmax][H]  bf16   rows source s routed to this rank, at [s][pos]
//   ids  [ep][capmax][K]  int32  their top-k expert ids local to this rank (-1 elsewhere /
//                                empty row)
//   w    [ep][capmax][K]  f32    their gate weights
//   back [ep][capmax][H]  bf16   partial outputs expert rank d returned for this rank's
//                                tokens, at [d][pos]
// Per MoE layer and rank:
//   dispatch  token t goes once to each rank d owning one of its top-k experts: ONE row store
//             into d's x[me][pos] (pos = tokens before t bound for d: stable, cap >= T, no
//             overflow), its ids / weights, empty-row markers for the rest of the block, the
//             row count; the last workgroup to arrive raises flag_d[me] at every peer.
//   wait      spin until every source's flag_d reached this epoch.
//   (local routed-rows expert FFN on the x / ids / w views: ops.moe_sparse_ffn)
//   return    the expert rank stores only the count[s] rows each source sent back into s's
//             back[me][pos]; the last workgroup raises flag_r[me] at every source.
//   combine   spin on flag_r, then out[t] = sum over the ranks t was sent to of back[d][pos]
//             (f32, fixed d order: bitwise the all-to-all path's ep_combine).
// Link bytes: only routed rows (plus K ids / weights each) travel, once each way.
// Single buffering is safe: a rank issues dispatch e+1 only after its combine e saw every
// peer's return e, which every peer issues after its FFN e consumed x / ids / w; and expert d
// writes back[] for call e+1 only after source s's dispatch e+1, issued after s's combine e
// read back[]. So every view has a fixed address: the layer replays inside the decode hipGraph.
// Flags hold monotonically increasing epochs (device-resident `cur`, so replays stay in step);
// a wait that outlives kEpSpinTimeoutTicks sets the sticky error word and gives up.
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

namespace {

constexpr long kEpCur = 0, kEpArriveD = 64, kEpArriveR = 128, kEpErr = 192;
constexpr long kEpFlagsD = 256, kEpFlagsR = 512, kEpCounts = 768, kEpStats = 1024;
constexpr long kEpTotals = 2048;   // prefill dispatch: this rank's per-destination row totals
constexpr int kEpThreads = 256;
constexpr long long kEpSpinTimeoutTicks = 20LL * 100000000LL;   // 20 s of the 100 MHz clock
constexpr int kEpSpinCombineMaxRows = 256;   // combines of more rows wait in a separate one-WG kernel

__device__ __forceinline__ uint32_t* ep_word(char* base, long off) {
  return reinterpret_cast<uint32_t*>(base + off);
}

__device__ __forceinline__ void ep_spin(const uint32_t* f, uint32_t e, uint32_t* err, uint32_t* herr) {
  if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= e) return;
  const long long t0 = wall_clock64();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > kEpSpinTimeoutTicks) {
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // host-visible copy for the error poller (plain vector store into mapped host memory)
      if (herr != nullptr) __hip_atomic_store(herr + kHealthEp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// Last-arriver of a grid: every block calls this after its stores (fenced at system scope);
// returns true in exactly one block, after every other block's stores are visible, with the
// counter re-armed at zero for the next call.
__device__ __forceinline__ bool ep_last_block(char* my, long counter_off) {
  __shared__ int s_last;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ep_word(my, counter_off), 1u, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_SYSTEM);
    s_last = old == gridDim.x - 1;
    if (s_last) __hip_atomic_store(ep_word(my, counter_off), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return s_last;
}

template <int EP>
__device__ __forceinline__ void ep_ipc_hits(const int* ids, int t, int K, int El, const int* slots, bool (&h)[EP]) {
#pragma unroll
  for (int d = 0; d < EP; ++d) h[d] = false;
  if (slots != nullptr && slots[t] < 0) return;   // graph padding row: routes nowhere
  for (int j = 0; j < K; ++j) {
    const int e = ids[t * K + j];
    if (e >= 0) {
      const int d = e / El;
#pragma unroll
      for (int q = 0; q < EP; ++q) h[q] |= (q == d);
    }
  }
}

// grid = capmax workgroups (capmax >= T); block b owns token b and empty-row slot b of every
// destination block
template <int EP>
__global__ void __launch_bounds__(kEpThreads)
ep_ipc_dispatch_kernel(const bf16* __restrict__ x, const int* __restrict__ ids, const float* __restrict__ w,
                       const int* __restrict__ slots, int T, int K, int H, int El, int capmax, ArPeers peers,
                       int rank, EpLayout L, int* __restrict__ slot_out) {
  __shared__ int red[2][EP][4];
  __shared__ uint32_t s_e;
  char* my = peers.base[rank];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_e = __hip_atomic_load(ep_word(my, kEpCur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  int before[EP], total[EP];
#pragma unroll
  for (int d = 0; d < EP; ++d) before[d] = total[d] = 0;
  for (int t = tid; t < T; t += kEpThreads) {
    bool h[EP];
    ep_ipc_hits<EP>(ids, t, K, El, slots, h);
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      total[d] += h[d];
      before[d] += (h[d] && t < b);
    }
  }
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    const float tb = wave_sum((float)before[d]), tt = wave_sum((float)total[d]);
    if (lane == 0) { red[0][d][wv] = (int)tb; red[1][d][wv] = (int)tt; }
  }
  __syncthreads();
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    before[d] = red[0][d][0] + red[0][d][1] + red[0][d][2] + red[0][d][3];
    total[d] = red[1][d][0] + red[1][d][1] + red[1][d][2] + red[1][d][3];
  }
  const uint32_t e = s_e;
  if (b < T) {
    bool h[EP];
    ep_ipc_hits<EP>(ids, b, K, El, slots, h);
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      if (tid == 0) slot_out[b * EP + d] = h[d] ? before[d] : -1;
      if (!h[d]) continue;
      const long row = (long)rank * capmax + before[d];
      char* pd = peers.base[d];
      const bf16x8* src = reinterpret_cast<const bf16x8*>(x + (long)b * H);
      bf16x8* dst = reinterpret_cast<bf16x8*>(pd + L.x) + row * (H / 8);
      for (int c = tid; c < H / 8; c += kEpThreads) dst[c] = src[c];
      if (tid < K) {
        const int ex = ids[b * K + tid];
        const bool mine = ex >= 0 && ex / El == d;
        reinterpret_cast<int*>(pd + L.ids)[row * K + tid] = mine ? ex : -1;
        reinterpret_cast<float*>(pd + L.w)[row * K + tid] = mine ? w[b * K + tid] : 0.f;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    if (b >= total[d] && tid < K) {       // empty row b of this source's block at d
      const long row = (long)rank * capmax + b;
      reinterpret_cast<int*>(peers.base[d] + L.ids)[row * K + tid] = -1;
      reinterpret_cast<float*>(peers.base[d] + L.w)[row * K + tid] = 0.f;
    }
  }
  if (b == 0 && tid == 0) {
    long remote = 0;
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      __hip_atomic_store(ep_word(peers.base[d], kEpCounts) + rank, (uint32_t)total[d], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      if (d != rank) remote += total[d];
    }
    reinterpret_cast<unsigned long long*>(my + kEpStats)[0] += (unsigned long long)remote;
  }
  if (ep_last_block(my, kEpArriveD)) {
    if (tid == 0) __hip_atomic_store(ep_word(my, kEpCur), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < EP)
      __hip_atomic_store(ep_word(peers.base[tid], kEpFlagsD) + rank, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int EP>
__global__ void __launch_bounds__(64)
ep_ipc_wait_kernel(ArPeers peers, int rank) {
  char* my = peers.base[rank];
  const uint32_t e = __hip_atomic_load(ep_word(my, kEpCur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < EP) ep_spin(ep_word(my, kEpFlagsD) + threadIdx.x, e, ep_word(my, kEpErr), peers.herr);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// grid = capmax workgroups: block b returns row b of every source block that holds >= b+1 rows
template <int EP>
__global__ void __launch_bounds__(kEpThreads)
ep_ipc_return_kernel(const bf16* __restrict__ y, int H, int capmax, ArPeers peers, int rank, EpLayout L) {
  char* my = peers.base[rank];
  const uint32_t e = __hip_atomic_load(ep_word(my, kEpCur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int b = blockIdx.x, tid = threadIdx.x;
  long remote = 0;
#pragma unroll
  for (int s = 0; s < EP; ++s) {
    const int n = (int)__hip_atomic_load(ep_word(my, kEpCounts) + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (s != rank) remote += n;
    if (b >= n) continue;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(y + ((long)s * capmax + b) * H);
    bf16x8* dst = reinterpret_cast<bf16x8*>(peers.base[s] + L.back) + ((long)rank * capmax + b) * (H / 8);
    for (int c = tid; c < H / 8; c += kEpThreads) dst[c] = src[c];
  }
  if (b == 0 && tid == 0) reinterpret_cast<unsigned long long*>(my + kEpStats)[1] += (unsigned long long)remote;
  if (ep_last_block(my, kEpArriveR)) {
    if (tid < EP)
      __hip_atomic_store(ep_word(peers.base[tid], kEpFlagsR) + rank, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// grid = max(T, 1) workgroups: out[t] = sum_d back[d][slot[t][d]] over the ranks t was sent
// to. A rank with no tokens (T == 0: EP-idle step) still runs one workgroup, whose only job is
// the flag_r wait: without it the rank's next dispatch could overwrite peers' x / ids / counts
// blocks before they finished this layer's FFN (the single-buffering invariant above).
// SPIN = false: a one-workgroup ep_ipc_wait_return_kernel already waited (prefill-sized T:
// thousands of workgroups spinning would only hold CUs a co-resident peer kernel may need).
template <int EP, bool SPIN>
__global__ void __launch_bounds__(kEpThreads)
ep_ipc_combine_kernel(const int* __restrict__ slot, int T, int H, int capmax, ArPeers peers, int rank, EpLayout L,
                      bf16* __restrict__ out) {
  char* my = peers.base[rank];
  if constexpr (SPIN) {
    const uint32_t e = __hip_atomic_load(ep_word(my, kEpCur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < EP) ep_spin(ep_word(my, kEpFlagsR) + threadIdx.x, e, ep_word(my, kEpErr), peers.herr);
    __syncthreads();
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const long t = blockIdx.x;
  if (t >= T) return;
  const bf16* back = reinterpret_cast<const bf16*>(my + L.back);
  int sl[EP];
#pragma unroll
  for (int d = 0; d < EP; ++d) sl[d] = slot[t * EP + d];
  for (int c = threadIdx.x; c < H / 8; c += kEpThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      if (sl[d] < 0) continue;
      const bf16x8 v = reinterpret_cast<const bf16x8*>(back + ((long)d * capmax + sl[d]) * H)[c];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += bf2f(v[q]);
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    reinterpret_cast<bf16x8*>(out + t * H)[c] = o;
  }
}

// one workgroup: wait until every expert rank returned this epoch's rows (flag_r)
template <int EP>
__global__ void __launch_bounds__(64)
ep_ipc_wait_return_kernel(ArPeers peers, int rank) {
  char* my = peers.base[rank];
  const uint32_t e = __hip_atomic_load(ep_word(my, kEpCur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < EP) ep_spin(ep_word(my, kEpFlagsR) + threadIdx.x, e, ep_word(my, kEpErr), peers.herr);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// ---- prefill-sized dispatch (T up to capmax: thousands of tokens) ----------------------
// The decode dispatch above recomputes every prefix count in every workgroup (O(T^2): fine
// for a 64-row batch, not for a 16k-token prefill). Here one 1024-thread workgroup routes all
// tokens with an exclusive scan: each thread counts its contiguous token chunk per destination,
// the counts are scanned across the workgroup (wave shuffles, then the 16 wave totals), and a
// second pass over the chunk writes slot[t][d] = rows of d before t (-1: not sent). Stable and
// deterministic: the same slots as the decode dispatch.
constexpr int kEpRouteThreads = 1024;

template <int EP>
__global__ void __launch_bounds__(kEpRouteThreads)
ep_route_kernel(const int* __restrict__ ids, int T, int K, int El, int* __restrict__ slot_out,
                int* __restrict__ totals) {
  __shared__ int wsum[EP][kEpRouteThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int chunk = (T + kEpRouteThreads - 1) / kEpRouteThreads;
  const int t0 = min(T, tid * chunk), t1 = min(T, t0 + chunk);
  int cnt[EP];
#pragma unroll
  for (int d = 0; d < EP; ++d) cnt[d] = 0;
  for (int t = t0; t < t1; ++t) {
    bool h[EP];
    ep_ipc_hits<EP>(ids, t, K, El, nullptr, h);
#pragma unroll
    for (int d = 0; d < EP; ++d) cnt[d] += h[d];
  }
  int excl[EP];
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    int v = cnt[d];                                  // inclusive scan inside the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    excl[d] = v - cnt[d];
    if (lane == 63) wsum[d][wv] = v;
  }
  __syncthreads();
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    int before = 0, total = 0;
    for (int w = 0; w < kEpRouteThreads / 64; ++w) {
      before += w < wv ? wsum[d][w] : 0;
      total += wsum[d][w];
    }
    excl[d] += before;
    if (tid == 0) totals[d] = total;
  }
  for (int t = t0; t < t1; ++t) {
    bool h[EP];
    ep_ipc_hits<EP>(ids, t, K, El, nullptr, h);
#pragma unroll
    for (int d = 0; d < EP; ++d) slot_out[t * EP + d] = h[d] ? excl[d]++ : -1;
  }
}

// grid = max(T, 1) workgroups: block t stores row t (ids / weights local to each destination)
// once into every owning rank's block at its routed position; the last arriver publishes this
// rank's row count at every destination and raises the dispatch flags (as the decode dispatch).
template <int EP>
__global__ void __launch_bounds__(kEpThreads)
ep_ipc_scatter_kernel(const bf16* __restrict__ x, const int* __restrict__ ids, const float* __restrict__ w,
                      int T, int K, int H, int El, int capmax, ArPeers peers, int rank, EpLayout L,
                      const int* __restrict__ slot) {
  __shared__ uint32_t s_e;
  char* my = peers.base[rank];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_e = __hip_atomic_load(ep_word(my, kEpCur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint32_t e = s_e;
  if (b < T) {
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      const int pos = slot[b * EP + d];
      if (pos < 0) continue;
      const long row = (long)rank * capmax + pos;
      char* pd = peers.base[d];
      const bf16x8* src = reinterpret_cast<const bf16x8*>(x + (long)b * H);
      bf16x8* dst = reinterpret_cast<bf16x8*>(pd + L.x) + row * (H / 8);
      for (int c = tid; c < H / 8; c += kEpThreads) dst[c] = src[c];
      if (tid < K) {
        const int ex = ids[b * K + tid];
        const bool mine = ex >= 0 && ex / El == d;
        reinterpret_cast<int*>(pd + L.ids)[row * K + tid] = mine ? ex : -1;
        reinterpret_cast<float*>(pd + L.w)[row * K + tid] = mine ? w[b * K + tid] : 0.f;
      }
    }
  }
  if (ep_last_block(my, kEpArriveD)) {
    if (tid == 0) {
      const int* totals = reinterpret_cast<const int*>(my + kEpTotals);
      long remote = 0;
      for (int d = 0; d < EP; ++d) {
        __hip_atomic_store(ep_word(peers.base[d], kEpCounts) + rank, (uint32_t)totals[d], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        if (d != rank) remote += totals[d];
      }
      reinterpret_cast<unsigned long long*>(my + kEpStats)[0] += (unsigned long long)remote;
      __hip_atomic_store(ep_word(my, kEpCur), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __threadfence_system();     // the counts before the flags
    __syncthreads();
    if (tid < EP)
      __hip_atomic_store(ep_word(peers.base[tid], kEpFlagsD) + rank, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

EpLayout ep_ipc_layout(int ep, int capmax, int H, int K) {
  auto al = [](long v) { return (v + 255) & ~255L; };
  const long rows = (long)ep * capmax;
  EpLayout L;
  L.x = kEpHeaderBytes;
  L.ids = al(L.x + rows * H * 2);
  L.w = al(L.ids + rows * K * 4);
  L.back = al(L.w + rows * K * 4);
  L.total = al(L.back + rows * H * 2);
  return L;
}

#define EP_SWITCH(EPV, CALL) \
  switch (EPV) {             \
    case 2: CALL(2); break;  \
    case 4: CALL(4); break;  \
    case 8: CALL(8); break;  \
    default: return -2;      \
  }

int launch_ep_ipc_dispatch(const bf16* x, const int* ids, const float* w, const int* slots, int T, int K,
                           int H, int El, int ep, int capmax, const ArPeers& peers, int rank, int* slot_out,
                           hipStream_t stream) {
  if (H % 8 != 0 || K > kEpThreads || capmax < T || capmax <= 0 || El <= 0 || rank < 0 || rank >= ep) return -1;
  const EpLayout L = ep_ipc_layout(ep, capmax, H, K);
#define EP_DISPATCH(N)                                                                             \
  ep_ipc_dispatch_kernel<N><<<capmax, kEpThreads, 0, stream>>>(x, ids, w, slots, T, K, H, El, capmax, \
                                                               peers, rank, L, slot_out)
  EP_SWITCH(ep, EP_DISPATCH)
#undef EP_DISPATCH
  return 0;
}

int launch_ep_ipc_dispatch_prefill(const bf16* x, const int* ids, const float* w, int T, int K, int H, int El,
                                   int ep, int capmax, const ArPeers& peers, int rank, int* slot_out,
                                   hipStream_t stream) {
  if (H % 8 != 0 || K > kEpThreads || T < 0 || capmax < T || capmax <= 0 || El <= 0 || rank < 0 || rank >= ep)
    return -1;
  const EpLayout L = ep_ipc_layout(ep, capmax, H, K);
  int* totals = reinterpret_cast<int*>(peers.base[rank] + kEpTotals);
#define EP_PREFILL(N)                                                                                  \
  do {                                                                                                 \
    ep_route_kernel<N><<<1, kEpRouteThreads, 0, stream>>>(ids, T, K, El, slot_out, totals);            \
    ep_ipc_scatter_kernel<N><<<T > 0 ? T : 1, kEpThreads, 0, stream>>>(x, ids, w, T, K, H, El, capmax,  \
                                                                        peers, rank, L, slot_out);     \
  } while (0)
  EP_SWITCH(ep, EP_PREFILL)
#undef EP_PREFILL
  return 0;
}

long ep_ipc_counts_offset() { return kEpCounts; }

int launch_ep_ipc_wait(const ArPeers& peers, int ep, int rank, hipStream_t stream) {
  if (rank < 0 || rank >= ep) return -1;
#define EP_WAIT(N) ep_ipc_wait_kernel<N><<<1, 64, 0, stream>>>(peers, rank)
  EP_SWITCH(ep, EP_WAIT)
#undef EP_WAIT
  return 0;
}

int launch_ep_ipc_return(const bf16* y, int H, int K, int ep, int capmax, const ArPeers& peers, int rank,
                         hipStream_t stream) {
  if (H % 8 != 0 || capmax <= 0 || rank < 0 || rank >= ep) return -1;
  const EpLayout L = ep_ipc_layout(ep, capmax, H, K);
#define EP_RETURN(N) ep_ipc_return_kernel<N><<<capmax, kEpThreads, 0, stream>>>(y, H, capmax, peers, rank, L)
  EP_SWITCH(ep, EP_RETURN)
#undef EP_RETURN
  return 0;
}

int launch_ep_ipc_combine(const int* slot, int T, int H, int K, int ep, int capmax, const ArPeers& peers,
                          int rank, bf16* out, hipStream_t stream) {
  if (H % 8 != 0 || capmax <= 0 || rank < 0 || rank >= ep) return -1;
  if (T < 0) return -1;
  const EpLayout L = ep_ipc_layout(ep, capmax, H, K);
  // decode-sized batches wait inside the combine (one launch); larger ones wait in one
  // workgroup first, so no spinning workgroup holds a CU a co-resident peer kernel needs
  const bool sep = T > kEpSpinCombineMaxRows;
#define EP_COMBINE(N)                                                                                      \
  do {                                                                                                     \
    if (sep) {                                                                                             \
      ep_ipc_wait_return_kernel<N><<<1, 64, 0, stream>>>(peers, rank);                                     \
      ep_ipc_combine_kernel<N, false><<<T, kEpThreads, 0, stream>>>(slot, T, H, capmax, peers, rank, L, out); \
    } else {                                                                                               \
      ep_ipc_combine_kernel<N, true><<<T > 0 ? T : 1, kEpThreads, 0, stream>>>(slot, T, H, capmax, peers,  \
                                                                             rank, L, out);                \
    }                                                                                                      \
  } while (0)
  EP_SWITCH(ep, EP_COMBINE)
#undef EP_COMBINE
  return 0;
}

#undef EP_SWITCH

// [rows dispatched to other ranks, rows returned to other ranks] since the buffer was created
int ep_ipc_stats(const void* base, long long* out2) {
  return hipMemcpy(out2, static_cast<const char*>(base) + kEpStats, 16, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

int ep_ipc_error(const void* base) {
  uint32_t e = 0;
  if (hipMemcpy(&e, static_cast<const char*>(base) + kEpErr, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)e;
}

}  // namespace bfly
