// One-shot peer-to-peer all-reduce over xGMI, with an
// optional fused residual-add + RMSNorm epilogue.
//
// Why not RCCL for decode: a Llama-70B TP decode step issues 2 all-reduces per layer of only
// B x hidden x 2 bytes (1 MiB at B=64). RCCL's ring protocol pays several link round trips
// and a kernel of its own per call; on a fully connected xGMI mesh every peer is one hop, so
// the cheapest schedule is: every rank publishes its slice, then reads all 7 peers' slices
// at once (7 links in parallel) and sums locally. One kernel, captured in the decode hipGraph.
//
// Memory: every rank owns ONE uncached device allocation (hipDeviceMallocUncached, so local
// stores are written through and remote readers never hit a stale L2 line) shared with its
// peers through hipIpc handles:
//   [0, 4 KiB)        flags[kArBlocks][8]   peer r stores its epoch into slot [b][r]
//   [4 KiB, 8 KiB)    cnt[kArBlocks]        this rank's per-block epoch counter
//   [8 KiB]           err                   sticky error word (spin timeout)
//   [12 KiB, 16 KiB)  flags2[kArBlocks][8]  second-rendezvous flags (two-shot)
//   [64 KiB, +2*cap)  two data buffers; epoch parity selects one (double buffering)
//   [+2*cap, +4*cap)  two reduced-chunk buffers (two-shot)
//
// Protocol for workgroup b of a grid of G <= kArBlocks workgroups (G is fixed for the life of a
// communicator and equal on every rank, so row r is always owned by block r % G and its epoch
// advances by one per call on every rank; G = kArBlocks, or kArBlocks / world when the ranks
// share one GPU — see launch_custom_allreduce):
//   e = cnt[b] + 1                       (device-resident, so graph replays stay in sync)
//   stage own rows into data[e & 1]; fence(system); barrier
//   thread p < W: store e into flags of peer p at [b][rank]  (release, system scope)
//                 spin until own flags[b][p] >= e             (bounded; sets err on timeout)
//   barrier; acquire fence(system); sum peers in rank order 0..W-1 in f32 (bitwise identical
//   on every rank); cnt[b] = e.
// Double buffering is enough: a rank can only stage call k+1 after every peer arrived at call
// k's barrier, i.e. after every peer finished reading call k-1 (same parity).
//
// TWO-SHOT (reduce-scatter + all-gather, for larger messages at W = 4 / 8): the one-shot read
// pulls the WHOLE message from every peer, S bytes per link. Two-shot splits every row into W
// column chunks; rank p
//   RS: sums chunk p of its block's rows over all ranks (fixed order 0..W-1, f32) and stores
//       the bf16 result in its `red[e & 1]` buffer; fence; flags2[b][p] = e at every peer;
//   AG: waits for flags2[b][*] >= e, then reads chunk q of every row from rank q's `red`
//       (and fuses residual add + RMSNorm exactly as one-shot does).
// Per-link traffic drops to 2S/W (S/4 at W = 8); the price is a second rendezvous. Results are
// bitwise identical to one-shot (same f32 order, same bf16 rounding points). `red` double
// buffering: a rank writes red[(e+2) & 1] only after passing call e+2's first rendezvous, i.e.
// after every peer started call e+2, so every peer finished call e's gather.
#include <string.h>

#include <mutex>

#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

namespace {

constexpr long kArFlagsOff = 0;
constexpr long kArCntOff = 4096;
constexpr long kArErrOff = 8192;
constexpr long kArFlags2Off = 12288;
constexpr int kArThreads = 256;

// Give-up time of a flag wait, in ticks of the 100 MHz constant clock (wall_clock64): a peer
// that is this late is not coming (crashed or hung rank). Wall time, not an iteration count, so
// a rank delayed by host work or by time-slicing (several ranks sharing one GPU) is waited for.
constexpr long long kArSpinTimeoutTicks = 20LL * 100000000LL;   // 20 s

__device__ __forceinline__ void spin_wait(const uint32_t* f, uint32_t e, uint32_t* err, uint32_t* herr) {
  if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= e) return;
  const long long t0 = wall_clock64();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > kArSpinTimeoutTicks) {   // record and give up
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // host-visible copy for the error poller: a plain (vector) store, no host-memory atomic
      if (herr != nullptr) __hip_atomic_store(herr + kHealthCar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// MODE 0: out = sum.  MODE 1: residual = bf16(bf16(sum) + residual); out = rmsnorm(residual) * w
// store epoch e at every peer's flag slot [b][rank] and wait until every peer stored e in ours
template <int W>
__device__ __forceinline__ void rendezvous(const ArPeers& peers, char* my, long off, int b, int rank,
                                           uint32_t e) {
  if (threadIdx.x < W) {
    uint32_t* pf = reinterpret_cast<uint32_t*>(peers.base[threadIdx.x] + off) + b * 8 + rank;
    __hip_atomic_store(pf, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* f = reinterpret_cast<const uint32_t*>(my + off) + b * 8 + threadIdx.x;
    spin_wait(f, e, reinterpret_cast<uint32_t*>(my + kArErrOff), peers.herr);
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

template <int W, int MODE, int NV, bool TWO>
__global__ void __launch_bounds__(kArThreads)
allreduce_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, bf16* __restrict__ residual,
                 const bf16* __restrict__ w, float eps, int rows, int dim, ArPeers peers,
                 int rank, long cap, const float* __restrict__ slabs, int sk) {
  __shared__ uint32_t s_epoch;
  __shared__ float red[16];
  const int b = blockIdx.x, nblk = gridDim.x;
  char* my = peers.base[rank];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(my + kArCntOff);
  if (threadIdx.x == 0) s_epoch = cnt[b] + 1;
  __syncthreads();
  const uint32_t e = s_epoch;
  const long data_off = kArDataOff + (long)(e & 1) * cap;
  const int nvec = dim >> 3;

  // 1. publish this rank's rows. With `slabs` the input is a split-K GEMM's f32 partials
  // [sk][rows][dim]: their reduce (rounded to bf16, exactly what the reduce kernel would
  // have written) is fused into the publish, and the local operand is read back from `mine`.
  bf16* mine = reinterpret_cast<bf16*>(my + data_off);
  const long slab = (long)rows * dim;
  for (int r = b; r < rows; r += nblk) {
    bf16x8* dst = reinterpret_cast<bf16x8*>(mine + (long)r * dim);
    if (slabs != nullptr) {
      for (int c = threadIdx.x; c < nvec; c += kArThreads) {
        const float* sp = slabs + (long)r * dim + c * 8;
        f32x4 lo = *reinterpret_cast<const f32x4*>(sp), hi = *reinterpret_cast<const f32x4*>(sp + 4);
        for (int q = 1; q < sk; ++q) {
          lo += *reinterpret_cast<const f32x4*>(sp + q * slab);
          hi += *reinterpret_cast<const f32x4*>(sp + q * slab + 4);
        }
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(lo[j]);
          o[j + 4] = f2bf(hi[j]);
        }
        dst[c] = o;
      }
    } else {
      const bf16x8* src = reinterpret_cast<const bf16x8*>(in + (long)r * dim);
      for (int c = threadIdx.x; c < nvec; c += kArThreads) dst[c] = src[c];
    }
  }
  const bf16* own = slabs != nullptr ? mine : in;   // this rank's operand for the sum
  __threadfence_system();
  __syncthreads();

  // 2. rendezvous with the peers for this block
  rendezvous<W>(peers, my, kArFlagsOff, b, rank, e);

  // 3. reduce
  const bf16* src[W];
#pragma unroll
  for (int p = 0; p < W; ++p) src[p] = reinterpret_cast<const bf16*>(peers.base[p] + data_off);
  if constexpr (TWO) {
    // 3a. reduce-scatter: this rank's column chunk of the block's rows
    const long red_off = kArDataOff + 2 * cap + (long)(e & 1) * cap;
    const int per = nvec / W, c0 = rank * per;
    bf16* red_mine = reinterpret_cast<bf16*>(my + red_off);
    for (int r = b; r < rows; r += nblk) {
      const long ro = (long)r * dim;
      for (int c = c0 + threadIdx.x; c < c0 + per; c += kArThreads) {
        bf16x8 v[W];
#pragma unroll
        for (int p = 0; p < W; ++p)
          v[p] = p == rank ? reinterpret_cast<const bf16x8*>(own + ro)[c]
                           : reinterpret_cast<const bf16x8*>(src[p] + ro)[c];
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = bf2f(v[0][j]);
#pragma unroll
        for (int p = 1; p < W; ++p)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[p][j]);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
        reinterpret_cast<bf16x8*>(red_mine + ro)[c] = o;
      }
    }
    __threadfence_system();
    __syncthreads();
    rendezvous<W>(peers, my, kArFlags2Off, b, rank, e);
    // 3b. all-gather: chunk q of every row comes from rank q's reduced buffer
#pragma unroll
    for (int p = 0; p < W; ++p) src[p] = reinterpret_cast<const bf16*>(peers.base[p] + red_off);
    for (int r = b; r < rows; r += nblk) {
      const long ro = (long)r * dim;
      if constexpr (MODE == 0) {
        for (int c = threadIdx.x; c < nvec; c += kArThreads)
          reinterpret_cast<bf16x8*>(out + ro)[c] = reinterpret_cast<const bf16x8*>(src[c / per] + ro)[c];
      } else {
        float v[NV][8];
        float ss = 0.f;
        // every remote and local load of the row first: the residual stores below may alias
        // them for the compiler, which would otherwise serialise one xGMI round trip per vector
        bf16x8 xs[NV], rs[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int c = threadIdx.x + i * kArThreads;
          if (c < nvec) {
            xs[i] = reinterpret_cast<const bf16x8*>(src[c / per] + ro)[c];
            rs[i] = reinterpret_cast<const bf16x8*>(residual + ro)[c];
          }
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int c = threadIdx.x + i * kArThreads;
          if (c < nvec) {
            const bf16x8 x = xs[i], rr = rs[i];
            bf16x8 sres;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              sres[j] = f2bf(bf2f(x[j]) + bf2f(rr[j]));
              v[i][j] = bf2f(sres[j]);
              ss += v[i][j] * v[i][j];
            }
            reinterpret_cast<bf16x8*>(residual + ro)[c] = sres;
          }
        }
        ss = block_sum(ss, red);
        const float inv = rsqrtf(ss / (float)dim + eps);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int c = threadIdx.x + i * kArThreads;
          if (c < nvec) {
            const bf16x8 g = reinterpret_cast<const bf16x8*>(w)[c];
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
            reinterpret_cast<bf16x8*>(out + ro)[c] = o;
          }
        }
      }
    }
    if (threadIdx.x == 0) cnt[b] = e;
    return;
  }
  for (int r = b; r < rows; r += nblk) {
    const long ro = (long)r * dim;
    if constexpr (MODE == 0) {
      // U vectors per thread per round, all peers' loads issued before the first store (the
      // stores may alias them for the compiler: one xGMI round trip per round, not per vector).
      // 8 loads per thread in flight at most: the VGPR budget keeps 8 ranks' grids co-resident
      // when ranks share a GPU (the flag rendezvous needs every peer's workgroup running).
      constexpr int U = W >= 8 ? 1 : 8 / W;
      for (int c0 = threadIdx.x; c0 < nvec; c0 += U * kArThreads) {
        bf16x8 v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int c = c0 + u * kArThreads;
          if (c < nvec) {
#pragma unroll
            for (int p = 0; p < W; ++p)
              v[u][p] = p == rank ? reinterpret_cast<const bf16x8*>(own + ro)[c]
                                  : reinterpret_cast<const bf16x8*>(src[p] + ro)[c];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int c = c0 + u * kArThreads;
          if (c < nvec) {
            float acc[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = bf2f(v[u][0][j]);
#pragma unroll
            for (int p = 1; p < W; ++p)
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[u][p][j]);
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
            reinterpret_cast<bf16x8*>(out + ro)[c] = o;
          }
        }
      }
    } else {
      float v[NV][8];
      float ss = 0.f;
      // the peers' vectors (and the residual) of CH register rows are loaded before the first
      // residual store, which may alias them for the compiler: one xGMI round trip per chunk
      // instead of per vector (at most 16 loads per thread in flight: see MODE 0)
      constexpr int CH = (16 / W) < NV ? (16 / W) : NV;
#pragma unroll
      for (int i0 = 0; i0 < NV; i0 += CH) {
      bf16x8 xs[CH][W], rs[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int c = threadIdx.x + (i0 + u) * kArThreads;
        if (c < nvec) {
#pragma unroll
          for (int p = 0; p < W; ++p)
            xs[u][p] = p == rank ? reinterpret_cast<const bf16x8*>(own + ro)[c]
                                 : reinterpret_cast<const bf16x8*>(src[p] + ro)[c];
          rs[u] = reinterpret_cast<const bf16x8*>(residual + ro)[c];
        }
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int i = i0 + u;
        const int c = threadIdx.x + i * kArThreads;
        if (c < nvec) {
          const bf16x8* x = xs[u];
          const bf16x8 rr = rs[u];
          bf16x8 s;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float a = bf2f(x[0][j]);
#pragma unroll
            for (int p = 1; p < W; ++p) a += bf2f(x[p][j]);
            // same roundings as all-reduce -> rms_norm(residual=...): sum to bf16, then add
            s[j] = f2bf(bf2f(f2bf(a)) + bf2f(rr[j]));
            v[i][j] = bf2f(s[j]);
            ss += v[i][j] * v[i][j];
          }
          reinterpret_cast<bf16x8*>(residual + ro)[c] = s;
        }
      }
      }
      ss = block_sum(ss, red);
      const float inv = rsqrtf(ss / (float)dim + eps);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = threadIdx.x + i * kArThreads;
        if (c < nvec) {
          const bf16x8 g = reinterpret_cast<const bf16x8*>(w)[c];
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
          reinterpret_cast<bf16x8*>(out + ro)[c] = o;
        }
      }
    }
  }
  if (threadIdx.x == 0) cnt[b] = e;
}

template <int W, bool TWO>
int launch_w(const bf16* in, bf16* out, bf16* residual, const bf16* w, float eps, int rows,
             int dim, const ArPeers& peers, int rank, long cap, const float* slabs, int sk,
             int blocks, hipStream_t stream) {
  const dim3 grid(blocks), block(kArThreads);
  if (residual == nullptr) {
    allreduce_kernel<W, 0, 1, TWO><<<grid, block, 0, stream>>>(in, out, nullptr, nullptr, 0.f, rows,
                                                               dim, peers, rank, cap, slabs, sk);
    return 0;
  }
  const int nv = (dim / 8 + kArThreads - 1) / kArThreads;
  // register rows per thread: 1, 2, 4 or 8 vectors of 8 (dim up to 16384)
  const int nvp = nv <= 1 ? 1 : nv <= 2 ? 2 : nv <= 4 ? 4 : nv <= 8 ? 8 : 0;
#define AR_NV(N)                                                                               \
  case N:                                                                                      \
    allreduce_kernel<W, 1, N, TWO><<<grid, block, 0, stream>>>(in, out, residual, w, eps, rows, \
                                                               dim, peers, rank, cap, slabs, sk); \
    return 0;
  switch (nvp) {
    AR_NV(1) AR_NV(2) AR_NV(4) AR_NV(8)
    default: return -1;
  }
#undef AR_NV
}

template <int W>
int launch_mode(bool two, const bf16* in, bf16* out, bf16* residual, const bf16* w, float eps,
                int rows, int dim, const ArPeers& peers, int rank, long cap, const float* slabs,
                int sk, int blocks, hipStream_t stream) {
  if (two) return launch_w<W, true>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, blocks, stream);
  return launch_w<W, false>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, blocks, stream);
}

}  // namespace

int launch_custom_allreduce(const bf16* in, bf16* out, bf16* residual, const bf16* w, float eps,
                            int rows, int dim, const ArPeers& peers, int world, int rank,
                            long cap, hipStream_t stream, const float* slabs, int sk, bool two_shot,
                            int blocks) {
  if (dim % 8 != 0 || dim > 16384 || rows < 0) return -2;
  if (blocks < 1 || blocks > kArBlocks) return -8;
  if (slabs != nullptr && sk < 1) return -6;
  if ((long)rows * dim * 2 > cap) return -3;
  if (rank < 0 || rank >= world) return -4;
  if (two_shot && (dim / 8) % world != 0) return -7;   // column chunks of whole 16-B vectors
  switch (world) {
    case 2: return launch_mode<2>(two_shot, in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, blocks, stream);
    case 4: return launch_mode<4>(two_shot, in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, blocks, stream);
    case 8: return launch_mode<8>(two_shot, in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, blocks, stream);
    default: return -5;
  }
}

// ---- buffer management (host) ----------------------------------------------------------

void* car_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  return p;
}

void car_free(void* p) { (void)hipFree(p); }

int car_ipc_handle(void* p, unsigned char* out64) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) return -1;
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t size");
  memcpy(out64, &h, sizeof(h));
  return 0;
}

void* car_ipc_open(const unsigned char* h64) {
  hipIpcMemHandle_t h;
  memcpy(&h, h64, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  return p;
}

void car_ipc_close(void* p) { (void)hipIpcCloseMemHandle(p); }

int car_clear_error(void* base) {
  return hipMemset(static_cast<char*>(base) + kArErrOff, 0, 4) == hipSuccess ? 0 : -1;
}

namespace {
std::mutex g_health_mu;
uint32_t* g_health_host = nullptr;   // pinned, coherent, mapped into every device
uint32_t* g_health_dev = nullptr;
}  // namespace

uint32_t* health_words_device() {
  std::lock_guard<std::mutex> lk(g_health_mu);
  if (g_health_dev == nullptr) {
    void* h = nullptr;
    if (hipHostMalloc(&h, kHealthWords * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent |
                                                               hipHostMallocPortable) != hipSuccess)
      return nullptr;
    memset(h, 0, kHealthWords * sizeof(uint32_t));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return nullptr;
    }
    g_health_host = static_cast<uint32_t*>(h);
    g_health_dev = static_cast<uint32_t*>(d);
  }
  return g_health_dev;
}

uint32_t health_word(int i) {
  std::lock_guard<std::mutex> lk(g_health_mu);
  if (g_health_host == nullptr || i < 0 || i >= kHealthWords) return 0;
  return reinterpret_cast<volatile uint32_t*>(g_health_host)[i];
}

void health_clear(int word) {
  std::lock_guard<std::mutex> lk(g_health_mu);
  if (g_health_host == nullptr) return;
  for (int i = 0; i < kHealthWords; ++i)
    if (word < 0 || i == word) reinterpret_cast<volatile uint32_t*>(g_health_host)[i] = 0;
}

int car_error(const void* base) {
  uint32_t e = 0;
  if (hipMemcpy(&e, static_cast<const char*>(base) + kArErrOff, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (int)e;
}

}  // namespace bfly
