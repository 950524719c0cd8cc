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
//   [64 KiB, +2*cap)  two data buffers; epoch parity selects one (double buffering)
//
// Protocol for workgroup b (grid is ALWAYS kArBlocks, so row r is always owned by block
// r % kArBlocks and its epoch advances by one per call on every rank):
//   e = cnt[b] + 1                       (device-resident, so graph replays stay in sync)
//   stage own rows into data[e & 1]; fence(system); barrier
//   thread p < W: store e into flags of peer p at [b][rank]  (release, system scope)
//                 spin until own flags[b][p] >= e             (bounded; sets err on timeout)
//   barrier; acquire fence(system); sum peers in rank order 0..W-1 in f32 (bitwise identical
//   on every rank); cnt[b] = e.
// Double buffering is enough: a rank can only stage call k+1 after every peer arrived at call
// k's barrier, i.e. after every peer finished reading call k-1 (same parity).
#include <string.h>

#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

namespace {

constexpr long kArFlagsOff = 0;
constexpr long kArCntOff = 4096;
constexpr long kArErrOff = 8192;
constexpr int kArThreads = 256;

__device__ __forceinline__ void spin_wait(const uint32_t* f, uint32_t e, uint32_t* err) {
  long it = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
    __builtin_amdgcn_s_sleep(2);
    if (++it > (1L << 26)) {   // ~seconds: a peer never arrived. Record and give up.
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// MODE 0: out = sum.  MODE 1: residual = bf16(bf16(sum) + residual); out = rmsnorm(residual) * w
template <int W, int MODE, int NV>
__global__ void __launch_bounds__(kArThreads)
allreduce_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, bf16* __restrict__ residual,
                 const bf16* __restrict__ w, float eps, int rows, int dim, ArPeers peers,
                 int rank, long cap, const float* __restrict__ slabs, int sk) {
  __shared__ uint32_t s_epoch;
  __shared__ float red[16];
  const int b = blockIdx.x;
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
  for (int r = b; r < rows; r += kArBlocks) {
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
  if (threadIdx.x < W) {
    uint32_t* pf = reinterpret_cast<uint32_t*>(peers.base[threadIdx.x] + kArFlagsOff) + b * 8 + rank;
    __hip_atomic_store(pf, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* f = reinterpret_cast<const uint32_t*>(my + kArFlagsOff) + b * 8 + threadIdx.x;
    spin_wait(f, e, reinterpret_cast<uint32_t*>(my + kArErrOff));
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 3. reduce
  const bf16* src[W];
#pragma unroll
  for (int p = 0; p < W; ++p) src[p] = reinterpret_cast<const bf16*>(peers.base[p] + data_off);
  for (int r = b; r < rows; r += kArBlocks) {
    const long ro = (long)r * dim;
    if constexpr (MODE == 0) {
      for (int c = threadIdx.x; c < nvec; c += kArThreads) {
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
        reinterpret_cast<bf16x8*>(out + ro)[c] = o;
      }
    } else {
      float v[NV][8];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = threadIdx.x + i * kArThreads;
        if (c < nvec) {
          bf16x8 x[W];
#pragma unroll
          for (int p = 0; p < W; ++p)
            x[p] = p == rank ? reinterpret_cast<const bf16x8*>(own + ro)[c]
                             : reinterpret_cast<const bf16x8*>(src[p] + ro)[c];
          const bf16x8 rr = reinterpret_cast<const bf16x8*>(residual + ro)[c];
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

template <int W>
int launch_w(const bf16* in, bf16* out, bf16* residual, const bf16* w, float eps, int rows,
             int dim, const ArPeers& peers, int rank, long cap, const float* slabs, int sk,
             hipStream_t stream) {
  const dim3 grid(kArBlocks), block(kArThreads);
  if (residual == nullptr) {
    allreduce_kernel<W, 0, 1><<<grid, block, 0, stream>>>(in, out, nullptr, nullptr, 0.f, rows,
                                                          dim, peers, rank, cap, slabs, sk);
    return 0;
  }
  const int nv = (dim / 8 + kArThreads - 1) / kArThreads;
#define AR_NV(N)                                                                          \
  case N:                                                                                 \
    allreduce_kernel<W, 1, N><<<grid, block, 0, stream>>>(in, out, residual, w, eps, rows, \
                                                          dim, peers, rank, cap, slabs, sk); \
    return 0;
  switch (nv) {
    AR_NV(1) AR_NV(2) AR_NV(4) AR_NV(8)
    case 3: allreduce_kernel<W, 1, 4><<<grid, block, 0, stream>>>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk); return 0;
    case 5: case 6: case 7:
      allreduce_kernel<W, 1, 8><<<grid, block, 0, stream>>>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk);
      return 0;
    default: return -1;
  }
#undef AR_NV
}

}  // namespace

int launch_custom_allreduce(const bf16* in, bf16* out, bf16* residual, const bf16* w, float eps,
                            int rows, int dim, const ArPeers& peers, int world, int rank,
                            long cap, hipStream_t stream, const float* slabs, int sk) {
  if (dim % 8 != 0 || dim > 16384 || rows < 0) return -2;
  if (slabs != nullptr && sk < 1) return -6;
  if ((long)rows * dim * 2 > cap) return -3;
  if (rank < 0 || rank >= world) return -4;
  switch (world) {
    case 2: return launch_w<2>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, stream);
    case 4: return launch_w<4>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, stream);
    case 8: return launch_w<8>(in, out, residual, w, eps, rows, dim, peers, rank, cap, slabs, sk, stream);
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

int car_error(const void* base) {
  uint32_t e = 0;
  if (hipMemcpy(&e, static_cast<const char*>(base) + kArErrOff, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (int)e;
}

}  // namespace bfly
