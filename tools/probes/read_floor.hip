// HBM read floor probe: every workgroup streams a contiguous share of a buffer with 16-byte
// loads, UNROLL loads in flight per lane, and folds them into one value per workgroup (so
// nothing is optimised away). Timed over buffer sizes that match single decode projections.
#include <hip/hip_runtime.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL>
__device__ void read_body(const u32x4* __restrict__ src, long n16, unsigned* __restrict__ sink) {
  const long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long b = per * blockIdx.x, e = min(b + per, n16);
  unsigned acc = 0;
  for (long i = b + threadIdx.x; i < e; i += (long)blockDim.x * UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const long j = i + (long)u * blockDim.x;
      v[u] = j < e ? __builtin_nontemporal_load(src + j) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;   // practically never: keeps the loads live
}

extern "C" __global__ void __launch_bounds__(256) read4(const u32x4* s, long n, unsigned* k) { read_body<4>(s, n, k); }
extern "C" __global__ void __launch_bounds__(256) read8(const u32x4* s, long n, unsigned* k) { read_body<8>(s, n, k); }
extern "C" __global__ void __launch_bounds__(256) read16(const u32x4* s, long n, unsigned* k) { read_body<16>(s, n, k); }

// GEMM-shaped weight walk: workgroup (n-tile, k-split) reads rows [n0, n0 + BN) of a row-major
// [N, K] bf16 matrix over its K range, 128 B of every row per 64-element K step (the pattern a
// decode GEMM's weight DMA has), UNROLL K steps in flight.
template <int BN, int UNROLL>
__device__ void tiled_body(const u32x4* __restrict__ src, int N, int K, int ksplit, unsigned* __restrict__ sink) {
  constexpr int PER = BN * 8 / 256;   // 16-byte loads per lane per K step
  const int nt = blockIdx.x / ksplit, ks = blockIdx.x % ksplit;
  const int ksteps = K / 64;
  const int k0 = ksteps * ks / ksplit, k1 = ksteps * (ks + 1) / ksplit;
  const long ld16 = K / 8;   // 16-byte chunks per row
  unsigned acc = 0;
  for (int k = k0; k < k1; k += UNROLL) {
    u32x4 v[UNROLL][PER];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int c = p * 256 + threadIdx.x;   // chunk c: row c >> 3, 16 B column c & 7
        const long idx = (long)(nt * BN + (c >> 3)) * ld16 + (long)min(k + u, k1 - 1) * 8 + (c & 7);
        v[u][p] = __builtin_nontemporal_load(src + idx);
      }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int p = 0; p < PER; ++p) acc ^= v[u][p].x ^ v[u][p].y ^ v[u][p].z ^ v[u][p].w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}

extern "C" __global__ void __launch_bounds__(256) tiled128(const u32x4* s, int N, int K, int sk, unsigned* k) {
  tiled_body<128, 4>(s, N, K, sk, k);
}
extern "C" __global__ void __launch_bounds__(256) tiled64(const u32x4* s, int N, int K, int sk, unsigned* k) {
  tiled_body<64, 8>(s, N, K, sk, k);
}
extern "C" __global__ void __launch_bounds__(256) tiled32(const u32x4* s, int N, int K, int sk, unsigned* k) {
  tiled_body<32, 16>(s, N, K, sk, k);
}

// MFMA-fragment weight walk (the skinny GEMM's load pattern): lane L reads row 16 t + (L & 15)
// at element 8 (L >> 4) + 32 s of a 128-element K chunk (4 instructions of 16 rows x 64 B per
// 16-row group), the 4 waves split the workgroup's K range, U chunks in flight per wave.
template <int NT, int U>
__device__ void frag_body(const u32x4* __restrict__ src, int N, int K, int ksplit, unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nt = blockIdx.x / ksplit, ks = blockIdx.x % ksplit;
  const int chunks = K / 128, S = ksplit * 4, si = ks * 4 + wid;
  const int c0 = chunks * si / S, c1 = chunks * (si + 1) / S;
  const long ld16 = K / 8;
  const int g = lane >> 4, r = lane & 15;
  unsigned acc = 0;
  for (int c = c0; c < c1; c += U) {
    u32x4 v[U][NT][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const long idx = (long)(nt * 16 * NT + 16 * t + r) * ld16 + (long)min(c + u, c1 - 1) * 16 + g + 4 * s;
          v[u][t][s] = __builtin_nontemporal_load(src + idx);
        }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc ^= v[u][t][s].x ^ v[u][t][s].w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}

extern "C" __global__ void __launch_bounds__(256) frag2(const u32x4* s, int N, int K, int sk, unsigned* k) {
  frag_body<2, 2>(s, N, K, sk, k);
}
extern "C" __global__ void __launch_bounds__(256) frag4(const u32x4* s, int N, int K, int sk, unsigned* k) {
  frag_body<4, 1>(s, N, K, sk, k);
}
extern "C" __global__ void __launch_bounds__(256) frag1(const u32x4* s, int N, int K, int sk, unsigned* k) {
  frag_body<1, 4>(s, N, K, sk, k);
}
