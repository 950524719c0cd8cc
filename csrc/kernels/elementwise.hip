// Small memory-bound kernels: SwiGLU activation (K7), GELU, residual add, vocab-parallel
// embedding gather (K9). Every access is 16 B per lane (Guideline 13); grids are capped
// and grid-strided (Guideline 11).
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

constexpr int kEwThreads = 256;
static inline int ew_grid(long nvec) {
  long g = (nvec + kEwThreads - 1) / kEwThreads;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

// out[r, c] = silu(gu[r, gate(c)]) * gu[r, up(c)].
// `interleave` = 0: gu = [gate | up] halves.  interleave = G > 0: gu rows are stored in
// alternating G-column groups (g0 u0 g1 u1 ...), the layout the fused gate/up GEMM emits.
__global__ void silu_mul_kernel(const bf16* __restrict__ gu, bf16* __restrict__ out, long rows,
                                int ffn, int interleave) {
  const long nvec = rows * (ffn / 8);
  const int vpr = ffn / 8;
  for (long i = blockIdx.x * (long)kEwThreads + threadIdx.x; i < nvec;
       i += (long)gridDim.x * kEwThreads) {
    const long r = i / vpr;
    const int c = (int)(i % vpr) * 8;
    long gi, ui;
    if (interleave == 0) {
      gi = r * 2L * ffn + c;
      ui = gi + ffn;
    } else {
      const int grp = c / interleave, w = c % interleave;
      gi = r * 2L * ffn + (long)grp * 2 * interleave + w;
      ui = gi + interleave;
    }
    const bf16x8 g = *reinterpret_cast<const bf16x8*>(gu + gi);
    const bf16x8 u = *reinterpret_cast<const bf16x8*>(gu + ui);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(silu(bf2f(g[j])) * bf2f(u[j]));
    *reinterpret_cast<bf16x8*>(out + r * (long)ffn + c) = o;
  }
}

__global__ void gelu_kernel(const bf16* __restrict__ x, bf16* __restrict__ out, long nvec) {
  for (long i = blockIdx.x * (long)kEwThreads + threadIdx.x; i < nvec;
       i += (long)gridDim.x * kEwThreads) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(x)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(gelu_tanh(bf2f(a[j])));
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

__global__ void add_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                           bf16* __restrict__ out, long nvec) {
  for (long i = blockIdx.x * (long)kEwThreads + threadIdx.x; i < nvec;
       i += (long)gridDim.x * kEwThreads) {
    const bf16x8 x = reinterpret_cast<const bf16x8*>(a)[i];
    const bf16x8 y = reinterpret_cast<const bf16x8*>(b)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(x[j]) + bf2f(y[j]));
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

// Vocab-parallel embedding: rows whose id falls outside [vstart, vstart + vlocal) are
// zero (the TP all-reduce that follows sums exactly one non-zero contribution per row).
__global__ void embed_kernel(const int* __restrict__ ids, const bf16* __restrict__ table,
                             bf16* __restrict__ out, int dim, int vstart, int vlocal) {
  const int t = blockIdx.x;
  const int id = ids[t] - vstart;
  const bool in = id >= 0 && id < vlocal;
  const bf16x8* src = reinterpret_cast<const bf16x8*>(table + (long)(in ? id : 0) * dim);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out + (long)t * dim);
  for (int c = threadIdx.x; c < dim / 8; c += kEwThreads) {
    bf16x8 v = src[c];
    if (!in) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = f2bf(0.f);
    }
    dst[c] = v;
  }
}

// Row gather: out[i] = src[idx[i]] for rows of `words` 4-byte words (bf16 / f32 / int32 rows);
// rows with idx < 0 are left as they are (the caller pre-filled them). Replaces torch's
// index_select / gather on serving paths (final-token rows, pipeline input ids): one small
// launch of our own instead of an at::native kernel. An index past the source (idx >= nsrc,
// which index_select rejects with an error) is loud instead of silent: the row is filled with
// all-ones words (NaN as f32 or bf16, -1 as int32 ids) so the fault shows downstream, and the
// host wrapper checks indices eagerly under BFLY_DEBUG_CHECKS.
template <typename IT>
__global__ void gather_rows_kernel(const uint32_t* __restrict__ src, long src_ld, const IT* __restrict__ idx,
                                   uint32_t* __restrict__ out, long out_ld, int words, long nsrc) {
  const long i = blockIdx.x;
  const long j = (long)idx[i];
  if (j < 0) return;
  uint32_t* o = out + i * out_ld;
  if (j >= nsrc) {
    for (int c = threadIdx.x; c < words; c += kEwThreads) o[c] = 0xffffffffu;
    return;
  }
  const uint32_t* s = src + j * src_ld;
  if ((words & 3) == 0 && ((src_ld | out_ld) & 3) == 0) {
    for (int c = threadIdx.x; c < words / 4; c += kEwThreads)
      reinterpret_cast<u32x4*>(o)[c] = reinterpret_cast<const u32x4*>(s)[c];
  } else {
    for (int c = threadIdx.x; c < words; c += kEwThreads) o[c] = s[c];
  }
}

// Deterministic, partition-independent random init: element (global_row, global_col) of a
// logical weight gets a value that depends only on (seed, global index), so every rank can
// generate exactly its own shard and any partition reproduces the same global weights.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__global__ void init_hash_kernel(bf16* __restrict__ out, long rows, int cols, long ld, long grow0,
                                 long gcol0, long gcols, uint32_t seed, float amp) {
  const long n = rows * cols;
  for (long e = blockIdx.x * (long)kEwThreads + threadIdx.x; e < n;
       e += (long)gridDim.x * kEwThreads) {
    const long r = e / cols;
    const int c = (int)(e % cols);
    const uint32_t idx = (uint32_t)((grow0 + r) * gcols + gcol0 + c);
    const uint32_t h = fmix32(idx * 0x9E3779B1u + seed);
    const float u = (float)(h >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f);
    out[r * ld + c] = f2bf(amp * (2.f * u - 1.f));
  }
}

void launch_init_hash(bf16* out, long rows, int cols, long ld, long grow0, long gcol0, long gcols,
                      uint32_t seed, float amp, hipStream_t stream) {
  const long n = rows * cols;
  if (n <= 0) return;
  long g = (n + kEwThreads - 1) / kEwThreads;
  if (g > 65536) g = 65536;
  init_hash_kernel<<<(int)g, kEwThreads, 0, stream>>>(out, rows, cols, ld, grow0, gcol0, gcols, seed, amp);
}

void launch_silu_mul(const bf16* gu, bf16* out, long rows, int ffn, int interleave,
                     hipStream_t stream) {
  const long nvec = rows * (ffn / 8);
  if (nvec <= 0) return;
  silu_mul_kernel<<<ew_grid(nvec), kEwThreads, 0, stream>>>(gu, out, rows, ffn, interleave);
}

void launch_gelu(const bf16* x, bf16* out, long n, hipStream_t stream) {
  if (n <= 0) return;
  gelu_kernel<<<ew_grid(n / 8), kEwThreads, 0, stream>>>(x, out, n / 8);
}

void launch_add(const bf16* a, const bf16* b, bf16* out, long n, hipStream_t stream) {
  if (n <= 0) return;
  add_kernel<<<ew_grid(n / 8), kEwThreads, 0, stream>>>(a, b, out, n / 8);
}

void launch_gather_rows(const void* src, long src_ld, const void* idx, bool idx64, void* out, long out_ld,
                        int words, long rows, long nsrc, hipStream_t stream) {
  if (rows <= 0 || words <= 0) return;
  if (idx64)
    gather_rows_kernel<long><<<rows, kEwThreads, 0, stream>>>(static_cast<const uint32_t*>(src), src_ld,
                                                              static_cast<const long*>(idx),
                                                              static_cast<uint32_t*>(out), out_ld, words, nsrc);
  else
    gather_rows_kernel<int><<<rows, kEwThreads, 0, stream>>>(static_cast<const uint32_t*>(src), src_ld,
                                                             static_cast<const int*>(idx),
                                                             static_cast<uint32_t*>(out), out_ld, words, nsrc);
}

void launch_embed(const int* ids, const bf16* table, bf16* out, int T, int dim, int vstart,
                  int vlocal, hipStream_t stream) {
  if (T <= 0) return;
  embed_kernel<<<T, kEwThreads, 0, stream>>>(ids, table, out, dim, vstart, vlocal);
}

}  // namespace bfly
