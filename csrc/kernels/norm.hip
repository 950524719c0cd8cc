// RMSNorm / fused residual-add + RMSNorm / LayerNorm kernels (K5, K15 in SURVEY.md §2.7-K).
//
// One workgroup per row; each lane moves 16 B (8 x bf16) per access (Guideline 13).
// The row is held in registers between the sum-of-squares pass and the scale pass, so
// each element is read from HBM exactly once and written once.
//   rows x dim, dim % 8 == 0, dim <= 8 * 8 * blockDim (checked on the host).
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

constexpr int kNormThreads = 256;
constexpr int kNormMaxVec = 8;  // up to 8 x 16 B per lane -> dim <= 16384 at 256 threads

template <int NV>
__global__ void __launch_bounds__(kNormThreads)
rmsnorm_kernel(const bf16* __restrict__ x, long x_stride, bf16* __restrict__ residual,
               const bf16* __restrict__ w, bf16* __restrict__ y, long y_stride, int dim,
               float eps, int add_residual) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * x_stride);
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + row * (long)dim);
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + row * y_stride);
  const int nvec = dim >> 3;
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      bf16x8 a = xr[c];
      if (add_residual) {
        bf16x8 r = rr[c];
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // Round the sum to bf16 first: the residual stream is stored in bf16 and the
          // normalised value must be computed from exactly what is stored.
          s[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));
          v[i][j] = bf2f(s[j]);
        }
        rr[c] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)dim + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      bf16x8 g = wr[c], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
      yr[c] = o;
    }
  }
}

// Add + RMSNorm whose input is the f32 split-K slabs [sk][rows][dim] of the producing GEMM
// (its deferred reduce fused here). 1024 threads per row and every slab load of a thread
// issued before the adds: at decode the rows are few (the batch), so each workgroup must keep
// many loads in flight to stream its sk x dim x 4 bytes.
// Measured and dropped (profiles/r2_norm_split_ab.log): cutting each row over 2048-column
// workgroups with a last-arriver rescale is 0.6-0.9 ms per 70B step SLOWER, since each
// workgroup's agent-scope release writes back its XCD's L2 and the hand-off crosses XCDs.
constexpr int kNormPartThreads = 1024;

// EC > 0 (MoE layers, EC = number of experts): the workgroup also routes the row it normalised
// — router logits from the stored bf16 row, then softmax / top-k (moe_select_topk) — which
// saves the separate moe_route launch per MoE layer (Mixtral 8x7B B = 64: 6.2 us per layer,
// profiles/r5_moe/mixtral_prefill_decode_trace.md).
template <int NV, int EC = 0>
__global__ void __launch_bounds__(kNormPartThreads)
rmsnorm_partial_kernel(const float* __restrict__ part, int sk, long slab, bf16* __restrict__ residual,
                       const bf16* __restrict__ w, bf16* __restrict__ y, int dim, float eps,
                       int add_residual, const bf16* __restrict__ rw = nullptr, int topk = 0,
                       float* __restrict__ gates = nullptr, int* __restrict__ topk_ids = nullptr,
                       float* __restrict__ topk_w = nullptr) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const int nvec = dim >> 3;
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + row * (long)dim);
  // MoE: the router chunks do not depend on the row, so their loads go out first and their
  // latency hides behind the slab loads
  constexpr int RE = EC > 0 ? EC : 1, RN = EC > 0 ? NV : 1;
  bf16x8 rv[RN][RE];
  if constexpr (EC > 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = threadIdx.x + i * kNormPartThreads;
      if (c < nvec)
#pragma unroll
        for (int e = 0; e < EC; ++e) rv[i][e] = reinterpret_cast<const bf16x8*>(rw + (long)e * dim)[c];
    }
  }
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormPartThreads;
    if (c < nvec) {
      const float* pr = part + row * (long)dim + c * 8;
      f32x4 lo = *reinterpret_cast<const f32x4*>(pr), hi = *reinterpret_cast<const f32x4*>(pr + 4);
#pragma unroll 8
      for (int k = 1; k < sk; ++k) {
        lo += *reinterpret_cast<const f32x4*>(pr + k * slab);
        hi += *reinterpret_cast<const f32x4*>(pr + k * slab + 4);
      }
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) { a[j] = f2bf(lo[j]); a[j + 4] = f2bf(hi[j]); }
      if (add_residual) {
        const bf16x8 r = rr[c];
        bf16x8 sm;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sm[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));
          v[i][j] = bf2f(sm[j]);
        }
        rr[c] = sm;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)dim + eps);
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + row * (long)dim);
  float racc[EC > 0 ? EC : 1];
#pragma unroll
  for (int e = 0; e < (EC > 0 ? EC : 1); ++e) racc[e] = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormPartThreads;
    if (c < nvec) {
      const bf16x8 g = wr[c];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
      yr[c] = o;
      if constexpr (EC > 0) {
#pragma unroll
        for (int e = 0; e < EC; ++e)
#pragma unroll
          for (int j = 0; j < 8; ++j) racc[e] += bf2f(o[j]) * bf2f(rv[i][e][j]);
      }
    }
  }
  if constexpr (EC > 0) {
    __shared__ float rred[kNormPartThreads / 64][EC];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int e = 0; e < EC; ++e) {
      const float s = wave_sum(racc[e]);
      if (lane == 0) rred[wv][e] = s;
    }
    __syncthreads();
    if (wv != 0) return;
    const bool live = lane < EC;
    float logit = 0.f;
    if (live)
#pragma unroll
      for (int q = 0; q < kNormPartThreads / 64; ++q) logit += rred[q][lane];
    moe_select_topk(logit, live, lane, (int)row, EC, topk, gates, topk_ids, topk_w);
  }
}

// Row-split add + RMSNorm for decode-sized batches whose consumer GEMM applies the row scale
// (launch_gemm(..., rs)). The norm is linear in its row scale: norm(x) W^T = rsqrt(ms(x) + eps)
// * ((x * g) W^T), so this kernel writes y = x * g and each (row, 1024-column chunk) workgroup
// only its partial sum of squares ssp[row][chunk]; the GEMM epilogue sums the chunk partials
// (the kernel boundary is the hand-off: no inter-workgroup protocol) and scales its rows.
// Why: rmsnorm_partial_kernel gives a row (sk x dim x 4 bytes of slabs) to ONE workgroup, so at
// a batch of 64 rows 64 CUs pull 8-16 MB while 192 idle; here rows x chunks workgroups share it.
// x is the sum of `sk` f32 slabs [sk][rows][dim] (part != nullptr) or a bf16 [rows][dim] input.
constexpr int kNormSplitThreads = 128;
constexpr int kNormSplitCols = kNormSplitThreads * 8;

__global__ void __launch_bounds__(kNormSplitThreads)
rmsnorm_rows_kernel(const float* __restrict__ part, int sk, long slab, const bf16* __restrict__ x,
                    long x_stride, bf16* __restrict__ residual, const bf16* __restrict__ w,
                    bf16* __restrict__ y, float* __restrict__ ssp, int dim, int add_residual) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const int col = blockIdx.y * kNormSplitCols + threadIdx.x * 8;
  float ss = 0.f;
  if (col < dim) {
    bf16x8 a;
    if (part != nullptr) {
      const float* pr = part + row * (long)dim + col;
      f32x4 lo = *reinterpret_cast<const f32x4*>(pr), hi = *reinterpret_cast<const f32x4*>(pr + 4);
#pragma unroll 8
      for (int k = 1; k < sk; ++k) {
        lo += *reinterpret_cast<const f32x4*>(pr + k * slab);
        hi += *reinterpret_cast<const f32x4*>(pr + k * slab + 4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) { a[j] = f2bf(lo[j]); a[j + 4] = f2bf(hi[j]); }
    } else {
      a = *reinterpret_cast<const bf16x8*>(x + row * x_stride + col);
    }
    float v[8];
    if (add_residual) {
      bf16x8* rp = reinterpret_cast<bf16x8*>(residual + row * (long)dim + col);
      const bf16x8 r = *rp;
      bf16x8 sm;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sm[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));   // the stored bf16 residual is what is normalised
        v[j] = bf2f(sm[j]);
      }
      *rp = sm;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
    }
    const bf16x8 g = *reinterpret_cast<const bf16x8*>(w + col);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ss += v[j] * v[j];
      o[j] = f2bf(v[j] * bf2f(g[j]));
    }
    *reinterpret_cast<bf16x8*>(y + row * (long)dim + col) = o;
  }
  ss = block_sum(ss, red);
  if (threadIdx.x == 0) ssp[row * gridDim.y + blockIdx.y] = ss;
}

int rmsnorm_rows_chunks(int dim) { return (dim + kNormSplitCols - 1) / kNormSplitCols; }

int launch_rmsnorm_rows(const bf16* x, long x_stride, bf16* residual, const bf16* w, bf16* y, float* ssp,
                        int rows, int dim, bool add_residual, hipStream_t stream, const float* part, int sk) {
  if (dim % 8 != 0) return -1;
  if (rows <= 0) return 0;
  dim3 grid(rows, rmsnorm_rows_chunks(dim));
  rmsnorm_rows_kernel<<<grid, kNormSplitThreads, 0, stream>>>(part, sk, (long)rows * dim, x, x_stride, residual,
                                                              w, y, ssp, dim, add_residual ? 1 : 0);
  return 0;
}

template <int NV>
__global__ void __launch_bounds__(kNormThreads)
layernorm_kernel(const bf16* __restrict__ x, bf16* __restrict__ residual,
                 const bf16* __restrict__ w, const bf16* __restrict__ b,
                 bf16* __restrict__ y, int dim, float eps, int add_residual) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * (long)dim);
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + row * (long)dim);
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  const bf16x8* br = reinterpret_cast<const bf16x8*>(b);
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + row * (long)dim);
  const int nvec = dim >> 3;
  float v[NV][8];
  float s1 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      bf16x8 a = xr[c];
      if (add_residual) {
        bf16x8 r = rr[c], s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = f2bf(bf2f(a[j]) + bf2f(r[j]));
          v[i][j] = bf2f(s[j]);
        }
        rr[c] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s1 += v[i][j];
    }
  }
  const float mean = block_sum(s1, red) / (float)dim;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum(s2, red) / (float)dim + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * kNormThreads;
    if (c < nvec) {
      bf16x8 g = wr[c], bb = br[c], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf((v[i][j] - mean) * inv * bf2f(g[j]) + bf2f(bb[j]));
      yr[c] = o;
    }
  }
}

void launch_rmsnorm(const bf16* x, long x_stride, bf16* residual, const bf16* w, bf16* y,
                    long y_stride, int rows, int dim, float eps, bool add_residual,
                    hipStream_t stream, const float* part, int sk) {
  if (part != nullptr) {
    if (rows <= 0) return;
    const long slab = (long)rows * dim;
    const int nv = (dim / 8 + kNormPartThreads - 1) / kNormPartThreads;
    const int ar = add_residual ? 1 : 0;
    if (nv <= 1)
      rmsnorm_partial_kernel<1><<<rows, kNormPartThreads, 0, stream>>>(part, sk, slab, residual, w, y, dim, eps, ar);
    else
      rmsnorm_partial_kernel<2><<<rows, kNormPartThreads, 0, stream>>>(part, sk, slab, residual, w, y, dim, eps, ar);
    return;
  }
  if (rows <= 0) return;
  const int nvec = dim / 8;
  const int nv = (nvec + kNormThreads - 1) / kNormThreads;
  dim3 grid(rows), block(kNormThreads);
  const int ar = add_residual ? 1 : 0;
  switch (nv) {
    case 1: rmsnorm_kernel<1><<<grid, block, 0, stream>>>(x, x_stride, residual, w, y, y_stride, dim, eps, ar); break;
    case 2: rmsnorm_kernel<2><<<grid, block, 0, stream>>>(x, x_stride, residual, w, y, y_stride, dim, eps, ar); break;
    case 3:
    case 4: rmsnorm_kernel<4><<<grid, block, 0, stream>>>(x, x_stride, residual, w, y, y_stride, dim, eps, ar); break;
    default: rmsnorm_kernel<kNormMaxVec><<<grid, block, 0, stream>>>(x, x_stride, residual, w, y, y_stride, dim, eps, ar); break;
  }
}

int launch_rmsnorm_route(const float* part, int sk, bf16* residual, const bf16* w, bf16* y, int rows,
                         int dim, float eps, bool add_residual, const bf16* router_w, int E, int topk,
                         float* gates, int* topk_ids, float* topk_w, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (part == nullptr || (E != 4 && E != 8) || topk < 1 || topk > E || dim % 8 != 0) return -1;
  const long slab = (long)rows * dim;
  const int nv = (dim / 8 + kNormPartThreads - 1) / kNormPartThreads;
  if (nv > 2) return -2;
  const int ar = add_residual ? 1 : 0;
#define NORM_ROUTE(NV_, EC_)                                                                          \
  rmsnorm_partial_kernel<NV_, EC_><<<rows, kNormPartThreads, 0, stream>>>(part, sk, slab, residual, w, y, dim, \
                                                                         eps, ar, router_w, topk, gates,   \
                                                                         topk_ids, topk_w)
  if (E == 8) {
    if (nv <= 1) NORM_ROUTE(1, 8); else NORM_ROUTE(2, 8);
  } else {
    if (nv <= 1) NORM_ROUTE(1, 4); else NORM_ROUTE(2, 4);
  }
#undef NORM_ROUTE
  return 0;
}

void launch_layernorm(const bf16* x, bf16* residual, const bf16* w, const bf16* b, bf16* y,
                      int rows, int dim, float eps, bool add_residual, hipStream_t stream) {
  if (rows <= 0) return;
  const int nvec = dim / 8;
  const int nv = (nvec + kNormThreads - 1) / kNormThreads;
  dim3 grid(rows), block(kNormThreads);
  const int ar = add_residual ? 1 : 0;
  switch (nv) {
    case 1: layernorm_kernel<1><<<grid, block, 0, stream>>>(x, residual, w, b, y, dim, eps, ar); break;
    case 2: layernorm_kernel<2><<<grid, block, 0, stream>>>(x, residual, w, b, y, dim, eps, ar); break;
    case 3:
    case 4: layernorm_kernel<4><<<grid, block, 0, stream>>>(x, residual, w, b, y, dim, eps, ar); break;
    default: layernorm_kernel<kNormMaxVec><<<grid, block, 0, stream>>>(x, residual, w, b, y, dim, eps, ar); break;
  }
}

}  // namespace bfly
