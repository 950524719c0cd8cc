// RoPE (rotate-half / NeoX convention) applied in place to the Q and K heads of the fused
// QKV projection output, fused with the paged KV-cache append (K6 + K8 in SURVEY.md §2.7-K).
//
// qkv       [T, (Hq + 2*Hkv) * D]  bf16 (GEMM output; Q heads, then K heads, then V heads)
// positions [T] int32
// cos/sin   [max_pos, D/2] f32 host-precomputed tables (no device trig: Appendix B)
// slots     [T] int32: cache slot = block * BS + offset, < 0 = do not cache
// k_cache   [num_blocks, Hkv, BS, D]      (K rows contiguous: decode QK^T operand)
// v_cache   [num_blocks, Hkv, D, BS]      (V stored transposed: decode PV operand reads
//                                          8 consecutive keys of one d as one 16-B load)
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

constexpr int kRopeThreads = 256;

template <int D>
__global__ void __launch_bounds__(kRopeThreads)
rope_kv_kernel(bf16* __restrict__ qkv, const int* __restrict__ positions,
               const float* __restrict__ cos_t, const float* __restrict__ sin_t,
               const int* __restrict__ slots, bf16* __restrict__ k_cache,
               bf16* __restrict__ v_cache, int Hq, int Hkv, int BS) {
  constexpr int H2 = D / 2;        // rotation pairs per head
  constexpr int LPH = H2 / 8;      // lanes per head (each lane: 8 pairs)
  const int t = blockIdx.x;
  const long row_stride = (long)(Hq + 2 * Hkv) * D;
  bf16* row = qkv + (long)t * row_stride;
  const int pos = positions[t];
  const float* cr = cos_t + (long)pos * H2;
  const float* sr = sin_t + (long)pos * H2;
  const int slot = slots ? slots[t] : -1;
  const int blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  const int nrot = (Hq + Hkv) * LPH;
  for (int i = threadIdx.x; i < nrot; i += kRopeThreads) {
    const int h = i / LPH, p0 = (i % LPH) * 8;
    bf16* hp = row + (long)h * D;
    bf16x8 a = *reinterpret_cast<const bf16x8*>(hp + p0);
    bf16x8 b = *reinterpret_cast<const bf16x8*>(hp + p0 + H2);
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(cr + p0);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(cr + p0 + 4);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sr + p0);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(sr + p0 + 4);
    bf16x8 oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? c0[j] : c1[j - 4];
      const float s = j < 4 ? s0[j] : s1[j - 4];
      const float x0 = bf2f(a[j]), x1 = bf2f(b[j]);
      oa[j] = f2bf(x0 * c - x1 * s);
      ob[j] = f2bf(x1 * c + x0 * s);
    }
    *reinterpret_cast<bf16x8*>(hp + p0) = oa;
    *reinterpret_cast<bf16x8*>(hp + p0 + H2) = ob;
    if (h >= Hq && slot >= 0 && k_cache) {
      const int kh = h - Hq;
      bf16* kp = k_cache + (((long)blk * Hkv + kh) * BS + off) * D;
      *reinterpret_cast<bf16x8*>(kp + p0) = oa;
      *reinterpret_cast<bf16x8*>(kp + p0 + H2) = ob;
    }
  }
  if (slot < 0 || !v_cache) return;
  // V heads: copy into the transposed cache page (8 scattered 2-B stores per lane).
  constexpr int LPV = D / 8;
  const int nv = Hkv * LPV;
  for (int i = threadIdx.x; i < nv; i += kRopeThreads) {
    const int kh = i / LPV, d0 = (i % LPV) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + (long)(Hq + Hkv + kh) * D + d0);
    bf16* vp = v_cache + ((long)blk * Hkv + kh) * D * BS + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) vp[(long)(d0 + j) * BS] = v[j];
  }
}

// Standalone paged-cache append for already-rotated K and V ([T, Hkv, D] each, any row
// stride): used by the prefill path when K/V come from somewhere other than a fused QKV row.
template <int D>
__global__ void __launch_bounds__(kRopeThreads)
kv_append_kernel(const bf16* __restrict__ k, long k_stride, const bf16* __restrict__ v,
                 long v_stride, const int* __restrict__ slots, bf16* __restrict__ k_cache,
                 bf16* __restrict__ v_cache, int Hkv, int BS) {
  const int t = blockIdx.x;
  const int slot = slots[t];
  if (slot < 0) return;
  const int blk = slot / BS, off = slot % BS;
  constexpr int LPV = D / 8;
  for (int i = threadIdx.x; i < Hkv * LPV; i += kRopeThreads) {
    const int h = i / LPV, d0 = (i % LPV) * 8;
    const bf16x8 kv = *reinterpret_cast<const bf16x8*>(k + (long)t * k_stride + (long)h * D + d0);
    const bf16x8 vv = *reinterpret_cast<const bf16x8*>(v + (long)t * v_stride + (long)h * D + d0);
    *reinterpret_cast<bf16x8*>(k_cache + (((long)blk * Hkv + h) * BS + off) * D + d0) = kv;
    bf16* vp = v_cache + ((long)blk * Hkv + h) * D * BS + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) vp[(long)(d0 + j) * BS] = vv[j];
  }
}

void launch_rope_kv(bf16* qkv, int T, int Hq, int Hkv, int D, const int* positions,
                    const float* cos_t, const float* sin_t, const int* slots, bf16* k_cache,
                    bf16* v_cache, int block_size, hipStream_t stream) {
  if (T <= 0) return;
  if (D == 128) {
    rope_kv_kernel<128><<<T, kRopeThreads, 0, stream>>>(qkv, positions, cos_t, sin_t, slots,
                                                       k_cache, v_cache, Hq, Hkv, block_size);
  } else if (D == 64) {
    rope_kv_kernel<64><<<T, kRopeThreads, 0, stream>>>(qkv, positions, cos_t, sin_t, slots,
                                                      k_cache, v_cache, Hq, Hkv, block_size);
  }
}

void launch_kv_append(const bf16* k, long k_stride, const bf16* v, long v_stride,
                      const int* slots, bf16* k_cache, bf16* v_cache, int T, int Hkv, int D,
                      int block_size, hipStream_t stream) {
  if (T <= 0) return;
  if (D == 128) {
    kv_append_kernel<128><<<T, kRopeThreads, 0, stream>>>(k, k_stride, v, v_stride, slots,
                                                         k_cache, v_cache, Hkv, block_size);
  } else if (D == 64) {
    kv_append_kernel<64><<<T, kRopeThreads, 0, stream>>>(k, k_stride, v, v_stride, slots,
                                                        k_cache, v_cache, Hkv, block_size);
  }
}

}  // namespace bfly
