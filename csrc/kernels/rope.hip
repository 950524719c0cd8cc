// RoPE (rotate-half / NeoX convention) applied in place to the Q and K heads of the fused
// QKV projection output, fused with the paged KV-cache append (K6 + K8 in SURVEY.md §2.7-K).
//
// qkv       [T, (Hq + 2*Hkv) * D]  bf16 (GEMM output; Q heads, then K heads, then V heads)
// positions [T] int32
// cos/sin   [max_pos, D/2] f32 host-precomputed tables (no device trig: Appendix B)
// slots     [T] int32: cache slot = block * BS + offset, < 0 = do not cache
// k_cache   [num_blocks, Hkv, BS, D]      (K rows contiguous: decode QK^T operand)
// v_cache   [num_blocks, Hkv, D, BS]      (V stored transposed: decode PV operand reads
//                                          8 consecutive keys of one d as one load)
// Cache elements are bf16 or FP8 e4m3 (bfly_kv.h); the rotated bf16 values are what is
// cached, so an FP8 cache holds exactly torch's bf16 -> float8_e4m3fn conversion of them.
#include "bfly_common.h"
#include "bfly_kernels.h"
#include "bfly_kv.h"

namespace bfly {

constexpr int kRopeThreads = 256;

// Grid (T, ceil(items / 256)): item i < Hrot*LPH rotates 8 pairs of one Q/K head, the rest copy
// 8 elements of one V head (so a token's work spreads over several workgroups: at decode T is
// only the batch size). With `part` the row is first assembled from the f32 split-K slabs of
// the QKV GEMM (its deferred reduce fused here) and written back to `qkv` in bf16.
// Deferred split-K reduce of NC 8-column pieces of one row (the rotation pair's two halves, or one
// V piece): slabs in batches of 8 with every load of the batch issued before any add — one
// dependent add chain over the 16 slabs of the tp8 B = 1 QKV plan waited a load latency per slab
// (14 us per launch, profiles/r6_latency.md). The adds keep the slab order (the reduce kernel's
// sum, bit for bit).
template <int NC>
__device__ __forceinline__ void slab_sum(const float* __restrict__ prow, int sk, long slab, const int (&col)[NC],
                                         f32x4 (&lo)[NC], f32x4 (&hi)[NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    lo[c] = *reinterpret_cast<const f32x4*>(prow + col[c]);
    hi[c] = *reinterpret_cast<const f32x4*>(prow + col[c] + 4);
  }
  for (int k0 = 1; k0 < sk; k0 += 8) {
    f32x4 l[8][NC], h[8][NC];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long off = (long)(k0 + j < sk ? k0 + j : k0) * slab;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        l[j][c] = *reinterpret_cast<const f32x4*>(prow + off + col[c]);
        h[j][c] = *reinterpret_cast<const f32x4*>(prow + off + col[c] + 4);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (k0 + j < sk) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          lo[c] += l[j][c];
          hi[c] += h[j][c];
        }
      }
  }
}

__device__ __forceinline__ bf16x8 pack8(f32x4 lo, f32x4 hi) {
  bf16x8 a;
#pragma unroll
  for (int j = 0; j < 4; ++j) { a[j] = f2bf(lo[j]); a[j + 4] = f2bf(hi[j]); }
  return a;
}

// SLABS: the row comes from the QKV GEMM's split-K slabs (a separate instantiation, so the
// register-hungry batched slab loads do not cost the plain path occupancy at prefill sizes)
template <int D, typename CT, bool SLABS>
__global__ void __launch_bounds__(kRopeThreads)
rope_kv_kernel(bf16* __restrict__ qkv, const int* __restrict__ positions,
               const float* __restrict__ cos_t, const float* __restrict__ sin_t,
               const int* __restrict__ slots, CT* __restrict__ k_cache,
               CT* __restrict__ v_cache, int Hq, int Hkv, int BS,
               const float* __restrict__ part, int sk, long slab) {
  constexpr int H2 = D / 2;        // rotation pairs per head
  constexpr int LPH = H2 / 8;      // lanes per head (each lane: 8 pairs)
  constexpr int LPV = D / 8;
  const int t = blockIdx.x;
  const int i = blockIdx.y * kRopeThreads + threadIdx.x;
  const int nrot = (Hq + Hkv) * LPH, nv = Hkv * LPV;
  if (i >= nrot + nv) return;
  const long row_stride = (long)(Hq + 2 * Hkv) * D;
  bf16* row = qkv + (long)t * row_stride;
  const float* prow = SLABS ? part + (long)t * row_stride : nullptr;
  const int slot = slots ? slots[t] : -1;
  const int blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  if (i < nrot) {
    const int pos = positions[t];
    const float* cr = cos_t + (long)pos * H2;
    const float* sr = sin_t + (long)pos * H2;
    const int h = i / LPH, p0 = (i % LPH) * 8;
    bf16x8 a, b;
    if constexpr (SLABS) {
      const int cols[2] = {h * D + p0, h * D + p0 + H2};
      f32x4 lo[2], hi[2];
      slab_sum<2>(prow, sk, slab, cols, lo, hi);
      a = pack8(lo[0], hi[0]);
      b = pack8(lo[1], hi[1]);
    } else {
      a = *reinterpret_cast<const bf16x8*>(row + h * D + p0);
      b = *reinterpret_cast<const bf16x8*>(row + h * D + p0 + H2);
    }
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(cr + p0);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(cr + p0 + 4);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sr + p0);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(sr + p0 + 4);
    bf16x8 oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? c0[j] : c1[j - 4];
      const float s = j < 4 ? s0[j] : s1[j - 4];
      float r0, r1;
      rope_rotate(bf2f(a[j]), bf2f(b[j]), c, s, r0, r1);
      oa[j] = f2bf(r0);
      ob[j] = f2bf(r1);
    }
    bf16* hp = row + (long)h * D;
    *reinterpret_cast<bf16x8*>(hp + p0) = oa;
    *reinterpret_cast<bf16x8*>(hp + p0 + H2) = ob;
    if (h >= Hq && slot >= 0 && k_cache) {
      const int kh = h - Hq;
      CT* kp = k_cache + (((long)blk * Hkv + kh) * BS + off) * D;
      KV<CT>::store8(kp + p0, oa);
      KV<CT>::store8(kp + p0 + H2, ob);
    }
    return;
  }
  // V heads: (materialise and) copy into the transposed cache page (8 scattered stores)
  const int iv = i - nrot;
  const int kh = iv / LPV, d0 = (iv % LPV) * 8;
  const int col = (Hq + Hkv + kh) * D + d0;
  bf16x8 v;
  if constexpr (SLABS) {
    const int cols[1] = {col};
    f32x4 lo[1], hi[1];
    slab_sum<1>(prow, sk, slab, cols, lo, hi);
    v = pack8(lo[0], hi[0]);
  } else {
    v = *reinterpret_cast<const bf16x8*>(row + col);
  }
  if constexpr (SLABS) *reinterpret_cast<bf16x8*>(row + col) = v;
  if (slot < 0 || !v_cache) return;
  CT* vp = v_cache + ((long)blk * Hkv + kh) * D * BS + off;
#pragma unroll
  for (int j = 0; j < 8; ++j) KV<CT>::store1(vp + (long)(d0 + j) * BS, v[j]);
}

// Standalone paged-cache append for already-rotated K and V ([T, Hkv, D] each, any row
// stride): used by the prefill path when K/V come from somewhere other than a fused QKV row.
template <int D, typename CT>
__global__ void __launch_bounds__(kRopeThreads)
kv_append_kernel(const bf16* __restrict__ k, long k_stride, const bf16* __restrict__ v,
                 long v_stride, const int* __restrict__ slots, CT* __restrict__ k_cache,
                 CT* __restrict__ v_cache, int Hkv, int BS) {
  const int t = blockIdx.x;
  const int slot = slots[t];
  if (slot < 0) return;
  const int blk = slot / BS, off = slot % BS;
  constexpr int LPV = D / 8;
  for (int i = threadIdx.x; i < Hkv * LPV; i += kRopeThreads) {
    const int h = i / LPV, d0 = (i % LPV) * 8;
    const bf16x8 kv = *reinterpret_cast<const bf16x8*>(k + (long)t * k_stride + (long)h * D + d0);
    const bf16x8 vv = *reinterpret_cast<const bf16x8*>(v + (long)t * v_stride + (long)h * D + d0);
    KV<CT>::store8(k_cache + (((long)blk * Hkv + h) * BS + off) * D + d0, kv);
    CT* vp = v_cache + ((long)blk * Hkv + h) * D * BS + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) KV<CT>::store1(vp + (long)(d0 + j) * BS, vv[j]);
  }
}

template <typename CT>
static void run_rope_kv(bf16* qkv, int T, int Hq, int Hkv, int D, const int* positions,
                        const float* cos_t, const float* sin_t, const int* slots, void* k_cache,
                        void* v_cache, int block_size, hipStream_t stream, const float* part, int sk) {
  const long slab = (long)T * (Hq + 2 * Hkv) * D;
  const int items = (Hq + Hkv) * (D / 16) + Hkv * (D / 8);
  const dim3 grid(T, (items + kRopeThreads - 1) / kRopeThreads);
  CT* kc = static_cast<CT*>(k_cache);
  CT* vc = static_cast<CT*>(v_cache);
#define ROPE_LAUNCH(D_, S_)                                                                             \
  rope_kv_kernel<D_, CT, S_><<<grid, kRopeThreads, 0, stream>>>(qkv, positions, cos_t, sin_t, slots, kc, vc, \
                                                                Hq, Hkv, block_size, part, sk, slab)
  if (D == 128) {
    if (part) ROPE_LAUNCH(128, true);
    else ROPE_LAUNCH(128, false);
  } else if (D == 64) {
    if (part) ROPE_LAUNCH(64, true);
    else ROPE_LAUNCH(64, false);
  }
#undef ROPE_LAUNCH
}

void launch_rope_kv(bf16* qkv, int T, int Hq, int Hkv, int D, const int* positions,
                    const float* cos_t, const float* sin_t, const int* slots, void* k_cache,
                    void* v_cache, int block_size, hipStream_t stream, const float* part, int sk,
                    int kv_fp8) {
  if (T <= 0) return;
  if (kv_fp8)
    run_rope_kv<fp8_t>(qkv, T, Hq, Hkv, D, positions, cos_t, sin_t, slots, k_cache, v_cache, block_size,
                       stream, part, sk);
  else
    run_rope_kv<bf16>(qkv, T, Hq, Hkv, D, positions, cos_t, sin_t, slots, k_cache, v_cache, block_size,
                      stream, part, sk);
}

template <typename CT>
static void run_kv_append(const bf16* k, long k_stride, const bf16* v, long v_stride, const int* slots,
                          void* k_cache, void* v_cache, int T, int Hkv, int D, int block_size,
                          hipStream_t stream) {
  CT* kc = static_cast<CT*>(k_cache);
  CT* vc = static_cast<CT*>(v_cache);
  if (D == 128) {
    kv_append_kernel<128, CT><<<T, kRopeThreads, 0, stream>>>(k, k_stride, v, v_stride, slots, kc, vc, Hkv,
                                                             block_size);
  } else if (D == 64) {
    kv_append_kernel<64, CT><<<T, kRopeThreads, 0, stream>>>(k, k_stride, v, v_stride, slots, kc, vc, Hkv,
                                                            block_size);
  }
}

void launch_kv_append(const bf16* k, long k_stride, const bf16* v, long v_stride,
                      const int* slots, void* k_cache, void* v_cache, int T, int Hkv, int D,
                      int block_size, hipStream_t stream, int kv_fp8) {
  if (T <= 0) return;
  if (kv_fp8)
    run_kv_append<fp8_t>(k, k_stride, v, v_stride, slots, k_cache, v_cache, T, Hkv, D, block_size, stream);
  else
    run_kv_append<bf16>(k, k_stride, v, v_stride, slots, k_cache, v_cache, T, Hkv, D, block_size, stream);
}

}  // namespace bfly
