// Shared device helpers for butterfly_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 storage is `__bf16`; arithmetic is f32; f32->bf16 uses the plain cast,
//     which hipcc lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
//   * Memory-bound kernels move 16 B per lane (8 x bf16) per access.
//   * Wave width is 64; the code hard-codes it (warpSize folds to 64 on gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bfly {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of up to 1024 threads. `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Non-temporal 16-byte load for once-read streams (decode weights, KV pages).
__device__ __forceinline__ bf16x8 ld_nt(const bf16x8* p) {
  return __builtin_nontemporal_load(p);
}

// Bijective XCD-aware remap of a linear workgroup id: blocks that the dispatcher deals
// round-robin over the 8 XCDs (b % 8 share an L2) are renumbered so that each XCD gets a
// contiguous range of logical tiles (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// MoE routing of token t from one wave holding expert `lane`'s router logit (E <= 64 experts,
// `live` = lane < E): softmax over all experts, top-K by probability (ties to the lowest
// expert id), the selected weights renormalised to sum 1. Writes gates[t][E] (0 for unselected
// experts), topk_ids[t][K] and topk_w[t][K]. Shared by moe_route_kernel and the add+RMSNorm
// that routes the rows it normalises (norm.hip).
__device__ __forceinline__ void moe_select_topk(float logit, bool live, int lane, int t, int E, int K,
                                                float* __restrict__ gates, int* __restrict__ topk_ids,
                                                float* __restrict__ topk_w) {
  logit = live ? logit : -INFINITY;
  const float mx = wave_max(logit);
  float p = live ? __expf(logit - mx) : 0.f;
  const float den = wave_sum(p);
  float g = 0.f, sel_sum = 0.f;
  int my_rank = -1;                     // this expert's position in the top-k (-1: not selected)
  for (int k = 0; k < K; ++k) {
    float bv = live ? p : -1.f;
    int bi = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    sel_sum += bv / den;
    if (lane == bi) { my_rank = k; g = p / den; p = -1.f; }
  }
  if (!live) return;
  const float w = my_rank >= 0 ? g / sel_sum : 0.f;
  gates[(long)t * E + lane] = w;
  if (my_rank >= 0) {
    topk_ids[(long)t * K + my_rank] = lane;
    topk_w[(long)t * K + my_rank] = w;
  }
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

}  // namespace bfly

#define BFLY_HIP_CHECK(expr)                                                  \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e),       \
              __FILE__, __LINE__);                                            \
    }                                                                         \
  } while (0)
