// Paged KV-cache element types (bf16, or FP8 e4m3 for the optional FP8 KV cache).
//
// FP8 is the OCP e4m3fn format that gfx950's conversion instructions and MFMAs use (not the
// MI300 "fnuz" variant), the same as torch.float8_e4m3fn: the engine can read and write the
// cache from PyTorch as well. Values are stored unscaled (range +-448, clamped on the way in);
// decode attention widens them back to bf16 in registers (v_cvt_pk_f32_fp8 + v_cvt_pk_bf16_f32)
// and runs the same bf16 MFMAs, so an FP8 cache halves the KV bytes streamed per decode step.
//
// KV<CT> gives the kernels one interface for both element types:
//   raw_t       what a lane loads for 8 consecutive elements (16 B bf16, 8 B fp8)
//   ld(p)       non-temporal load of 8 elements (decode: KV pages are read once per step)
//   widen(r)    raw_t -> bf16x8 (MFMA operand)
//   store8(p,v) store 8 bf16 values as 8 cache elements
//   store1(p,v) store one bf16 value as one cache element (transposed V scatter)
#pragma once
#include "bfly_common.h"

namespace bfly {

typedef uint8_t fp8_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr float kFp8Max = 448.f;

// Rotate-half RoPE of one pair (x0 at d, x1 at d + D/2) with explicit FMAs, shared by every
// kernel that rotates (rope.hip, the QKV GEMM's seam in gemm.hip): a plain `x0*c - x1*s` leaves
// the contraction choice to the compiler per call site, so two kernels could round differently.
__device__ __forceinline__ void rope_rotate(float x0, float x1, float c, float s, float& o0, float& o1) {
  o0 = __builtin_fmaf(x0, c, -(x1 * s));
  o1 = __builtin_fmaf(x1, c, x0 * s);
}

__device__ __forceinline__ float fp8_clamp(float x) { return fminf(fmaxf(x, -kFp8Max), kFp8Max); }

// 4 floats -> 4 e4m3 bytes (RNE), little-endian in one dword
__device__ __forceinline__ uint32_t fp8_pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(a), fp8_clamp(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(c), fp8_clamp(d), w, true);
  return (uint32_t)w;
}

template <typename CT>
struct KV;

template <>
struct KV<bf16> {
  typedef bf16x8 raw_t;
  static __device__ __forceinline__ raw_t ld(const bf16* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
  }
  static __device__ __forceinline__ bf16x8 widen(raw_t r) { return r; }
  static __device__ __forceinline__ void store8(bf16* p, bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }
  static __device__ __forceinline__ void store1(bf16* p, bf16 v) { *p = v; }
};

template <>
struct KV<fp8_t> {
  typedef u32x2 raw_t;
  static __device__ __forceinline__ raw_t ld(const fp8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
  }
  static __device__ __forceinline__ bf16x8 widen(raw_t r) {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x2 lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)r[i], false);   // bytes 0, 1
      const f32x2 hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)r[i], true);    // bytes 2, 3
      o[4 * i + 0] = f2bf(lo[0]);
      o[4 * i + 1] = f2bf(lo[1]);
      o[4 * i + 2] = f2bf(hi[0]);
      o[4 * i + 3] = f2bf(hi[1]);
    }
    return o;
  }
  static __device__ __forceinline__ void store8(fp8_t* p, bf16x8 v) {
    u32x2 w;
    w[0] = fp8_pack4(bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3]));
    w[1] = fp8_pack4(bf2f(v[4]), bf2f(v[5]), bf2f(v[6]), bf2f(v[7]));
    *reinterpret_cast<u32x2*>(p) = w;
  }
  static __device__ __forceinline__ void store1(fp8_t* p, bf16 v) {
    *p = (fp8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(bf2f(v)), 0.f, 0, false) & 0xff);
  }
};

}  // namespace bfly
