// Attention kernels (K3 flash prefill, K4 paged decode, split-K combine) for GQA, head_dim 128.
//
// Decode (attn_decode_kernel): one workgroup per (context split, kv head, sequence), 4 waves
// that walk the split's KV pages round-robin. The whole query group of a kv head (Hq/Hkv <= 16
// rows, padded to 16) rides in ONE mfma_f32_16x16x32_bf16 B operand, so every K/V byte
// streamed from HBM feeds all query heads that share it. K/V go straight to VGPRs (decode
// row of cdna_hip_programming.md §5 table); no LDS round trip.
//   S^T = K . Q^T  ("swapped", K is the A operand): lane column = query row, so the softmax
//   state (m, l) is per lane and the P^T tile is already in the B-operand layout of the PV
//   product O^T = V^T . P^T. The key order inside each 16x16 S tile is chosen by which K row
//   each lane loads (sigma below) so that the 8 keys a lane holds for the PV step are 8
//   CONSECUTIVE keys: with V^T pages ([D][BS], written transposed by rope_kv) the PV A
//   operand is then one 16-B load.
//   Split-K over the context (flash-decoding) with an f32 partial combine kernel.
//   The cache may hold FP8 e4m3 instead of bf16 (bfly_kv.h): half the bytes per page, widened
//   to bf16 in registers before the same MFMAs.
//
// Prefill (attn_prefill_persist_kernel): causal varlen flash attention. Workgroup = 256 query rows
// of one head (8 waves x 32 rows, 2 waves per SIMD), KV tiles of 64 keys staged by LDS-DMA
// into a 4-deep ring of XOR-swizzled LDS images (cdna_hip_programming.md T10 image (b)): K is
// read by ds_read_b128 as the 32x32x16 A operand of S^T = K . Q^T, V by ds_read_b64_tr_b16 as
// the A operand of O^T = V^T . P^T; the S^T accumulator is converted in registers into the
// P^T B operand (§3 "An accumulator tile as the next MFMA's operand").
#include <type_traits>

#include "bfly_common.h"
#include "bfly_kernels.h"
#include "bfly_kv.h"

namespace bfly {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4* lds_s4_ptr;

constexpr int kAttnThreads = 256;
constexpr float kNegInf = -INFINITY;

// ---------------------------------------------------------------------------------------
// Decode
// ---------------------------------------------------------------------------------------
template <int D, int BS, typename CT>
__global__ void __launch_bounds__(kAttnThreads)
attn_decode_kernel(const bf16* __restrict__ q, long q_stride, const CT* __restrict__ k_cache,
                   const CT* __restrict__ v_cache, const int* __restrict__ block_tables,
                   int bt_stride, const int* __restrict__ ctx_lens, int Hq, int Hkv,
                   float scale_log2, int part_tokens, bf16* __restrict__ out,
                   float* __restrict__ part_o, float* __restrict__ part_ml) {
  static_assert(D == 128 && BS == 32, "decode kernel is specialised for D=128, BS=32");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int s = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int nsplit = gridDim.x;
  const int G = Hq / Hkv;
  const int ctx = ctx_lens[b];
  const int tok0 = s * part_tokens;
  const int tok1 = min(ctx, tok0 + part_tokens);
  const long part_base = ((long)(b * Hkv + h) * nsplit + s);

  __shared__ float s_o[4][8][4][64];
  __shared__ float s_m[4][16], s_l[4][16];

  if (tok0 >= tok1) {  // empty split: mark it so the combine skips it
    if (nsplit > 1 && threadIdx.x < 16) {
      part_ml[(part_base * 16 + threadIdx.x) * 2 + 0] = kNegInf;
      part_ml[(part_base * 16 + threadIdx.x) * 2 + 1] = 0.f;
    }
    return;
  }

  const int g = lane >> 4, r = lane & 15;
  // d permutation: sub-step ds, lane group g, element j hold d = 32 ds + 8 g + j, so each K
  // load instruction reads 64 contiguous bytes of every key row (full cache-line pairs).
  // FP8 rows are 128 B: there a lane loads 16 B covering TWO sub-steps,
  // d = 64 (ds >> 1) + 16 g + 8 (ds & 1) + j, again 64 contiguous bytes per row and load.
  // (Any d order works as long as Q uses the same one: QK^T sums over d.)
  constexpr bool kF8 = sizeof(CT) == 1;
  auto d_off = [&](int ds) { return kF8 ? 64 * (ds >> 1) + 16 * g + 8 * (ds & 1) : 32 * ds + 8 * g; };
  // Q^T fragment (B operand): lane holds Q[row r][d]; rows >= G are zero.
  bf16x8 qf[4];
  const int qr = r < G ? r : 0;
  const bf16* qp = q + (long)b * q_stride + (long)(h * G + qr) * D;
#pragma unroll
  for (int ds = 0; ds < 4; ++ds) {
    qf[ds] = *reinterpret_cast<const bf16x8*>(qp + d_off(ds));
    if (r >= G) qf[ds] = bf16x8{};
  }

  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = kNegInf, l = 0.f;

  const int p0 = tok0 / BS, p1 = (tok1 + BS - 1) / BS;
  const int* bt = block_tables + (long)b * bt_stride;

  // K rows: tile kt, lane row r -> key sigma(kt, r) = 8*(r>>2) + 4*kt + (r&3)
  // K/V are loaded raw (bf16, or FP8 at half the bytes) and widened to bf16 right before
  // their MFMA, so the prefetched page costs half the VGPRs with an FP8 cache
  typedef typename KV<CT>::raw_t raw_t;
  auto load_page = [&](int p, raw_t (&kf)[2][4], raw_t (&vf)[8]) {
    const long blk = bt[p];
    const CT* kb = k_cache + ((blk * Hkv + h) * BS) * D;
    const CT* vb = v_cache + (blk * Hkv + h) * (long)D * BS;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int key = 8 * (r >> 2) + 4 * kt + (r & 3);
#pragma unroll
      for (int ds = 0; ds < 4; ++ds)
        if constexpr (kF8) {
          if (ds & 1) continue;
          const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(kb + key * D + d_off(ds)));
          kf[kt][ds] = raw_t{w[0], w[1]};
          kf[kt][ds + 1] = raw_t{w[2], w[3]};
        } else {
          kf[kt][ds] = KV<CT>::ld(kb + key * D + d_off(ds));
        }
    }
    // V^T rows: d = 16dt + r, keys 8g .. 8g+7
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vf[dt] = KV<CT>::ld(vb + (16 * dt + r) * BS + 8 * g);
  };
  auto compute_page = [&](int p, const raw_t (&kf)[2][4], const raw_t (&vf)[8]) {
    f32x4 st[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      st[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 4; ++ds) st[kt] = mfma16(KV<CT>::widen(kf[kt][ds]), qf[ds], st[kt]);
    }
    // st[kt][i] = S[key = p*BS + 8g + 4kt + i][query r]
    float x[8];
    float tmax = kNegInf;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = p * BS + 8 * g + 4 * kt + i;
        const float v = key < tok1 ? st[kt][i] * scale_log2 : kNegInf;
        x[kt * 4 + i] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float mb = mn == kNegInf ? 0.f : mn;
    const float alpha = exp2f(m - mb);
    bf16x8 pb;
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float pv = exp2f(x[j] - mb);
      ps += pv;
      pb[j] = f2bf(pv);
    }
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      o[dt] *= alpha;
      o[dt] = mfma16(KV<CT>::widen(vf[dt]), pb, o[dt]);
    }
  };

  // software pipeline over this wave's pages (p0 + wid, +4, ...): the next page's K/V loads
  // are in flight while the current page is computed; two named register sets (rule 20).
  raw_t kA[2][4], vA[8], kB[2][4], vB[8];
  int p = p0 + wid;
  if (p < p1) load_page(p, kA, vA);
  if constexpr (sizeof(CT) == 2) {
    while (p < p1) {
      if (p + 4 < p1) load_page(p + 4, kB, vB);
      compute_page(p, kA, vA);
      p += 4;
      if (p >= p1) break;
      if (p + 4 < p1) load_page(p + 4, kA, vA);
      compute_page(p, kB, vB);
      p += 4;
    }
  } else {
    // FP8 pages are half the bytes: keep TWO pages in flight (three register sets in
    // rotation, the VGPRs of 1.5 bf16 sets) so the bytes in flight per wave, which bound a
    // latency-limited stream, match the bf16 kernel's
    raw_t kC[2][4], vC[8];
    if (p + 4 < p1) load_page(p + 4, kB, vB);
    while (p < p1) {
      if (p + 8 < p1) load_page(p + 8, kC, vC);
      compute_page(p, kA, vA);
      p += 4;
      if (p >= p1) break;
      if (p + 8 < p1) load_page(p + 8, kA, vA);
      compute_page(p, kB, vB);
      p += 4;
      if (p >= p1) break;
      if (p + 8 < p1) load_page(p + 8, kB, vB);
      compute_page(p, kC, vC);
      p += 4;
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  // Merge the 4 waves: o[dt][i] = O[query r][d = 16dt + 4g + i]
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_o[wid][dt][i][lane] = o[dt][i];
  if (g == 0) {
    s_m[wid][r] = m;
    s_l[wid][r] = l;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * D; e += kAttnThreads) {
    const int qr = e / D, d = e % D;
    if (qr >= G) continue;
    float M = kNegInf;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, s_m[w][qr]);
    const float Mb = M == kNegInf ? 0.f : M;
    float L = 0.f, O = 0.f;
    const int dt = d >> 4, i = d & 3, ln = qr + 16 * ((d & 15) >> 2);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = exp2f(s_m[w][qr] - Mb);
      L += f * s_l[w][qr];
      O += f * s_o[w][dt][i][ln];
    }
    if (nsplit == 1) {
      out[((long)b * Hq + h * G + qr) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      part_o[(part_base * 16 + qr) * D + d] = O;
      if (d == 0) {
        part_ml[(part_base * 16 + qr) * 2 + 0] = M;
        part_ml[(part_base * 16 + qr) * 2 + 1] = L;
      }
    }
  }
}

// One workgroup per (query row, kv head, sequence); thread = head dim element. The split
// (max, sum) pairs are loaded by all threads at once into LDS and reduced by one wave; every
// thread then streams its column of the split outputs with 4 loads in flight. (The first
// version reduced the pairs in thread 0 with dependent global loads: 2 x nsplit load latencies,
// 4.8 us for 5 splits at B = 1 — profiles/r6_latency.md.)
template <int D>
__global__ void __launch_bounds__(D)
attn_decode_combine_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                           int nsplit, int Hq, int Hkv, bf16* __restrict__ out) {
  static_assert(D >= 64, "one full wave reduces the split pairs");
  __shared__ float s_m[256], s_l[256], s_w[256];
  __shared__ float s_inv;
  const int qr = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int G = Hq / Hkv;
  const long base = (long)(b * Hkv + h) * nsplit;
  const int d = threadIdx.x;
  const int ns = nsplit < 256 ? nsplit : 256;
  for (int s = d; s < ns; s += D) {
    const float2 ml = *reinterpret_cast<const float2*>(part_ml + ((base + s) * 16 + qr) * 2);
    s_m[s] = ml.x;
    s_l[s] = ml.y;
  }
  __syncthreads();
  if (d < 64) {
    float M = kNegInf;
    for (int s = d; s < ns; s += 64) M = fmaxf(M, s_m[s]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    const float Mb = M == kNegInf ? 0.f : M;
    float L = 0.f;
    for (int s = d; s < ns; s += 64) {
      const float ms = s_m[s];
      const float w = ms == kNegInf ? 0.f : exp2f(ms - Mb);
      s_w[s] = w;
      L += w * s_l[s];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) L += __shfl_xor(L, o, 64);
    if (d == 0) s_inv = L > 0.f ? 1.f / L : 0.f;
  }
  __syncthreads();
  const float* po = part_o + (base * 16 + qr) * D + d;
  const long sstride = 16L * D;
  float O = 0.f;
  int s = 0;
  for (; s + 4 <= ns; s += 4) {
    float x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = po[(s + j) * sstride];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float w = s_w[s + j];
      O += w != 0.f ? w * x[j] : 0.f;   // empty splits wrote no output (it may be poison)
    }
  }
  for (; s < ns; ++s) {
    const float w = s_w[s];
    if (w != 0.f) O += w * po[s * sstride];
  }
  out[((long)b * Hq + h * G + qr) * D + d] = f2bf(O * s_inv);
}

// ---------------------------------------------------------------------------------------
// Prefill
// ---------------------------------------------------------------------------------------
// 256 query rows (8 waves x 32) and an S-deep 32 KiB-per-tile K/V ring (S = 3 by default: with
// the VALU trimmed, 3 deep is 1-2 % faster than 4). Measured alternative: 128 rows / 2 stages
// (two workgroups per CU, uncoupled barriers) is 6-15 % slower: one tile of compute does not
// hide the K/V fetch (profiles/r1_attn_prefill_valu_trim.log).
constexpr int kPfBQ = 256, kPfBKV = 64, kPfWaves = kPfBQ / 32;
constexpr int kPfIters = 16 / kPfWaves;   // 16 pieces of 4 key rows per K (and V) tile
constexpr int kPfThreads = kPfWaves * 64;
constexpr int kPfLPW = 2 * kPfIters;      // LDS-DMA instructions per wave per staged tile

// Byte offset of 16-B chunk `ch` (0..15) of row `row` in a [rows][128 x bf16] LDS image
// (T10 image (b): conflict-free for 32x32x16 row reads and for the transposed reads).
__device__ __forceinline__ int pf_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int pf_off(int row, int ch) { return row * 256 + 16 * (ch ^ pf_swz(row)); }

// PAD: the first read of an MFMA accumulator — 12 wait states inside the string (8-pass XDL D
// -> VALU read; hipcc pads no hazard whose consumer is inside an asm string). volatile keeps
// the later reads of the same accumulator behind it.
template <bool PAD = false>
__device__ __forceinline__ float pf_max3(float a, float b, float c) {
  float r;
  if constexpr (PAD)
    asm volatile("s_nop 11\n\tv_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  else
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

typedef __attribute__((address_space(3))) void* pf_lds_t;
typedef __attribute__((address_space(1))) void* pf_gbl_t;

template <int N>
__device__ __forceinline__ void pf_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until this wave's DMA pieces of a tile landed, leaving `after` later tiles in flight
__device__ __forceinline__ void pf_wait_tiles(int after) {
  if (after >= 3) pf_vm_wait<3 * kPfLPW>();
  else if (after == 2) pf_vm_wait<2 * kPfLPW>();
  else if (after == 1) pf_vm_wait<kPfLPW>();
  else pf_vm_wait<0>();
}

// S^T tiles of one 64-key tile: s[kt][r] = S[key = kv0 + 32kt + (r&3) + 8(r>>2) + 4hi][query c]
__device__ __forceinline__ void pf_qk(const char* kb, const bf16x8 (&qf)[8], int lane,
                                      f32x16 (&s)[2]) {
  const int hi = lane >> 5, c = lane & 31;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    s[kt] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + pf_off(c, 2 * ks + hi) + kt * 32 * 256);
      s[kt] = mfma32(kf, qf[ks], s[kt]);
    }
  }
}

// Row max of a tile's raw scores (masked first on diagonal / ragged tiles): 4 independent
// v_max3 chains (fmaxf on MFMA results would add canonicalising v_max_f32 per element under
// this build's float flags), then the other half-wave's keys by v_permlane32_swap instead of an
// LDS bpermute round trip. Returns the max in the scaled log2 domain. The mask compares each
// element's compile-time key offset with ONE per-lane limit (the last visible key relative
// to the tile and the lane's half): a compare and a select per element, no per-element
// index math or scalar mask merging.
template <bool MASK>
__device__ __forceinline__ float pf_tile_max(f32x16 (&s)[2], int lim, float scale_log2) {
  // The v_max3 below are inline asm, and hipcc pads no hazard whose consumer is inside an asm
  // string: read straight off the accumulators they raced the MFMAs' write-back (8-pass XDL D
  // -> VALU read needs 12 wait states; cdna_hip_programming.md §5.7 item 2). The row max then
  // came from stale values on some waves of some launches — finite, rounding-level different
  // outputs from launch to launch on every unmasked tile. The first read of each accumulator
  // carries the wait states in its own string (pf_max3<true>); every later read is ordered
  // behind it (volatile) — no register copies, 2 x 12 states per tile.
  if (MASK) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        s[kt][r] = (32 * kt + (r & 3) + 8 * (r >> 2)) <= lim ? s[kt][r] : kNegInf;
  }
  float tc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int kt = c >> 1, r0 = 8 * (c & 1);
    // c = 0 / 2: the first reads of s[0] / s[1] (padded; the masked path reads the select's
    // outputs instead, which the compiler padded)
    tc[c] = (c & 1) ? pf_max3(s[kt][r0], s[kt][r0 + 1], s[kt][r0 + 2])
                    : pf_max3<!MASK>(s[kt][r0], s[kt][r0 + 1], s[kt][r0 + 2]);
    tc[c] = pf_max3(tc[c], s[kt][r0 + 3], s[kt][r0 + 4]);
    tc[c] = pf_max3(tc[c], s[kt][r0 + 5], s[kt][r0 + 6]);
    tc[c] = pf_max3(tc[c], s[kt][r0 + 7], tc[c]);
  }
  float tmax = pf_max3(pf_max3(tc[0], tc[1], tc[2]), tc[3], tc[3]);
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tmax), __float_as_uint(tmax), false, false);
  return pf_max3(__uint_as_float(sw[0]), __uint_as_float(sw[1]), __uint_as_float(sw[1])) * scale_log2;  // scale > 0
}

// P^T = exp2(S * scale - m) as bf16 MFMA B fragments (one FMA and a bare v_exp_f32 per element:
// no denormal range fix-up, p underflowing to 0 is what softmax wants); returns the row sum.
__device__ __forceinline__ float pf_exp(const f32x16 (&s)[2], float scale_log2, float mb,
                                        bf16x8 (&pb)[2][2]) {
  float ps = 0.f;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][8 * h + j], scale_log2, -mb));
        ps += pv;
        pb[kt][h][j] = f2bf(pv);
      }
  return ps;
}

// O^T[d][q] += V^T[d][key] P^T[key][q]; the A operand comes from transposed LDS reads.
__device__ __forceinline__ void pf_pv(const char* vb, const bf16x8 (&pb)[2][2], int lane,
                                      f32x16 (&o)[4]) {
  const int hi = lane >> 5, tq = (lane & 15) >> 2, tp = lane & 3, tg = (lane >> 4) & 1;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int ch = 4 * dt + 2 * tg + (tp >> 1);
    const int vlo = pf_off(4 * hi + tq, ch) + 8 * (tp & 1), vhi = pf_off(4 * hi + tq + 8, ch) + 8 * (tp & 1);
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rows = (32 * kt + 16 * h) * 256;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(vb + vlo + rows));
        const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(vb + vhi + rows));
        // Assemble the fragment as whole dwords (element-wise bf16 inserts from the
        // v4i16 result were miscompiled: hipcc kept only the low dword and duplicated it).
        const u32x2 a2 = __builtin_bit_cast(u32x2, lo);
        const u32x2 b2 = __builtin_bit_cast(u32x2, hi4);
        const u32x4 w4 = {a2.x, a2.y, b2.x, b2.y};
        const bf16x8 vf = __builtin_bit_cast(bf16x8, w4);
        o[dt] = mfma32(vf, pb[kt][h], o[dt]);
      }
  }
}

// K/V tile staging by buffer_load ... lds: the buffer descriptor (SGPRs) starts at the tile's
// first key row and ends at the chunk's last one, so per tile only scalar work moves the
// window, the per-lane byte offsets stay constant (computed once), and rows past the end read
// as zeros (masked anyway) instead of needing a per-lane clamp. (The 64-bit per-lane address
// math of global_load_lds cost ~45 VALU per tile, next to ~200 of softmax.)
struct PfDma {
  int k[kPfIters], v[kPfIters];   // per-lane byte offsets of the lane's 16 B in each piece
};

__device__ __forceinline__ PfDma pf_dma_offsets(long k_stride, long v_stride, int wid, int lane) {
  PfDma d;
#pragma unroll
  for (int i = 0; i < kPfIters; ++i) {
    const int row = (i * kPfWaves + wid) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ pf_swz(row);
    d.k[i] = (int)((row * k_stride + ch * 8) * 2);
    d.v[i] = (int)((row * v_stride + ch * 8) * 2);
  }
  return d;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pf_rsrc(const bf16* base, long rows, long stride) {
  const long bytes = rows * stride * 2;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}

__device__ __forceinline__ void pf_stage_buf(const bf16* __restrict__ k, long k_stride,
                                             const bf16* __restrict__ v, long v_stride, int s0, int L,
                                             int kh, int t, char* kb, int wid, const PfDma& d) {
  const long r0 = (long)s0 + (long)t * kPfBKV;
  const long rows = L - t * kPfBKV;
  const auto rk = pf_rsrc(k + r0 * k_stride + (long)kh * 128, rows, k_stride);
  const auto rv = pf_rsrc(v + r0 * v_stride + (long)kh * 128, rows, v_stride);
#pragma unroll
  for (int i = 0; i < kPfIters; ++i) {
    const int piece = i * kPfWaves + wid;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (pf_lds_t)(kb + piece * 1024), 16, d.k[i], 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (pf_lds_t)(kb + kPfBKV * 256 + piece * 1024), 16, d.v[i], 0, 0, 0);
  }
}

// Deferred rescale threshold (log2 units): a tile whose row max exceeds the running max by at
// most this much keeps the old max, so P stays <= 2^8 and the O rescale (64 multiplies per
// lane) is skipped; the decision is wave-uniform and taken before the tile is exponentiated
// (cdna_hip_programming.md T13).
constexpr float kPfRescaleThr = 8.f;


// ---------------------------------------------------------------------------------------
// Persistent prefill: one workgroup per CU walks the (query block, sequence, head) items in
// heaviest-first order (item i: query block index descending, then sequence, then head, so the
// 8 query heads of a kv head run side by side and share K/V in L2), i = blockIdx.x + j * grid.
// The K/V ring runs ACROSS items: the tiles of the next item are staged while the current
// item's last tiles are computed, and no workgroup launch, Q/ring prologue or grid tail sits
// between items. Short prompts gain most (a 1024-token causal block is 4-16 tiles of work next
// to a fixed per-workgroup start): 423 / 583 / 804 -> 663 / 862 / 925 TF/s at 16x1024 / 4x4096 /
// 1x16384 tokens against one workgroup per item (profiles/r2_attn_prefill_persistent.log).
// Per tile: S^T = K Q^T on 32x32x16 MFMAs (the lane owns one query column: row max/sum are
// lane-local plus one swap), P^T built in registers from the accumulator, O^T += V^T P^T with V
// fed by transposed LDS reads (ds_read_b64_tr_b16). The loop is VALU-bound next to its MFMAs, so
// the VALU is trimmed: buffer-descriptor K/V staging (scalar tile windows), the deferred O
// rescale, and s_setprio 1 for waves 4-7 (which lose VALU arbitration to their older SIMD
// partners). The wave-local vmcnt wait counts the tiles issued after the consumed one (later
// stores and Q loads only make the wait conservative).
// Measured and dropped (profiles/r2_attn_prefill_variants*.log, r2_attn_prefill_wide_variant.log):
// a 5-stage ring (-7 % on 16k tokens), waves 4-7 running PV one tile late (-15..-25 %), a
// one-tile software pipeline of QK(t+1) beside softmax(t) (spills at 256 VGPRs, -35 %), a
// 4-wave x 64-row layout sharing K/V fragments (-25..-35 %), row sums on the matrix core (+-1 %),
// and the round-1 non-persistent kernel (one workgroup per item; 16-40 % slower).
// Round 3 (profiles/r3_attn_prefill_variants.log): the XCD-aware item walk (+5..10 %; the 8
// query heads of a kv head had landed on 8 different L2s) and a wave-uniform wid (+1..3 %)
// are kept; measured and dropped: 4 or 5 ring slots (equal), a one-wave-per-SIMD 4 x 64-row
// kernel with two q-blocks pipelined inside the wave (-25..-65 %: the compiler puts every MFMA
// result in AGPRs above 256 registers and serialises the LDS reads), K/V LDS-DMA as inline asm
// (drops the compiler's per-tile vmcnt(0) before PV, yet -2 %), and Q rows staged by LDS-DMA
// with position-counted vmcnt waits and fixed-count buffer stores (-1..-6 %).
// ---------------------------------------------------------------------------------------
struct PfItem {
  int valid, rows, ntiles;  // valid: item index in range; rows: query rows to write (q0 < L);
  int s0, L, sk0, Lk, q0, h, kh;   // ntiles: K/V tiles (0 with no keys: O = 0, lse = -inf)
};

__device__ __forceinline__ PfItem pf_item(int i, int nqb, int nseq, int Hq, int Hkv,
                                          const int* __restrict__ cu_seqlens, const int* __restrict__ cu_k,
                                          bool causal) {
  PfItem it{};
  const int per = nseq * Hq;
  if (i >= nqb * per) return it;
  it.valid = 1;
  const int qr = i / per, rem = i - qr * per;
  const int seq = rem / Hq;
  it.h = rem - seq * Hq;
  it.kh = it.h / (Hq / Hkv);
  it.s0 = cu_seqlens[seq];
  it.L = cu_seqlens[seq + 1] - it.s0;
  it.sk0 = cu_k[seq];
  it.Lk = cu_k[seq + 1] - it.sk0;
  it.q0 = (causal ? nqb - 1 - qr : qr) * kPfBQ;
  if (it.q0 >= it.L) return it;   // rows = ntiles = 0
  it.rows = 1;
  if (it.Lk <= 0) return it;      // no keys (an empty key chunk): rows written, no tiles
  const int kv_end = causal ? min(it.Lk, it.q0 + kPfBQ) : it.Lk;
  it.ntiles = (kv_end + kPfBKV - 1) / kPfBKV;
  return it;
}

template <int D, int S, bool TR = false>
__global__ void __launch_bounds__(kPfThreads)
attn_prefill_persist_kernel(const bf16* __restrict__ q, long q_stride, const bf16* __restrict__ k,
                            long k_stride, const bf16* __restrict__ v, long v_stride,
                            const int* __restrict__ cu_seqlens, const int* __restrict__ cu_k, int nseq,
                            int nqb, int Hq, int Hkv, float scale_log2, int causal,
                            bf16* __restrict__ out, long o_stride, float* __restrict__ lse, int xr) {
  static_assert(D == 128 && S >= 2, "persistent prefill kernel is specialised for D=128");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE_BYTES = 2 * kPfBKV * D * 2;
  constexpr int AHEAD = S - 1;
  // wid through readfirstlane: the compiler then knows every per-wave branch on it is
  // wave-uniform (1-3 % faster: profiles/r3_attn_prefill_variants.log)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hi = lane >> 5, c = lane & 31;
  const bool cz = causal != 0;
  const int G = gridDim.x;
  if (wid >= kPfWaves / 2) __builtin_amdgcn_s_setprio(1);
  const PfDma dma = pf_dma_offsets(k_stride, v_stride, wid, lane);

  // consume cursor (C: the item being computed; items with query rows) and issue cursor
  // (I: the item whose next tile is staged; items with K/V tiles)
  auto next_item = [&](int& idx, PfItem& it, bool need_tiles) {
    do {
      idx += G;
      it = pf_item(idx, nqb, nseq, Hq, Hkv, cu_seqlens, cu_k, cz);
    } while (it.valid && (need_tiles ? it.ntiles == 0 : it.rows == 0));
  };
  // XCD-aware walk: the dispatcher deals workgroups round-robin over the 8 XCDs (b % 8 share
  // an L2); renumbered, each XCD's workgroups take consecutive items, i.e. the query heads
  // of one kv head side by side, so their K/V tiles are fetched into ONE L2
  int ci = (xr ? xcd_remap((int)blockIdx.x, G) : (int)blockIdx.x) - G;
  PfItem C{};
  next_item(ci, C, false);
  if (!C.valid) return;
  int ii = ci, it_t = 0;
  PfItem I = C;
  if (I.ntiles == 0) next_item(ii, I, true);
  int issued = 0, consumed = 0, islot = 0, cslot = 0;
  // TR (BFLY_ATTN_TRACE=1, tools/attn_trace.py): wave 0 stamps s_memtime at the item phases
  // into the LSE buffer instead of writing LSE / O
  int trj = 0;
  auto trace = [&](int e) {
    if constexpr (TR) {
      if (wid == 0 && lane == 0 && trj < 32)
        reinterpret_cast<long long*>(lse)[((long)blockIdx.x * 32 + trj) * 8 + e] = (long long)__builtin_amdgcn_s_memtime();
    }
  };
  auto issue_one = [&]() {
    if (!I.valid) return;
    pf_stage_buf(k, k_stride, v, v_stride, I.sk0, I.Lk, I.kh, it_t, smem + islot * STAGE_BYTES, wid, dma);
    if (++islot == S) islot = 0;
    ++issued;
    if (++it_t == I.ntiles) {
      it_t = 0;
      next_item(ii, I, true);
    }
  };
#pragma unroll
  for (int st = 0; st < AHEAD; ++st) issue_one();

  // Q fragments of this lane's query row of item X (rows clamped into the sequence)
  auto load_q = [&](const PfItem& X, bf16x8 (&qd)[8]) {
    const int qrow = X.q0 + 32 * wid + c;
    const int qr = qrow < X.L ? qrow : X.L - 1;
    const bf16x8* qp = reinterpret_cast<const bf16x8*>(q + (long)(X.s0 + qr) * q_stride + (long)X.h * D + 8 * hi);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qd[ks] = qp[2 * ks];
  };
  while (true) {
    // ---- item start: Q fragments and softmax state of this lane's query row. The next item
    // is looked up (scalar loads of cu_seqlens) during this item's last tile, so that latency
    // does not sit between two items. (Loading its Q there as well, into the dead qf, makes
    // the allocator spill: measured and dropped.)
    trace(0);
    const int qrow = C.q0 + 32 * wid + c;
    bf16x8 qf[8];
    load_q(C, qf);
    int cin = ci;
    PfItem Cn{};
    auto prefetch_next = [&]() { next_item(cin, Cn, false); };
    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16{};
    float m = kNegInf, lsum = 0.f;
    const int wave_qmax = C.q0 + 32 * wid + 31;
    const int last_key = cz ? min(qrow, C.Lk - 1) : C.Lk - 1;
    for (int t = 0; t < C.ntiles; ++t) {
      // this tile landed; the tiles issued after it may still fly
      pf_wait_tiles(min(issued - consumed - 1, AHEAD - 1));
      if (t == 0) trace(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t == 0) trace(2);
      if (t == C.ntiles - 1) trace(3);
      issue_one();                      // into the slot every wave finished reading last tile
      const char* kb = smem + cslot * STAGE_BYTES;
      const int kv0 = t * kPfBKV;
      if (t == C.ntiles - 1) prefetch_next();
      if (!(cz && kv0 > wave_qmax)) {
        f32x16 sc[2];
        pf_qk(kb, qf, lane, sc);
        const bool need_mask = (cz && kv0 + kPfBKV - 1 > C.q0 + 32 * wid) || kv0 + kPfBKV > C.Lk;
        const int lim = last_key - kv0 - 4 * hi;
        const float tmax = need_mask ? pf_tile_max<true>(sc, lim, scale_log2) : pf_tile_max<false>(sc, lim, scale_log2);
        float alpha = 1.f;
        if (!__all(tmax - m <= kPfRescaleThr)) {
          const float mn = fmaxf(m, tmax);
          const float mb = mn == kNegInf ? 0.f : mn;
          alpha = __builtin_amdgcn_exp2f(m - mb);
          m = mn;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        }
        const float mb = m == kNegInf ? 0.f : m;
        bf16x8 pb[2][2];
        lsum = lsum * alpha + pf_exp(sc, scale_log2, mb, pb);
        pf_pv(kb + kPfBKV * 256, pb, lane, o);
      }
      if (++cslot == S) cslot = 0;
      ++consumed;
    }
    if (C.ntiles == 0) prefetch_next();
    // ---- item end: normalise and store this lane's query row (no barrier: the next item's
    // first wait + barrier orders the ring; these stores only make that wait conservative)
    trace(4);
    lsum += __shfl_xor(lsum, 32, 64);
    if (!TR && qrow < C.L) {
      if (lse != nullptr && hi == 0)
        lse[(long)(C.s0 + qrow) * Hq + C.h] = lsum > 0.f ? (m + __log2f(lsum)) * 0.69314718055994531f : kNegInf;
      const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
      bf16* op = out + (long)(C.s0 + qrow) * o_stride + (long)C.h * D;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          bf16x4 w;
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] = f2bf(o[dt][4 * a + j] * inv);
          *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * a + 4 * hi) = w;
        }
    }
    trace(5);
    if constexpr (TR) {
      if (wid == 0 && lane == 0 && trj < 32)
        reinterpret_cast<long long*>(lse)[((long)blockIdx.x * 32 + trj) * 8 + 6] = C.ntiles;
    }
    ++trj;
    ci = cin;
    C = Cn;
    if (!C.valid) break;
  }
}

// ---------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------
int attn_decode_splits(int max_ctx, int part_tokens) {
  return (max_ctx + part_tokens - 1) / part_tokens;
}

// Context split size, from a split-size sweep on MI355X (tools/bench_attn.py --parts): aim at
// ~256 (b, kv-head, split) workgroups (one per CU), splitting the context evenly and never
// below 256 tokens per split; a single split skips the combine launch entirely.
//   B=64 Hkv=8 ctx 1K: 1 split 46 us (2 splits 53);  B=8 ctx 4K: 4 splits 30 us (16: 38);
//   B=64 Hkv=1: 4 splits 13.5 us (8: 15.4);        B=1 ctx 8K: 32 splits 27 us (64: 43).
int attn_decode_part_tokens(int B, int Hkv, int max_ctx) {
  const int pairs = B * Hkv > 0 ? B * Hkv : 1;
  const int splits = (256 + pairs - 1) / pairs;
  int part = (max_ctx + splits - 1) / splits;
  part = (part + 31) / 32 * 32;
  if (splits > 1 && part < 256) part = 256;
  if (part < 32) part = 32;
  while ((max_ctx + part - 1) / part > 256) part += 32;   // combine kernel: <= 256 splits
  return part;
}

int launch_attn_decode(const bf16* q, long q_stride, const void* k_cache, const void* v_cache,
                       const int* block_tables, int bt_stride, const int* ctx_lens, int B, int Hq,
                       int Hkv, int D, int block_size, float scale, int max_ctx, int part_tokens,
                       bf16* out, float* part_o, float* part_ml, hipStream_t stream, int kv_fp8) {
  if (B <= 0) return 0;
  if (D != 128 || block_size != 32 || Hq % Hkv != 0 || Hq / Hkv > 16) return -1;
  if (part_tokens <= 0) part_tokens = attn_decode_part_tokens(B, Hkv, max_ctx);
  if (part_tokens % block_size != 0) return -2;
  if (attn_decode_splits(max_ctx, part_tokens) > 256) return -4;
  const int nsplit = attn_decode_splits(max_ctx, part_tokens);
  if (nsplit > 1 && (part_o == nullptr || part_ml == nullptr)) return -3;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(nsplit, Hkv, B);
#define DEC_LAUNCH(CT)                                                                                      \
  attn_decode_kernel<128, 32, CT><<<grid, kAttnThreads, 0, stream>>>(                                        \
      q, q_stride, static_cast<const CT*>(k_cache), static_cast<const CT*>(v_cache), block_tables, bt_stride, \
      ctx_lens, Hq, Hkv, scale_log2, part_tokens, out, part_o, part_ml)
  if (kv_fp8) DEC_LAUNCH(fp8_t);
  else DEC_LAUNCH(bf16);
#undef DEC_LAUNCH
  if (nsplit > 1) {
    // Measured and dropped: merging the splits inside the decode kernel (last arriver, agent-
    // scope release/acquire per workgroup) ran 2x slower than this parallel combine launch
    // (B=64 ctx 1024: 104 vs 53 us); RoPE + KV append fused into the decode kernel ran 1.1 %
    // slower per 70B step than rope_kv + attention and was removed
    // (profiles/r2_fused_decode_rope_ab.log, profiles/r4_fused_decode_rope_ab.log).
    dim3 g2(Hq / Hkv, Hkv, B);
    attn_decode_combine_kernel<128><<<g2, 128, 0, stream>>>(part_o, part_ml, nsplit, Hq, Hkv, out);
  }
  return 0;
}

int launch_attn_prefill(const bf16* q, long q_stride, const bf16* k, long k_stride, const bf16* v,
                        long v_stride, const int* cu_seqlens, int nseq, int max_seqlen, int Hq,
                        int Hkv, int D, float scale, bool causal, bf16* out, long o_stride,
                        hipStream_t stream, const int* cu_k, float* lse) {
  if (nseq <= 0 || max_seqlen <= 0) return 0;
  if (D != 128 || Hq % Hkv != 0) return -1;
  const float scale_log2 = scale * 1.4426950408889634f;
  const int* cuk = cu_k != nullptr ? cu_k : cu_seqlens;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const int nqb = (max_seqlen + kPfBQ - 1) / kPfBQ;
  const long items = (long)nqb * nseq * Hq;
  const int g = (int)(items < ncu ? items : ncu);
  static const bool tr = getenv("BFLY_ATTN_TRACE") != nullptr;
  static const int xr = [] {
    const char* e = getenv("BFLY_ATTN_XCD");
    return e ? atoi(e) : 1;
  }();
  auto launch = [&](auto sc) {
    constexpr int S_ = decltype(sc)::value;
    const size_t lds = (size_t)S_ * 2 * kPfBKV * D * 2;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_prefill_persist_kernel<128, S_>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_prefill_persist_kernel<128, S_, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    if (tr && lse != nullptr)
      attn_prefill_persist_kernel<128, S_, true><<<g, kPfThreads, lds, stream>>>(
          q, q_stride, k, k_stride, v, v_stride, cu_seqlens, cuk, nseq, nqb, Hq, Hkv, scale_log2,
          causal ? 1 : 0, out, o_stride, lse, xr);
    else
      attn_prefill_persist_kernel<128, S_><<<g, kPfThreads, lds, stream>>>(
          q, q_stride, k, k_stride, v, v_stride, cu_seqlens, cuk, nseq, nqb, Hq, Hkv, scale_log2,
          causal ? 1 : 0, out, o_stride, lse, xr);
  };
  launch(std::integral_constant<int, 3>{});   // 3 ring slots: 4 and 5 measured equal
  return 0;
}

// K16: merge a partial attention result over another key chunk into running accumulators
// (context-parallel ring attention): acc_lse' = log(e^acc_lse + e^lse),
// acc_o' = acc_o * e^(acc_lse - acc_lse') + o * e^(lse - acc_lse'). One workgroup of 128
// threads per (token, head) row; rows where both sides are empty (-inf) stay untouched.
__global__ void __launch_bounds__(128)
attn_lse_merge_kernel(float* __restrict__ acc_o, float* __restrict__ acc_lse,
                      const bf16* __restrict__ o, long o_stride, const float* __restrict__ lse,
                      int H) {
  const long row = blockIdx.x;
  const long t = row / H;
  const int h = (int)(row % H), d = threadIdx.x;
  const float a = acc_lse[row], b = lse[row];
  const float mx = fmaxf(a, b);
  if (mx == kNegInf) return;
  const float wa = a == kNegInf ? 0.f : __expf(a - mx);
  const float wb = b == kNegInf ? 0.f : __expf(b - mx);
  const float inv = 1.f / (wa + wb);
  const float ov = bf2f(o[t * o_stride + (long)h * 128 + d]);
  float* ap = acc_o + row * 128 + d;
  *ap = (*ap * wa + ov * wb) * inv;
  __syncthreads();   // every thread read acc_lse[row] before it changes
  if (d == 0) acc_lse[row] = mx + __logf(wa + wb);
}

int launch_attn_lse_merge(float* acc_o, float* acc_lse, const bf16* o, long o_stride,
                          const float* lse, int T, int H, int D, hipStream_t stream) {
  if (D != 128) return -1;
  if ((long)T * H == 0) return 0;
  attn_lse_merge_kernel<<<(unsigned)((long)T * H), 128, 0, stream>>>(acc_o, acc_lse, o, o_stride, lse, H);
  return 0;
}

}  // namespace bfly
