// Paged-prefix flash attention for chunked prefill (SURVEY.md §2.7-K K3/K4 "paged KV with
// holes").
//
// A mixed serving step prefills a prompt CHUNK of n tokens at positions [st, st + n) of a
// sequence whose first st tokens are already in the paged cache (an earlier chunk, or a
// prefix-cache hit). rope_kv has just appended the chunk's own K/V to the same pages, so every
// key a chunk query may see — the cached prefix AND the causal part of the chunk — lives in the
// paged cache: ONE pass over the sequence's block table computes the whole attention row, with
// no contiguous K/V gather, no second flash pass over the chunk and no log-sum-exp merge.
//
// Workgroup = (16-token query block of one sequence's chunk, kv head), 4 waves. The 16 tokens
// are the 16 columns of the MFMA B operand (one query head per 16x16 tile), so the causal mask
// is one per-lane position compare; wave w owns the query heads w, w + 4 (< G) of the kv head
// and reuses every K / V fragment it loads for both. Structure of the decode kernel
// (attention.hip): S^T = K . Q^T with K as the A operand (key order sigma so that each lane
// ends up with 8 CONSECUTIVE keys), P^T converted in registers into the B operand of
// O^T = V^T . P^T, V^T pages ([D][BS], written transposed by rope_kv) loaded as 16-B A
// fragments; the next page's K/V are in flight while the current one is computed. The four
// waves read the same pages (L1 / L2 hits for three of them). FP8 e4m3 pages are widened to bf16
// in registers (bfly_kv.h).
#include <stdlib.h>

#include <type_traits>

#include "bfly_common.h"
#include "bfly_kernels.h"
#include "bfly_kv.h"

namespace bfly {

namespace {

constexpr int kPgThreads = 256;
constexpr int kPgQ = 16;            // query tokens per workgroup (MFMA columns)
constexpr float kPgNegInf = -INFINITY;

// HPW = query heads per wave (G <= 4 HPW)
template <int D, int BS, typename CT, int HPW>
__global__ void __launch_bounds__(kPgThreads)
attn_prefill_paged_kernel(const bf16* __restrict__ q, long q_stride, const CT* __restrict__ k_cache,
                          const CT* __restrict__ v_cache, const int* __restrict__ tables, int bt_stride,
                          const int* __restrict__ cu_q, const int* __restrict__ positions, int Hq, int Hkv,
                          float scale_log2, bf16* __restrict__ out, long o_stride) {
  static_assert(D == 128 && BS == 32, "paged prefill kernel is specialised for D=128, BS=32");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
  const int G = Hq / Hkv;
  const int row0 = cu_q[s] + qb * kPgQ, rend = min(cu_q[s + 1], row0 + kPgQ);
  if (row0 >= rend) return;
  const int nval = rend - row0;
  const int g = lane >> 4, r = lane & 15;
  // this lane's query token: its position bounds the keys it sees (causal); padding lanes
  // (r >= nval) see none
  const int qpos = r < nval ? positions[row0 + r] : -1;
  const int kmax = positions[rend - 1] + 1;           // keys [0, kmax) of the whole block
  constexpr bool kF8 = sizeof(CT) == 1;
  auto d_off = [&](int ds) { return kF8 ? 64 * (ds >> 1) + 16 * g + 8 * (ds & 1) : 32 * ds + 8 * g; };

  // Q^T fragments (B operand): lane holds Q[token r][head][d]
  bf16x8 qf[HPW][4];
  bool on[HPW];
#pragma unroll
  for (int c = 0; c < HPW; ++c) {
    const int hh = wid + 4 * c;
    on[c] = hh < G;
    const int head = h * G + (on[c] ? hh : 0);
    const bf16* qp = q + (long)(row0 + (r < nval ? r : 0)) * q_stride + (long)head * D;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      qf[c][ds] = *reinterpret_cast<const bf16x8*>(qp + d_off(ds));
      if (r >= nval) qf[c][ds] = bf16x8{};
    }
  }
  f32x4 o[HPW][8];
  float m[HPW], l[HPW];
#pragma unroll
  for (int c = 0; c < HPW; ++c) {
    m[c] = kPgNegInf;
    l[c] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[c][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int* bt = tables + (long)s * bt_stride;
  const int npages = (kmax + BS - 1) / BS;
  typedef typename KV<CT>::raw_t raw_t;
  // plain (cached) loads: the four waves share every page through L1 / L2
  auto ldkv = [&](const CT* p) -> raw_t { return *reinterpret_cast<const raw_t*>(p); };
  auto load_page = [&](int p, raw_t (&kf)[2][4], raw_t (&vf)[8]) {
    const long blk = bt[p];
    const CT* kb = k_cache + ((blk * Hkv + h) * BS) * D;
    const CT* vb = v_cache + (blk * Hkv + h) * (long)D * BS;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int key = 8 * (r >> 2) + 4 * kt + (r & 3);   // sigma: lane ends with 8 consecutive keys
#pragma unroll
      for (int ds = 0; ds < 4; ++ds)
        if constexpr (kF8) {
          if (ds & 1) continue;
          const u32x4 w = *reinterpret_cast<const u32x4*>(kb + key * D + d_off(ds));
          kf[kt][ds] = raw_t{w[0], w[1]};
          kf[kt][ds + 1] = raw_t{w[2], w[3]};
        } else {
          kf[kt][ds] = ldkv(kb + key * D + d_off(ds));
        }
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) vf[dt] = ldkv(vb + (16 * dt + r) * BS + 8 * g);   // V^T rows d
  };
  auto compute_page = [&](int p, const raw_t (&kf)[2][4], const raw_t (&vf)[8]) {
    bf16x8 kw[2][4];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int ds = 0; ds < 4; ++ds) kw[kt][ds] = KV<CT>::widen(kf[kt][ds]);
    bf16x8 pb[HPW];
    float alpha[HPW];
#pragma unroll
    for (int c = 0; c < HPW; ++c) {
      f32x4 st[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        st[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ds = 0; ds < 4; ++ds) st[kt] = mfma16(kw[kt][ds], qf[c][ds], st[kt]);
      }
      // st[kt][i] = S[key = p*BS + 8g + 4kt + i][query r]
      float x[8];
      float tmax = kPgNegInf;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = p * BS + 8 * g + 4 * kt + i;
          const float v = key <= qpos ? st[kt][i] * scale_log2 : kPgNegInf;
          x[kt * 4 + i] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m[c], tmax);
      const float mb = mn == kPgNegInf ? 0.f : mn;
      alpha[c] = exp2f(m[c] - mb);
      float ps = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = exp2f(x[j] - mb);
        ps += pv;
        pb[c][j] = f2bf(pv);
      }
      l[c] = l[c] * alpha[c] + ps;
      m[c] = mn;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const bf16x8 vw = KV<CT>::widen(vf[dt]);
#pragma unroll
      for (int c = 0; c < HPW; ++c) {
        o[c][dt] *= alpha[c];
        o[c][dt] = mfma16(vw, pb[c], o[c][dt]);
      }
    }
  };

  raw_t kA[2][4], vA[8], kB[2][4], vB[8];
  int p = 0;
  if constexpr (HPW == 1) {
    // one head per wave leaves the VGPRs for a third page set: two pages in flight per wave
    // (the per-wave page stream is latency-bound: one workgroup per CU for a single sequence)
    raw_t kC[2][4], vC[8];
    if (p < npages) load_page(p, kA, vA);
    if (p + 1 < npages) load_page(p + 1, kB, vB);
    while (p < npages) {
      if (p + 2 < npages) load_page(p + 2, kC, vC);
      compute_page(p, kA, vA);
      if (++p >= npages) break;
      if (p + 2 < npages) load_page(p + 2, kA, vA);
      compute_page(p, kB, vB);
      if (++p >= npages) break;
      if (p + 2 < npages) load_page(p + 2, kB, vB);
      compute_page(p, kC, vC);
      ++p;
    }
  } else {
    if (p < npages) load_page(p, kA, vA);
    while (p < npages) {
      if (p + 1 < npages) load_page(p + 1, kB, vB);
      compute_page(p, kA, vA);
      if (++p >= npages) break;
      if (p + 1 < npages) load_page(p + 1, kA, vA);
      compute_page(p, kB, vB);
      ++p;
    }
  }
#pragma unroll
  for (int c = 0; c < HPW; ++c) {
    l[c] += __shfl_xor(l[c], 16, 64);
    l[c] += __shfl_xor(l[c], 32, 64);
  }
  if (r >= nval) return;
  // o[c][dt][i] = O[query r][d = 16dt + 4g + i]
#pragma unroll
  for (int c = 0; c < HPW; ++c) {
    if (!on[c]) continue;
    const float inv = l[c] > 0.f ? 1.f / l[c] : 0.f;
    bf16* op = out + (long)(row0 + r) * o_stride + (long)(h * G + wid + 4 * c) * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(o[c][dt][i] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// LDS-staged variant (default). The register kernel above lets every wave fetch every page for
// its own query head, so a page crosses L2 -> CU four times per workgroup, and a workgroup
// serves only 16 query tokens: the prefix is re-read from L2 once per 16 tokens per head
// (measured 94 us per Llama-3-8B layer for a 512-token chunk over a ~1.4k-token prefix, ~125
// TF/s: profiles/r4_traces/). Here the workgroup DMAs each K / V page ONCE into a 3-slot LDS
// ring (global_load_lds, XOR-swizzled on the source so the MFMA fragment reads below are bank-
// conflict free) and every wave reads its fragments from LDS; the 4 waves cover 8 (head, 16-
// token group) column groups: all G heads of the kv head and 8 / G token groups, so a
// workgroup serves 16 * 8 / G query tokens (32 for Llama's G = 4, 16 for G = 8) from one page
// stream. One raw barrier per page: the page issued at step p goes to the slot every wave
// finished reading at step p - 1.
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* pg_lds_t;
typedef __attribute__((address_space(1))) void* pg_gbl_t;

template <int N>
__device__ __forceinline__ void pg_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-B chunk swizzles of the LDS page images (see the bank analysis at each use)
template <typename CT>
__device__ __forceinline__ int pg_swz_k(int key) {
  if constexpr (sizeof(CT) == 2) return (key & 3) | (((key >> 3) & 3) << 2);      // 16 chunks per 256-B row
  else return ((key >> 1) & 1) | (((key >> 3) & 3) << 1);                          // 8 chunks per 128-B row
}
template <typename CT>
__device__ __forceinline__ int pg_swz_v(int d) {
  if constexpr (sizeof(CT) == 2) return (d >> 1) & 3;                              // 4 chunks per 64-B row
  else return (d >> 3) & 1;                                                        // 2 chunks per 32-B row
}

// wait until this wave's DMA pieces of a page landed, leaving `ahead` later pages (PW pieces
// each) in flight
template <int PW>
__device__ __forceinline__ void pg_wait_pages(int ahead) {
  switch (ahead) {
    case 0: pg_vm_wait<0>(); break;
    case 1: pg_vm_wait<PW>(); break;
    case 2: pg_vm_wait<2 * PW>(); break;
    case 3: pg_vm_wait<3 * PW>(); break;
    case 4: pg_vm_wait<4 * PW>(); break;
    case 5: pg_vm_wait<5 * PW>(); break;
    default: pg_vm_wait<6 * PW>(); break;
  }
}

template <int D, int BS, typename CT, int S>
__global__ void __launch_bounds__(kPgThreads)
attn_prefill_paged_lds_kernel(const bf16* __restrict__ q, long q_stride, const CT* __restrict__ k_cache,
                              const CT* __restrict__ v_cache, const int* __restrict__ tables, int bt_stride,
                              const int* __restrict__ cu_q, const int* __restrict__ positions, int Hq, int Hkv,
                              int tg_per_wg, float scale_log2, bf16* __restrict__ out, long o_stride) {
  static_assert(D == 128 && BS == 32, "paged prefill kernel is specialised for D=128, BS=32");
  constexpr bool kF8 = sizeof(CT) == 1;
  constexpr int KB = BS * D * (int)sizeof(CT);        // bytes of one K (or V) page of one kv head
  constexpr int STAGE = 2 * KB;                         // [K image | V image]
  constexpr int LPW = KB / 1024 / 4;                    // DMA instructions per wave per image
  constexpr int RBK = D * (int)sizeof(CT), RBV = BS * (int)sizeof(CT);   // row bytes
  static_assert(S >= 3 && S <= 8, "ring of 3 .. 8 pages");
  extern __shared__ __attribute__((aligned(16))) char smem[];   // S * STAGE bytes
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = blockIdx.y, s = blockIdx.z;
  const int G = Hq / Hkv;
  const int ntok = 16 * tg_per_wg;
  const int row0 = cu_q[s] + blockIdx.x * ntok, rend = min(cu_q[s + 1], row0 + ntok);
  if (row0 >= rend) return;
  const int g = lane >> 4, r = lane & 15;
  auto d_off = [&](int ds) { return kF8 ? 64 * (ds >> 1) + 16 * g + 8 * (ds & 1) : 32 * ds + 8 * g; };

  // column groups j = wid, wid + 4 (< G * tg_per_wg): head j % G, token group j / G
  bf16x8 qf[2][4];
  bool on[2];
  int qpos[2], orow[2], ohead[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int j = wid + 4 * c;
    on[c] = j < G * tg_per_wg;
    const int hh = on[c] ? j % G : 0, tg = on[c] ? j / G : 0;
    const int row = row0 + 16 * tg + r;
    const bool valid = on[c] && row < rend;
    qpos[c] = valid ? positions[row] : -1;          // padding lanes see no key
    orow[c] = valid ? row : -1;
    ohead[c] = h * G + hh;
    const bf16* qp = q + (long)(valid ? row : row0) * q_stride + (long)ohead[c] * D;
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      qf[c][ds] = *reinterpret_cast<const bf16x8*>(qp + d_off(ds));
      if (!valid) qf[c][ds] = bf16x8{};
    }
  }
  f32x4 o[2][8];
  float m[2], l[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    m[c] = kPgNegInf;
    l[c] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[c][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int kmax = positions[rend - 1] + 1;             // keys [0, kmax) of the whole workgroup
  const int npages = min((kmax + BS - 1) / BS, bt_stride);
  // the sequence's block ids in LDS (after the ring): a scalar load per page issue would put
  // its latency between every two pages (the page loop is latency-bound)
  int* lbt = reinterpret_cast<int*>(smem + S * STAGE);
  {
    const int* bt = tables + (long)s * bt_stride;
    for (int i = threadIdx.x; i < npages; i += kPgThreads) lbt[i] = bt[i];
    __syncthreads();
  }
  // DMA of page p into ring slot `slot`: K image rows = keys (RBK bytes), V image rows = d
  // (RBV bytes); LDS position `pos` of a row holds the source chunk pos ^ swz(row)
  auto issue = [&](int p, int slot) {
    const long blk = lbt[p];
    const char* kb = reinterpret_cast<const char*>(k_cache + ((blk * Hkv + h) * BS) * D);
    const char* vb = reinterpret_cast<const char*>(v_cache + (blk * Hkv + h) * (long)D * BS);
    char* lk = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < LPW; ++i) {
      const int off = ((i * 4 + wid) * 64 + lane) * 16;      // byte of this lane in the image
      const int krow = off / RBK, kpos = (off % RBK) / 16;
      __builtin_amdgcn_global_load_lds((pg_gbl_t)(kb + krow * RBK + 16 * (kpos ^ pg_swz_k<CT>(krow))),
                                       (pg_lds_t)(lk + (i * 4 + wid) * 1024), 16, 0, 0);
      const int vrow = off / RBV, vpos = (off % RBV) / 16;
      __builtin_amdgcn_global_load_lds((pg_gbl_t)(vb + vrow * RBV + 16 * (vpos ^ pg_swz_v<CT>(vrow))),
                                       (pg_lds_t)(lk + KB + (i * 4 + wid) * 1024), 16, 0, 0);
    }
  };
  typedef typename KV<CT>::raw_t raw_t;
  auto compute = [&](int p, const char* lk) {
    // K fragments (A operand of S^T = K . Q^T), key order sigma as in the decode kernel
    bf16x8 kw[2][4];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int key = 8 * (r >> 2) + 4 * kt + (r & 3);
      const char* kr = lk + key * RBK;
      if constexpr (kF8) {
#pragma unroll
        for (int ds = 0; ds < 4; ds += 2) {
          const int c16 = 4 * (ds >> 1) + g;                 // 16-B chunk: ds and ds + 1
          const u32x4 w = *reinterpret_cast<const u32x4*>(kr + 16 * (c16 ^ pg_swz_k<CT>(key)));
          kw[kt][ds] = KV<CT>::widen(raw_t{w[0], w[1]});
          kw[kt][ds + 1] = KV<CT>::widen(raw_t{w[2], w[3]});
        }
      } else {
#pragma unroll
        for (int ds = 0; ds < 4; ++ds) {
          const int c16 = 4 * ds + g;
          kw[kt][ds] = *reinterpret_cast<const bf16x8*>(kr + 16 * (c16 ^ pg_swz_k<CT>(key)));
        }
      }
    }
    bf16x8 pb[2];
    float alpha[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (!on[c]) continue;
      f32x4 st[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        st[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ds = 0; ds < 4; ++ds) st[kt] = mfma16(kw[kt][ds], qf[c][ds], st[kt]);
      }
      float x[8];
      float tmax = kPgNegInf;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = p * BS + 8 * g + 4 * kt + i;
          const float v = key <= qpos[c] ? st[kt][i] * scale_log2 : kPgNegInf;
          x[kt * 4 + i] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m[c], tmax);
      const float mb = mn == kPgNegInf ? 0.f : mn;
      alpha[c] = exp2f(m[c] - mb);
      float ps = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = exp2f(x[j] - mb);
        ps += pv;
        pb[c][j] = f2bf(pv);
      }
      l[c] = l[c] * alpha[c] + ps;
      m[c] = mn;
    }
    // V^T fragments (A operand of O^T = V^T . P^T): row d = 16 dt + r, keys 8g .. 8g + 7
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int d = 16 * dt + r;
      bf16x8 vw;
      if constexpr (kF8) {
        const int pos = (g >> 1) ^ pg_swz_v<CT>(d);           // 16-B chunk, then its 8-B half
        vw = KV<CT>::widen(*reinterpret_cast<const raw_t*>(lk + KB + d * RBV + 16 * pos + 8 * (g & 1)));
      } else {
        vw = *reinterpret_cast<const bf16x8*>(lk + KB + d * RBV + 16 * (g ^ pg_swz_v<CT>(d)));
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (!on[c]) continue;
        o[c][dt] *= alpha[c];
        o[c][dt] = mfma16(vw, pb[c], o[c][dt]);
      }
    }
  };

  // S - 1 pages in flight: the stream is latency-bound (a workgroup reads one kv head's pages
  // at a few GB/s), so the ring depth, not bandwidth, sets its speed
  for (int st = 0; st < S - 1 && st < npages; ++st) issue(st, st);
  for (int p = 0; p < npages; ++p) {
    // page p landed (this wave's part; later issued pages may still fly), then every wave's part
    pg_wait_pages<2 * LPW>(min(S - 2, npages - 1 - p));
    __builtin_amdgcn_s_barrier();
    if (p + S - 1 < npages) issue(p + S - 1, (p + S - 1) % S);   // the slot of page p - 1: read by all
    compute(p, smem + (p % S) * STAGE);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    l[c] += __shfl_xor(l[c], 16, 64);
    l[c] += __shfl_xor(l[c], 32, 64);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (orow[c] < 0) continue;
    const float inv = l[c] > 0.f ? 1.f / l[c] : 0.f;
    bf16* op = out + (long)orow[c] * o_stride + (long)ohead[c] * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(o[c][dt][i] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt) = v;
    }
  }
}

}  // namespace

int launch_attn_prefill_paged(const bf16* q, long q_stride, const void* k_cache, const void* v_cache,
                              const int* tables, int bt_stride, const int* cu_q, const int* positions,
                              int nseq, int max_q, int Hq, int Hkv, int D, int block_size, float scale,
                              bf16* out, long o_stride, hipStream_t stream, int kv_fp8) {
  if (D != 128 || block_size != 32 || Hkv <= 0 || Hq % Hkv != 0) return -1;
  const int G = Hq / Hkv;
  if (G > 8) return -2;
  if (nseq <= 0 || max_q <= 0) return 0;
  const float scale_log2 = scale * 1.4426950408889634f;
  // BFLY_ATTN_PAGED_LDS=0: the register kernel (every wave fetches its own pages; A/B runs)
  static const bool lds = [] {
    const char* e = getenv("BFLY_ATTN_PAGED_LDS");
    return !(e && e[0] == '0');
  }();
  // one sequence's chunk: the register kernel (its 4 independent page streams per workgroup
  // win there, 72 vs 86-89 us for 512 tokens at 70B); several: the LDS kernel (1.15-1.45x,
  // profiles/r4_paged_prefill_ab.log)
  if (lds && nseq >= 2) {
    // 16-token groups per workgroup: 8 / G fill the 8 column groups of the 4 waves; fewer
    // while the grid would leave CUs idle (a short chunk of one sequence)
    int tg = 8 / G;
    while (tg > 1 && (long)((max_q + 16 * tg - 1) / (16 * tg)) * Hkv * nseq < 256) tg /= 2;
    const dim3 g2((max_q + 16 * tg - 1) / (16 * tg), Hkv, nseq);
    // a grid that fits one workgroup per CU gets the deep ring (8 pages: 128 KiB bf16), a
    // larger one 4 pages (64 KiB: two workgroups per CU keep as many pages in flight)
    const long wgs = (long)g2.x * g2.y * g2.z;
    auto run = [&](auto ct, auto sc) -> bool {
      typedef decltype(ct) CT;
      constexpr int S_ = decltype(sc)::value;
      const size_t lds_bytes = (size_t)S_ * 2 * 32 * 128 * sizeof(CT) + (size_t)bt_stride * 4;
      if (lds_bytes > 160 * 1024) return false;       // very long block tables: register kernel
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_prefill_paged_lds_kernel<128, 32, CT, S_>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
      }
      attn_prefill_paged_lds_kernel<128, 32, CT, S_><<<g2, kPgThreads, lds_bytes, stream>>>(
          q, q_stride, static_cast<const CT*>(k_cache), static_cast<const CT*>(v_cache), tables, bt_stride, cu_q,
          positions, Hq, Hkv, tg, scale_log2, out, o_stride);
      return true;
    };
    const bool deep = wgs <= 256;
    bool ran;
    if (kv_fp8)
      ran = deep ? run(fp8_t{}, std::integral_constant<int, 8>{}) : run(fp8_t{}, std::integral_constant<int, 4>{});
    else
      ran = deep ? run(bf16{}, std::integral_constant<int, 8>{}) : run(bf16{}, std::integral_constant<int, 4>{});
    if (ran) return 0;
  }
  const dim3 grid((max_q + kPgQ - 1) / kPgQ, Hkv, nseq);
#define PG_LAUNCH(CT, HPW)                                                                       \
  attn_prefill_paged_kernel<128, 32, CT, HPW><<<grid, kPgThreads, 0, stream>>>(                  \
      q, q_stride, static_cast<const CT*>(k_cache), static_cast<const CT*>(v_cache), tables,     \
      bt_stride, cu_q, positions, Hq, Hkv, scale_log2, out, o_stride)
  if (kv_fp8) {
    if (G <= 4) PG_LAUNCH(fp8_t, 1); else PG_LAUNCH(fp8_t, 2);
  } else {
    if (G <= 4) PG_LAUNCH(bf16, 1); else PG_LAUNCH(bf16, 2);
  }
#undef PG_LAUNCH
  return 0;
}

}  // namespace bfly
