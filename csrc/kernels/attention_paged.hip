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
  if (p < npages) load_page(p, kA, vA);
  while (p < npages) {
    if (p + 1 < npages) load_page(p + 1, kB, vB);
    compute_page(p, kA, vA);
    if (++p >= npages) break;
    if (p + 1 < npages) load_page(p + 1, kA, vA);
    compute_page(p, kB, vB);
    ++p;
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
