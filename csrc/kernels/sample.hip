// On-device token selection (K10): greedy argmax and temperature sampling by the Gumbel-max
// trick, over the (possibly vocab-parallel) logits shard.
//
// Stage 1 (grid rows x chunks): every workgroup reduces one chunk of one row to a packed
// u64 key = ordered(score) << 32 | (~index), so max(key) = (max score, smallest index).
// Stage 2 (one wave per row): reduce the chunk keys; emit the winning global token id and
// its score. With tensor parallelism the caller all-gathers (score, id) pairs and takes the
// max: scores are comparable across ranks because the Gumbel noise is keyed on the GLOBAL
// vocab index and the per-row seed, not on the rank.
//
// check_finite: a row whose logits shard holds an Inf or NaN yields id -1 and score +inf (so
// it also wins the TP merge on every rank): the engine's NaN guard without extra kernels.
//
// Top-k / top-p: `thresh[row]` (optional) is a lower bound on the temperature-scaled logit;
// tokens below it are excluded before the Gumbel-max. Gumbel-max over the kept set samples
// exactly the renormalised truncated distribution, so filtering reduces to one threshold per
// row (computed from the global top candidates by the sampler, engine/sampler.py).
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

constexpr int kSampleThreads = 256;

__device__ __forceinline__ uint32_t ordered_f32(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordered_f32(uint32_t o) {
  const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
// Uniform in (0, 1) from (seed, global index).
__device__ __forceinline__ float uniform01(uint64_t seed, uint32_t idx) {
  const uint64_t h = mix64(seed * 0x9E3779B97F4A7C15ULL + idx + 1);
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v = umax64(v, ((uint64_t)hi << 32) | lo);
  }
  return v;
}

__global__ void __launch_bounds__(kSampleThreads)
sample_partial_kernel(const bf16* __restrict__ logits, long row_stride, int V, int chunk,
                      int vstart, const float* __restrict__ temps,
                      const long* __restrict__ seeds, const float* __restrict__ thresh,
                      uint64_t* __restrict__ partial, int check_finite) {
  __shared__ uint64_t red[kSampleThreads / 64];
  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = 0;
  const int row = blockIdx.x, c = blockIdx.y;
  const float temp = temps ? temps[row] : 0.f;
  const bool greedy = temp <= 0.f;
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0;
  const float thr = (thresh != nullptr && !greedy) ? thresh[row] : -INFINITY;
  const int begin = c * chunk, end = min(V, begin + chunk);
  const bf16* lr = logits + (long)row * row_stride;
  uint64_t best = 0;
  uint32_t nonfinite = 0;   // OR of exponent-all-ones tests (Inf / NaN bf16)
  for (int i = begin + threadIdx.x * 8; i < end; i += kSampleThreads * 8) {
    if (i + 8 <= end) {
      const u32x4 raw = *reinterpret_cast<const u32x4*>(lr + i);
#pragma unroll
      for (int k = 0; k < 4; ++k)   // bf16 exponent all ones: Inf or NaN
        nonfinite |= (uint32_t)((raw[k] & 0x7F80u) == 0x7F80u) | (uint32_t)((raw[k] & 0x7F800000u) == 0x7F800000u);
      const bf16x8 v = __builtin_bit_cast(bf16x8, raw);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = bf2f(v[j]);
        if (!greedy) {
          s = s * inv_t;
          if (s < thr) continue;            // outside the top-k / top-p set
          s -= __logf(-__logf(uniform01(seed, (uint32_t)(vstart + i + j))));
        }
        const uint64_t key = ((uint64_t)ordered_f32(s) << 32) | (uint32_t)(~(uint32_t)(vstart + i + j));
        best = umax64(best, key);
      }
    } else {
      for (int j = 0; i + j < end; ++j) {
        const uint32_t bits = reinterpret_cast<const uint16_t*>(lr)[i + j];
        nonfinite |= (uint32_t)((bits & 0x7F80u) == 0x7F80u);
        float s = bf2f(lr[i + j]);
        if (!greedy) {
          s = s * inv_t;
          if (s < thr) continue;
          s -= __logf(-__logf(uniform01(seed, (uint32_t)(vstart + i + j))));
        }
        const uint64_t key = ((uint64_t)ordered_f32(s) << 32) | (uint32_t)(~(uint32_t)(vstart + i + j));
        best = umax64(best, key);
      }
    }
  }
  best = wave_max_u64(best);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();   // also orders s_bad's initialisation before the atomics below
  if (check_finite && nonfinite) atomicOr(&s_bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = red[0];
    for (int w = 1; w < kSampleThreads / 64; ++w) b = umax64(b, red[w]);
    partial[(long)row * gridDim.y + c] = s_bad ? ~0ULL : b;   // ~0: a NaN key, never a real one
  }
}

__global__ void sample_final_kernel(const uint64_t* __restrict__ partial, int chunks, int vstart,
                                    int* __restrict__ out_ids, float* __restrict__ out_scores) {
  const int row = blockIdx.x;
  uint64_t b = 0;
  for (int c = threadIdx.x; c < chunks; c += 64) b = umax64(b, partial[(long)row * chunks + c]);
  b = wave_max_u64(b);
  if (threadIdx.x == 0) {
    const bool bad = b == ~0ULL;
    // b == 0: every token of this shard lies below the row's top-k / top-p threshold (common
    // with vocab-parallel shards). No candidate: score -inf (loses the TP merge to any real
    // candidate), id kept in range.
    const bool none = b == 0;
    out_ids[row] = bad ? -1 : (none ? vstart : (int)(~(uint32_t)b));
    if (out_scores) out_scores[row] = bad ? INFINITY : (none ? -INFINITY : unordered_f32((uint32_t)(b >> 32)));
  }
}

// ---------------------------------------------------------------------------------------
// Exact top-k / top-p thresholds by radix select (A17/K10). The filter of a row is one
// threshold on s = logit * (1 / temperature): top-k keeps the k largest s (ties included),
// top-p then keeps, in descending order, every token whose preceding probability mass (under
// the top-k-renormalised distribution) is <= p. Both thresholds are exact token values found
// by a most-significant-digit-first radix select over the 32-bit order-preserving key of s:
// 4 passes of 8 bits per filter, each a 256-bin histogram of the keys that still match the
// selected prefix. Under tensor parallelism the caller SUM-all-reduces every histogram (and
// MAX-all-reduces the row maximum), so each vocab shard contributes its tokens and all ranks
// select the same digits; no candidate cap, no sort, fixed shapes (graph-capturable).
//
// Workspace per row (f32 bits; int32 fields stored through __float_as_int):
//   state[8] : 0 top-k prefix (u32)  1 k remaining  2 top-p prefix (u32)  3 mass above prefix
//              4 Z (mass of the top-k set)  5 flags (1 = top-k active, 2 = top-p active)
//   smax[1]  : row max of s as a signed-comparable ordered int (MAX-reducible as int32)
//   hist[512]: 256 counts + 256 masses exp(s - max) (SUM-reducible as f32; counts exact < 2^24)
// ---------------------------------------------------------------------------------------
constexpr int kTkpThreads = 256;

__device__ __forceinline__ int signed_ordered(float f) { return (int)(ordered_f32(f) ^ 0x80000000u); }
__device__ __forceinline__ float from_signed_ordered(int v) { return unordered_f32((uint32_t)v ^ 0x80000000u); }

// Row maximum of s over this shard (atomicMax into smax, set to INT_MIN by the caller) and the row's
// initial select state.
__global__ void __launch_bounds__(kTkpThreads)
tkp_begin_kernel(const bf16* __restrict__ logits, long row_stride, int V, int chunk,
                 const float* __restrict__ temps, const int* __restrict__ top_k,
                 const float* __restrict__ top_p, float* __restrict__ state, int* __restrict__ smax) {
  __shared__ float red[kTkpThreads / 64];
  const int row = blockIdx.x, c = blockIdx.y;
  const float temp = temps[row];
  const float inv_t = temp > 0.f ? 1.f / temp : 1.f;
  const bf16* lr = logits + (long)row * row_stride;
  const int begin = c * chunk, end = min(V, begin + chunk);
  float m = -INFINITY;
  for (int i = begin + threadIdx.x * 8; i < end; i += kTkpThreads * 8) {
    if (i + 8 <= end) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(lr + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, bf2f(v[j]) * inv_t);
    } else {
      for (int j = 0; i + j < end; ++j) m = fmaxf(m, bf2f(lr[i + j]) * inv_t);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kTkpThreads / 64; ++w) m = fmaxf(m, red[w]);
    atomicMax(smax + row, signed_ordered(m));
    if (c == 0) {
      float* st = state + row * 8;
      const int k = temp > 0.f ? top_k[row] : 0;
      const int flags = (k > 0 ? 1 : 0) | (temp > 0.f && top_p[row] < 1.f ? 2 : 0);
      st[0] = __int_as_float(0);
      st[1] = __int_as_float(k);
      st[2] = __int_as_float(0);
      st[3] = 0.f;
      st[4] = 0.f;
      st[5] = __int_as_float(flags);
    }
  }
}

// One radix pass: histogram of digit `pass` (bits 31-8*pass .. 24-8*pass) of the keys whose
// higher digits equal the selected prefix. phase 0 = top-k (counts), 1 = top-p (counts and
// masses, restricted to keys >= the top-k threshold key).
__global__ void __launch_bounds__(kTkpThreads)
tkp_hist_kernel(const bf16* __restrict__ logits, long row_stride, int V, int chunk,
                const float* __restrict__ temps, const float* __restrict__ state,
                const int* __restrict__ smax, float* __restrict__ hist, int pass, int phase) {
  __shared__ float h[512];
  const int row = blockIdx.x, c = blockIdx.y;
  const float* st = state + row * 8;
  const int flags = __float_as_int(st[5]);
  if (!(flags & (phase == 0 ? 1 : 2))) return;   // block-uniform
  for (int i = threadIdx.x; i < 512; i += kTkpThreads) h[i] = 0.f;
  __syncthreads();
  const float inv_t = 1.f / temps[row];
  const uint32_t prefix = (uint32_t)__float_as_int(st[phase == 0 ? 0 : 2]);
  const uint32_t kmin = (phase == 1 && (flags & 1)) ? (uint32_t)__float_as_int(st[0]) : 0u;
  const float mx = from_signed_ordered(smax[row]);
  const int shift = 24 - 8 * pass;
  const bf16* lr = logits + (long)row * row_stride;
  const int begin = c * chunk, end = min(V, begin + chunk);
  auto add = [&](float s) {
    const uint32_t key = ordered_f32(s);
    if (key < kmin) return;
    if (pass > 0 && (key >> (shift + 8)) != prefix) return;
    const int d = (key >> shift) & 255;
    atomicAdd(&h[d], 1.f);
    if (phase == 1) atomicAdd(&h[256 + d], __expf(s - mx));
  };
  for (int i = begin + threadIdx.x * 8; i < end; i += kTkpThreads * 8) {
    if (i + 8 <= end) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(lr + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) add(bf2f(v[j]) * inv_t);
    } else {
      for (int j = 0; i + j < end; ++j) add(bf2f(lr[i + j]) * inv_t);
    }
  }
  __syncthreads();
  float* hr = hist + (long)row * 512;
  for (int i = threadIdx.x; i < (phase == 1 ? 512 : 256); i += kTkpThreads)
    if (h[i] != 0.f) atomicAdd(hr + i, h[i]);
}

// Pick this pass's digit from the (reduced) histogram and clear it for the next pass. One
// wave per row; lane l owns bins 4l .. 4l+3, and the scan runs from the top bin down.
__global__ void __launch_bounds__(64)
tkp_select_kernel(const float* __restrict__ top_p, float* __restrict__ state,
                  float* __restrict__ hist, int pass, int phase) {
  const int row = blockIdx.x, lane = threadIdx.x;
  float* st = state + row * 8;
  const int flags = __float_as_int(st[5]);
  float* hr = hist + (long)row * 512;
  if (!(flags & (phase == 0 ? 1 : 2))) return;
  // lanes in DESCENDING bin order: lane l holds bins 255-4l .. 252-4l
  float cnt[4], mass[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cnt[j] = hr[255 - 4 * lane - j];
    mass[j] = phase == 1 ? hr[256 + 255 - 4 * lane - j] : 0.f;
  }
  // inclusive prefix sums over the descending order: per-lane, then across lanes
  float cs = cnt[0] + cnt[1] + cnt[2] + cnt[3];
  float ms = mass[0] + mass[1] + mass[2] + mass[3];
  float cex = cs, mex = ms;   // becomes the exclusive prefix of the lane
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float a = __shfl_up(cex, o, 64), b = __shfl_up(mex, o, 64);
    if (lane >= o) { cex += a; mex += b; }
  }
  const float ctot = __shfl(cex, 63, 64), mtot = __shfl(mex, 63, 64);
  cex -= cs;
  mex -= ms;
  int choice = -1;   // digit chosen by this lane (the wave takes the max / min below)
  if (phase == 0) {
    const int k_rem = __float_as_int(st[1]);
    if (pass == 0 && ctot < (float)k_rem) {   // k >= tokens: keep everything
      if (lane == 0) st[5] = __int_as_float(flags & ~1);
    } else {
      // first bin (descending) where the inclusive count reaches k_rem
      float run = cex;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float before = run;
        run += cnt[j];
        if (choice < 0 && before < (float)k_rem && run >= (float)k_rem) choice = 255 - 4 * lane - j;
      }
      // exactly one lane holds the crossing bin
      int d = choice;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) d = max(d, __shfl_xor(d, o, 64));
      float above = 0.f;   // count of bins strictly above d
      run = cex;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (255 - 4 * lane - j == d) above = run;
        run += cnt[j];
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) above += __shfl_xor(above, o, 64);
      if (lane == 0) {
        st[0] = __int_as_float((int)(((uint32_t)__float_as_int(st[0]) << 8) | (uint32_t)d));
        st[1] = __int_as_float(k_rem - (int)above);
      }
    }
  } else {
    float z = st[4], mabove = st[3];
    if (pass == 0) { z = mtot; mabove = 0.f; }
    const float lim = top_p[row] * z;
    // lowest non-empty bin whose mass strictly above it (within the prefix) keeps
    // mabove + that <= lim; scanning descending, that is the LAST qualifying bin
    float run = mex, keep_above = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (cnt[j] > 0.f && mabove + run <= lim) { choice = 255 - 4 * lane - j; keep_above = run; }
      run += mass[j];
    }
    // smallest digit among lanes' choices (descending order: the largest lane index wins)
    int d = choice < 0 ? 256 : choice;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = min(d, __shfl_xor(d, o, 64));
    float ka = (choice == d) ? keep_above : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ka += __shfl_xor(ka, o, 64);
    if (lane == 0) {
      if (d == 256) d = 255;   // unreachable with a consistent histogram (the top bin qualifies)
      st[2] = __int_as_float((int)(((uint32_t)__float_as_int(st[2]) << 8) | (uint32_t)d));
      st[3] = mabove + ka;
      st[4] = z;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hr[255 - 4 * lane - j] = 0.f;
    hr[256 + 255 - 4 * lane - j] = 0.f;
  }
}

// Final per-row threshold on s (-inf = no filter), as read by sample_partial_kernel.
__global__ void tkp_final_kernel(const float* __restrict__ state, int rows, float* __restrict__ thresh) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  const float* st = state + row * 8;
  const int flags = __float_as_int(st[5]);
  uint32_t key = 0;
  if (flags & 1) key = (uint32_t)__float_as_int(st[0]);
  if (flags & 2) key = max(key, (uint32_t)__float_as_int(st[2]));
  thresh[row] = flags ? unordered_f32(key) : -INFINITY;
}

static void tkp_chunks(int V, int& chunks, int& chunk) {
  chunks = (V + 8191) / 8192;
  if (chunks > 64) chunks = 64;
  chunk = (V + chunks - 1) / chunks;
  chunk = (chunk + 7) / 8 * 8;
  chunks = (V + chunk - 1) / chunk;
}

void launch_tkp_begin(const bf16* logits, long row_stride, int rows, int V, const float* temps,
                      const int* top_k, const float* top_p, float* state, int* smax, hipStream_t stream) {
  if (rows <= 0) return;
  int chunks, chunk;
  tkp_chunks(V, chunks, chunk);
  tkp_begin_kernel<<<dim3(rows, chunks), kTkpThreads, 0, stream>>>(logits, row_stride, V, chunk, temps, top_k,
                                                                    top_p, state, smax);
}

void launch_tkp_pass(const bf16* logits, long row_stride, int rows, int V, const float* temps,
                     float* state, const int* smax, float* hist, int pass, int phase, hipStream_t stream) {
  if (rows <= 0) return;
  int chunks, chunk;
  tkp_chunks(V, chunks, chunk);
  tkp_hist_kernel<<<dim3(rows, chunks), kTkpThreads, 0, stream>>>(logits, row_stride, V, chunk, temps, state,
                                                                   smax, hist, pass, phase);
}

void launch_tkp_select(const float* top_p, float* state, float* hist, int rows, int pass, int phase,
                       hipStream_t stream) {
  if (rows <= 0) return;
  tkp_select_kernel<<<rows, 64, 0, stream>>>(top_p, state, hist, pass, phase);
}

void launch_tkp_final(const float* state, int rows, float* thresh, hipStream_t stream) {
  if (rows <= 0) return;
  tkp_final_kernel<<<(rows + 63) / 64, 64, 0, stream>>>(state, rows, thresh);
}

// TP sampling merge: each vocab shard's winner as an f32 (score, id) pair
// (ids < 2^24 are exact in f32) -> all-gathered [tp][rows][2] -> the highest score per row, the
// lowest rank on ties (torch.argmax's first maximum). Two tiny kernels in place of torch's
// stack / cast / argmax / gather on every TP decode step.
__global__ void sample_pack_kernel(const float* __restrict__ scores, const int* __restrict__ ids,
                                   float* __restrict__ pair, int rows) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  pair[2 * r] = scores[r];
  pair[2 * r + 1] = (float)ids[r];
}

__global__ void sample_merge_kernel(const float* __restrict__ allp, int tp, int rows, int* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  int best = 0;
  float bs = allp[2 * r];
  for (int k = 1; k < tp; ++k) {
    const float sc = allp[((long)k * rows + r) * 2];
    if (sc > bs || (sc != sc && bs == bs)) {   // argmax semantics: NaN counts as the maximum
      bs = sc;
      best = k;
    }
  }
  out[r] = (int)allp[((long)best * rows + r) * 2 + 1];
}

void launch_sample_pack(const float* scores, const int* ids, float* pair, int rows, hipStream_t stream) {
  if (rows <= 0) return;
  sample_pack_kernel<<<(rows + 255) / 256, 256, 0, stream>>>(scores, ids, pair, rows);
}

void launch_sample_merge(const float* allp, int tp, int rows, int* out, hipStream_t stream) {
  if (rows <= 0) return;
  sample_merge_kernel<<<(rows + 255) / 256, 256, 0, stream>>>(allp, tp, rows, out);
}

void launch_sample(const bf16* logits, long row_stride, int rows, int V, int vstart,
                   const float* temps, const long* seeds, uint64_t* workspace, int* out_ids,
                   float* out_scores, hipStream_t stream, const float* thresh, int check_finite) {
  if (rows <= 0) return;
  int chunks = (V + 4095) / 4096;
  if (chunks > kSampleMaxChunks) chunks = kSampleMaxChunks;
  int chunk = (V + chunks - 1) / chunks;
  chunk = (chunk + 7) / 8 * 8;
  chunks = (V + chunk - 1) / chunk;
  dim3 g1(rows, chunks);
  sample_partial_kernel<<<g1, kSampleThreads, 0, stream>>>(logits, row_stride, V, chunk, vstart,
                                                           temps, seeds, thresh, workspace, check_finite);
  sample_final_kernel<<<rows, 64, 0, stream>>>(workspace, chunks, vstart, out_ids, out_scores);
}

}  // namespace bfly
