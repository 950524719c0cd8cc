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

__global__ void sample_final_kernel(const uint64_t* __restrict__ partial, int chunks,
                                    int* __restrict__ out_ids, float* __restrict__ out_scores) {
  const int row = blockIdx.x;
  uint64_t b = 0;
  for (int c = threadIdx.x; c < chunks; c += 64) b = umax64(b, partial[(long)row * chunks + c]);
  b = wave_max_u64(b);
  if (threadIdx.x == 0) {
    const bool bad = b == ~0ULL;
    out_ids[row] = bad ? -1 : (int)(~(uint32_t)b);
    if (out_scores) out_scores[row] = bad ? INFINITY : unordered_f32((uint32_t)(b >> 32));
  }
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
  sample_final_kernel<<<rows, 64, 0, stream>>>(workspace, chunks, out_ids, out_scores);
}

}  // namespace bfly
