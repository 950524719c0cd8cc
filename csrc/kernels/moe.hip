// Mixture-of-experts kernels (K11 router, K12 gating) for the dense-dispatch MoE path.
//
// moe_route: one workgroup per token. logits[e] = x . Wr[e] (E <= 64 experts, 16-B loads of
// the token row and of each router row, 4-wave reduction), softmax over experts, top-k
// selection, renormalisation over the selected experts (Mixtral semantics), and a dense gate
// row gates[t, e] (0 for experts not selected) used by the fixed-shape expert GEMMs; topk ids/weights are also
// emitted for the sparse (grouped) path and for routing statistics.
//
// moe_gate_scale: h[t, e*F + f] *= gates[t, e0 + e] for the local experts: the gate weight is
// folded into the intermediate activation so that ONE GEMM over the concatenated local experts
// (K = E_local * F) both applies every expert's down projection and sums over experts.
//
// Sparse path (K12 permute / K13 grouped GEMM / weighted combine), used for prefill where the
// dense path would spend E/top_k times the FLOPs:
//   moe_align:   counting sort of the (token, k) pairs routed to local experts into per-expert
//                contiguous row slots; emits rows[slot] = token, slot_of[pair] (-1: not local)
//                and the grouped-GEMM tile list {expert, first slot, end slot} (+ its count),
//                all on the device so the whole layer is graph-capturable with fixed grids.
//   (grouped gate/up GEMM with SiLU, grouped down GEMM: gemm.hip GROUPED tile kernel)
//   moe_combine: out[t] = sum_j w[t, j] * Y[slot_of[t, j]] (f32, fixed j order).
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

constexpr int kMaxExperts = 64;

template <int EC>   // EC > 0: compile-time expert count (E == EC); 0: runtime E
__global__ void __launch_bounds__(256)
moe_route_kernel(const bf16* __restrict__ x, long x_stride, const bf16* __restrict__ wr, int T,
                 int H, int E, int K, float* __restrict__ gates, int* __restrict__ topk_ids,
                 float* __restrict__ topk_w) {
  // one workgroup per token: the 256 threads split the hidden dim (16-B chunks), every expert's
  // partial dot is wave-reduced and the 4 wave partials summed through LDS; wave 0 then holds
  // logit e in lane e (E <= 64) for the softmax / top-k, all in registers (no scratch arrays).
  __shared__ float red[4][kMaxExperts];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int t = blockIdx.x;
  const bf16* xr = x + (long)t * x_stride;
  if constexpr (EC > 0) {
    // compile-time expert count: every router-row load of a chunk is independent and in
    // flight together; E accumulators in registers
    float acc[EC];
#pragma unroll
    for (int e = 0; e < EC; ++e) acc[e] = 0.f;
    for (int c = tid * 8; c < H; c += 256 * 8) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(xr + c);
      bf16x8 w[EC];
#pragma unroll
      for (int e = 0; e < EC; ++e) w[e] = *reinterpret_cast<const bf16x8*>(wr + (long)e * H + c);
#pragma unroll
      for (int e = 0; e < EC; ++e)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[e] += bf2f(a[j]) * bf2f(w[e][j]);
    }
#pragma unroll
    for (int e = 0; e < EC; ++e) {
      const float s = wave_sum(acc[e]);
      if (lane == 0) red[wv][e] = s;
    }
  } else {
#pragma unroll 2
    for (int e = 0; e < E; ++e) {
      float acc = 0.f;
      for (int c = tid * 8; c < H; c += 256 * 8) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(xr + c);
        const bf16x8 w = *reinterpret_cast<const bf16x8*>(wr + (long)e * H + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += bf2f(a[j]) * bf2f(w[j]);
      }
      acc = wave_sum(acc);
      if (lane == 0) red[wv][e] = acc;
    }
  }
  __syncthreads();
  if (wv != 0) return;
  const bool live = lane < E;
  const float logit = live ? red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane] : 0.f;
  moe_select_topk(logit, live, lane, t, E, K, gates, topk_ids, topk_w);
}

__global__ void moe_gate_scale_kernel(bf16* __restrict__ h, const float* __restrict__ gates,
                                      long T, int E, int e0, int El, int F) {
  const long nvec = T * (long)El * F / 8;
  const int vpr = El * F / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nvec; i += (long)gridDim.x * 256) {
    const long t = i / vpr;
    const int c = (int)(i % vpr) * 8;
    const int e = c / F;
    const float g = gates[t * E + e0 + e];
    bf16x8 v = reinterpret_cast<bf16x8*>(h)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * g);
    reinterpret_cast<bf16x8*>(h)[i] = v;
  }
}

// `bcnt` (optional): the rows are ep blocks of `bcap` rows (the EP IPC receive buffer) of which
// only the first bcnt[block] are valid this call; pairs of the other rows are skipped (slot -1),
// so a receive buffer sized for the worst case costs work only for the rows that arrived.
__global__ void __launch_bounds__(1024)
moe_align_kernel(const int* __restrict__ topk_ids, int TK, int K, int e0, int El, int BM,
                 int* __restrict__ rows, int* __restrict__ slot_of, int4* __restrict__ tiles,
                 int* __restrict__ count, const int* __restrict__ bcnt, int bcap) {
  __shared__ int cnt[kMaxExperts], cur[kMaxExperts];
  auto valid = [&](int i) {
    if (bcnt == nullptr) return true;
    const int row = i / K;
    return row % bcap < bcnt[row / bcap];
  };
  for (int e = threadIdx.x; e < El; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < TK; i += blockDim.x) {
    const int e = topk_ids[i] - e0;
    if (e >= 0 && e < El && valid(i)) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int off = 0, nt = 0;
    for (int e = 0; e < El; ++e) {
      cur[e] = off;
      // .w = 1: the expert's rows fit one tile, so its weights are read exactly once
      for (int r = off; r < off + cnt[e]; r += BM)
        tiles[nt++] = int4{e, r, min(r + BM, off + cnt[e]), cnt[e] <= BM ? 1 : 0};
      off += cnt[e];
    }
    *count = nt;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TK; i += blockDim.x) {
    const int e = topk_ids[i] - e0;
    if (e >= 0 && e < El && valid(i)) {
      const int pos = atomicAdd(&cur[e], 1);
      rows[pos] = i / K;
      slot_of[i] = pos;
    } else {
      slot_of[i] = -1;
    }
  }
}

__global__ void __launch_bounds__(256)
moe_combine_kernel(const bf16* __restrict__ y, const int* __restrict__ slot_of,
                   const float* __restrict__ w, int K, int H, bf16* __restrict__ out,
                   const int* __restrict__ bcnt, int bcap) {
  const long t = blockIdx.x;
  if (bcnt != nullptr && t % bcap >= bcnt[t / bcap]) return;   // row did not arrive: not written
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < K; ++j) {
      const int sl = slot_of[t * K + j];
      if (sl < 0) continue;
      const float g = w[t * K + j];
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(y + (long)sl * H + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += g * bf2f(v[q]);
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *reinterpret_cast<bf16x8*>(out + t * H + c) = o;
  }
}

// out[t] = sum_j w[t, j] * sum_s part[s][slot_of[t, j]]: the weighted combine with the
// grouped down GEMM's split-K reduce folded in (f32 throughout, one bf16 rounding)
__global__ void __launch_bounds__(256)
moe_combine_slabs_kernel(const float* __restrict__ part, int sk, long slab, const int* __restrict__ slot_of,
                         const float* __restrict__ w, int K, int H, bf16* __restrict__ out,
                         const int* __restrict__ bcnt, int bcap) {
  const long t = blockIdx.x;
  if (bcnt != nullptr && t % bcap >= bcnt[t / bcap]) return;
  for (int c = threadIdx.x * 4; c < H; c += 256 * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < K; ++j) {
      const int sl = slot_of[t * K + j];
      if (sl < 0) continue;
      const float g = w[t * K + j];
      f32x4 y = *reinterpret_cast<const f32x4*>(part + (long)sl * H + c);
      for (int s = 1; s < sk; ++s) y += *reinterpret_cast<const f32x4*>(part + s * slab + (long)sl * H + c);
      acc += g * y;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) out[t * H + c + q] = f2bf(acc[q]);
  }
}

int launch_moe_combine_slabs(const float* part, int sk, long slab, const int* slot_of, const float* w,
                             int T, int K, int H, bf16* out, hipStream_t stream, const int* bcnt, int bcap) {
  if (H % 4 != 0 || sk < 1 || (bcnt != nullptr && bcap <= 0)) return -1;
  if (T <= 0) return 0;
  moe_combine_slabs_kernel<<<T, 256, 0, stream>>>(part, sk, slab, slot_of, w, K, H, out, bcnt, bcap);
  return 0;
}

// ---- expert-parallel dispatch over a fixed-capacity all-to-all (decode) ----------------
// Token t goes once to every EP rank d owning one of its top-k experts (El experts per rank),
// into row d * cap + pos[t][d], pos = number of earlier tokens bound for d (a stable order,
// so no capacity can overflow: cap >= T). Every workgroup recomputes the prefix counts it
// needs from the (tiny) id array instead of a separate scan kernel.
template <int EP>
__device__ __forceinline__ void ep_hits(const int* ids, int t, int K, int El, const int* slots, bool (&h)[EP]) {
#pragma unroll
  for (int d = 0; d < EP; ++d) h[d] = false;
  if (slots != nullptr && slots[t] < 0) return;   // graph padding row: routes nowhere
  for (int j = 0; j < K; ++j) {
    const int e = ids[t * K + j];
    if (e >= 0) {
      const int d = e / El;
#pragma unroll
      for (int q = 0; q < EP; ++q) h[q] |= (q == d);
    }
  }
}

// grid = cap workgroups (cap >= T). Block b: (1) counts, over tokens t' < b and over all
// tokens, the hits per destination; (2) if b < T, copies row b to each destination it hits
// and writes that row's metadata (expert ids local to d as int32 bits, gate weights; other
// slots -1 / 0) and slot[b][d] (-1: not sent); (3) for every destination whose total count
// is <= b, marks metadata row d * cap + b empty (all ids -1).
template <int EP>
__global__ void __launch_bounds__(256)
ep_pack_kernel(const bf16* __restrict__ x, const int* __restrict__ ids, const float* __restrict__ w,
               const int* __restrict__ slots, int T, int K, int H, int El, int cap,
               bf16* __restrict__ send, float* __restrict__ meta, int* __restrict__ slot) {
  __shared__ int red[2][EP][4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int before[EP], total[EP];
#pragma unroll
  for (int d = 0; d < EP; ++d) before[d] = total[d] = 0;
  for (int t = tid; t < T; t += 256) {
    bool h[EP];
    ep_hits<EP>(ids, t, K, El, slots, h);
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      total[d] += h[d];
      before[d] += (h[d] && t < b);
    }
  }
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    const float tb = wave_sum((float)before[d]), tt = wave_sum((float)total[d]);
    if (lane == 0) { red[0][d][wv] = (int)tb; red[1][d][wv] = (int)tt; }
  }
  __syncthreads();
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    before[d] = red[0][d][0] + red[0][d][1] + red[0][d][2] + red[0][d][3];
    total[d] = red[1][d][0] + red[1][d][1] + red[1][d][2] + red[1][d][3];
  }
  const int M2 = 2 * K;
  if (b < T) {
    bool h[EP];
    ep_hits<EP>(ids, b, K, El, slots, h);
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      if (tid == 0) slot[b * EP + d] = h[d] ? d * cap + before[d] : -1;
      if (!h[d]) continue;
      const long row = (long)d * cap + before[d];
      const bf16x8* src = reinterpret_cast<const bf16x8*>(x + (long)b * H);
      bf16x8* dst = reinterpret_cast<bf16x8*>(send + row * H);
      for (int c = tid; c < H / 8; c += 256) dst[c] = src[c];
      if (tid < K) {
        const int e = ids[b * K + tid];
        const bool mine = e >= 0 && e / El == d;
        meta[row * M2 + tid] = __int_as_float(mine ? e : -1);
        meta[row * M2 + K + tid] = mine ? w[b * K + tid] : 0.f;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < EP; ++d) {
    if (b >= total[d] && tid < K) {
      const long row = (long)d * cap + b;
      meta[row * M2 + tid] = __int_as_float(-1);
      meta[row * M2 + K + tid] = 0.f;
    }
  }
}

// out[t] = sum over destinations d that t was sent to of back[slot[t][d]] (f32, fixed d order)
template <int EP>
__global__ void __launch_bounds__(256)
ep_combine_kernel(const bf16* __restrict__ back, const int* __restrict__ slot, int H, bf16* __restrict__ out) {
  const long t = blockIdx.x;
  int sl[EP];
#pragma unroll
  for (int d = 0; d < EP; ++d) sl[d] = slot[t * EP + d];
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < EP; ++d) {
      if (sl[d] < 0) continue;
      const bf16x8 v = reinterpret_cast<const bf16x8*>(back + (long)sl[d] * H)[c];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += bf2f(v[q]);
    }
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    reinterpret_cast<bf16x8*>(out + t * H)[c] = o;
  }
}

int launch_ep_pack(const bf16* x, const int* ids, const float* w, const int* slots, int T, int K, int H,
                   int El, int ep, int cap, bf16* send, float* meta, int* slot, hipStream_t stream) {
  if (H % 8 != 0 || K > 64 || cap < T || cap <= 0 || El <= 0) return -1;
  const dim3 grid(cap);
  switch (ep) {
    case 2: ep_pack_kernel<2><<<grid, 256, 0, stream>>>(x, ids, w, slots, T, K, H, El, cap, send, meta, slot); return 0;
    case 4: ep_pack_kernel<4><<<grid, 256, 0, stream>>>(x, ids, w, slots, T, K, H, El, cap, send, meta, slot); return 0;
    case 8: ep_pack_kernel<8><<<grid, 256, 0, stream>>>(x, ids, w, slots, T, K, H, El, cap, send, meta, slot); return 0;
    default: return -2;
  }
}

int launch_ep_combine(const bf16* back, const int* slot, int T, int H, int ep, bf16* out, hipStream_t stream) {
  if (H % 8 != 0) return -1;
  if (T <= 0) return 0;
  switch (ep) {
    case 2: ep_combine_kernel<2><<<T, 256, 0, stream>>>(back, slot, H, out); return 0;
    case 4: ep_combine_kernel<4><<<T, 256, 0, stream>>>(back, slot, H, out); return 0;
    case 8: ep_combine_kernel<8><<<T, 256, 0, stream>>>(back, slot, H, out); return 0;
    default: return -2;
  }
}

int moe_max_tiles(int TK, int El, int BM) { return (TK + BM - 1) / BM + El; }

int launch_moe_align(const int* topk_ids, int T, int K, int e0, int El, int BM, int* rows,
                     int* slot_of, int4* tiles, int* count, hipStream_t stream, const int* bcnt, int bcap) {
  if (El <= 0 || El > kMaxExperts || BM <= 0 || (bcnt != nullptr && (bcap <= 0 || T % bcap != 0))) return -1;
  if (T <= 0) return (int)hipMemsetAsync(count, 0, sizeof(int), stream);   // no tiles
  moe_align_kernel<<<1, 1024, 0, stream>>>(topk_ids, T * K, K, e0, El, BM, rows, slot_of, tiles, count, bcnt, bcap);
  return 0;
}

int launch_moe_combine(const bf16* y, const int* slot_of, const float* w, int T, int K, int H,
                       bf16* out, hipStream_t stream, const int* bcnt, int bcap) {
  if (H % 8 != 0 || (bcnt != nullptr && bcap <= 0)) return -1;
  if (T <= 0) return 0;
  moe_combine_kernel<<<T, 256, 0, stream>>>(y, slot_of, w, K, H, out, bcnt, bcap);
  return 0;
}

int launch_moe_route(const bf16* x, long x_stride, const bf16* wr, int T, int H, int E, int K,
                     float* gates, int* topk_ids, float* topk_w, hipStream_t stream) {
  if (T <= 0) return 0;
  if (E > kMaxExperts || K > 8 || K > E || H % 8 != 0) return -1;
  if (E == 8)
    moe_route_kernel<8><<<T, 256, 0, stream>>>(x, x_stride, wr, T, H, E, K, gates, topk_ids, topk_w);
  else
    moe_route_kernel<0><<<T, 256, 0, stream>>>(x, x_stride, wr, T, H, E, K, gates, topk_ids, topk_w);
  return 0;
}

void launch_moe_gate_scale(bf16* h, const float* gates, long T, int E, int e0, int El, int F,
                           hipStream_t stream) {
  const long nvec = T * (long)El * F / 8;
  if (nvec <= 0) return;
  long g = (nvec + 255) / 256;
  if (g > 4096) g = 4096;
  moe_gate_scale_kernel<<<(int)g, 256, 0, stream>>>(h, gates, T, E, e0, El, F);
}

}  // namespace bfly
