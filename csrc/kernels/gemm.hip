// MFMA GEMMs for every linear layer (K1 prefill GEMM, K2 decode skinny GEMM, K13 expert GEMM).
//
//   Y[M, N] = X[M, K] . W[N, K]^T        (W in nn.Linear [out, in] layout: both operands are
//                                          K-contiguous, the natural MFMA "NT" layout)
// Epilogues (fused, so the activation never makes an extra HBM round trip):
//   EPI_NONE  : Y = acc
//   EPI_BIAS  : Y = acc + bias[n]
//   EPI_SILU  : W's rows are gate/up interleaved in 16-row groups (g0 u0 g1 u1 ...);
//               Y[M, N/2] = silu(gate) * up  (the SwiGLU FFN's first half in one kernel)
//
// Two kernels, picked by M on the host:
//  * gemm_skinny (M <= 64, decode): weight-streaming. Each wave streams 16*NT rows of W
//    straight into VGPRs with non-temporal 16-B loads (no LDS round trip for an operand that is
//    read exactly once: cdna_hip_programming.md §5 table, "GEMV / M <= 16" row), X fragments
//    come from L2. W is the MFMA A operand (16 weight rows per mfma_f32_16x16x32_bf16) and the
//    tokens are the B operand, so one weight fragment feeds MT token tiles. The K loop is
//    split over the 4 waves of a workgroup and, for narrow N, over workgroups (split-K with
//    f32 partial slabs and a reduce kernel that applies the epilogue).
//    K permutation: per 128-wide K chunk, sub-step s, lane group g = lane>>4 and element j
//    hold physical k = 32s + 8g + j, so each load instruction reads 64 contiguous bytes per
//    row; the same map is used for both operands, so every product pairs matching k.
//  * gemm_tile (M > 64, prefill / large-batch decode): BMx128x64 LDS-tiled, 4 waves (2x2),
//    both operands staged global->LDS by global_load_lds_dwordx4 (no VGPR round trip) into
//    two buffers (load of tile t+1 overlaps MFMAs on tile t), XOR-swizzled LDS image
//    (slot = chunk ^ ((row >> 1) & 7), applied on the per-lane SOURCE address because the
//    DMA writes lane-linearly; rule 21) which makes every ds_read_b128 lane group hit 16
//    distinct bank slots; bijective XCD-aware tile remap (T1).
#include "bfly_common.h"

#include <cstdio>
#include <string>
#include <vector>
#include "bfly_kernels.h"
#include "bfly_kv.h"

namespace bfly {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Non-temporal weight policy switch (BFLY_GEMM_NT_WEIGHTS=0 disables it; A/B measurements).
__constant__ int g_tile_w_nt = 1;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// ---------------------------------------------------------------------------------------
// Epilogue helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void store_out(bf16* out, long ldo, int m, int n, float v) {
  out[(long)m * ldo + n] = f2bf(v);
}

// Four consecutive output columns of one row (the tile / decode-ring accumulators hold 4
// consecutive n per lane: W is their MFMA A operand). 8-B store when the row start allows it.
__device__ __forceinline__ void store_out4(bf16* out, long ldo, int m, int n, f32x4 v, bool vec) {
  bf16* p = out + (long)m * ldo + n;
  if (vec) {
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = f2bf(v[r]);
    *reinterpret_cast<bf16x4*>(p) = o;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = f2bf(v[r]);
  }
}

// Split-K partial slabs: 16 B per lane through a buffer descriptor, plain (write-back) stores.
// Measured and dropped: write-through (`sc1`) slab stores, meant to spare the consumer the
// write-back of MBs of dirty f32 lines (MI355X_MICROARCH.md 'boundary'), made the whole decode
// step SLOWER: Llama-3-70B 30.28-30.32 vs 29.99-30.02 ms, Llama-3-8B 5.58 vs 5.49 ms
// (profiles/r2_slab_writethrough_ab.log).

__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(float* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                           (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL), 0x00020000);
}

__device__ __forceinline__ void store_slab4(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

// Reduce split-K partial slabs [SK][M][N] (f32) and apply the epilogue.
__global__ void gemm_splitk_reduce_kernel(const float* __restrict__ part, int SK, int M, int N,
                                          int epi, const bf16* __restrict__ bias,
                                          bf16* __restrict__ out, long ldo) {
  const int nout = epi == EPI_SILU ? N / 2 : N;
  const long total = (long)M * nout;
  const long slab = (long)M * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int m = (int)(e / nout), f = (int)(e % nout);
    if (epi == EPI_SILU) {
      const int g = f >> 4, w = f & 15;
      const long gi = (long)m * N + g * 32 + w, ui = gi + 16;
      float gs = 0.f, us = 0.f;
      for (int s = 0; s < SK; ++s) {
        gs += part[s * slab + gi];
        us += part[s * slab + ui];
      }
      store_out(out, ldo, m, f, silu(gs) * us);
    } else {
      const long i = (long)m * N + f;
      float acc = 0.f;
      for (int s = 0; s < SK; ++s) acc += part[s * slab + i];
      if (epi == EPI_BIAS) acc += bf2f(bias[f]);
      store_out(out, ldo, m, f, acc);
    }
  }
}

// Workspace head: kCounterBytes reserved ahead of the split-K slabs (the slab offset every
// consumer of deferred slabs uses, gemm_slab_offset_floats). Measured and removed: an in-kernel
// "last arriver reduces" fixup on these words; it only paid when sk x slab bytes per tile were
// a few tens of KB, and the decode plans write 256 KB per tile.
constexpr int kSplitCounters = 16384;
constexpr size_t kCounterBytes = kSplitCounters * sizeof(int);

// ---------------------------------------------------------------------------------------
// Skinny (decode) GEMM
// ---------------------------------------------------------------------------------------
constexpr int kSkThreads = 256;

template <int MT, int NT>
__device__ __forceinline__ void skinny_load(const bf16* __restrict__ W, const bf16* __restrict__ X,
                                            long ldw, long ldx, int n0, int kc, int lane, int M,
                                            bf16x8 (&a)[NT][4], bf16x8 (&b)[MT][4]) {
  // physical k of (lane group g, sub-step s, element j) = 32 s + 8 g + j: in each load
  // instruction the 4 lane groups of a row read 64 contiguous bytes.
  const int g = lane >> 4, r = lane & 15;
  const long kofs = (long)kc * 128 + 8 * g;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const bf16* p = W + (long)(n0 + 16 * t + r) * ldw + kofs;
#pragma unroll
    for (int s = 0; s < 4; ++s) a[t][s] = ld_nt(reinterpret_cast<const bf16x8*>(p + 32 * s));
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int m = 16 * mt + r;
    m = m < M ? m : M - 1;
    const bf16* p = X + (long)m * ldx + kofs;
#pragma unroll
    for (int s = 0; s < 4; ++s) b[mt][s] = *reinterpret_cast<const bf16x8*>(p + 32 * s);
  }
}

template <int MT, int NT>
__device__ __forceinline__ void skinny_mma(const bf16x8 (&a)[NT][4], const bf16x8 (&b)[MT][4],
                                           f32x4 (&acc)[NT][MT]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[t][mt] = mfma16(a[t][s], b[mt][s], acc[t][mt]);
}

// WK = waves of a workgroup that split K (their partials are summed through LDS); the other
// 4 / WK waves split N and share the same K range (their X fragments hit the same L1 lines).
template <int MT, int NT, int WK>
__global__ void __launch_bounds__(kSkThreads)
gemm_skinny_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                   int M, int N, int K, int epi, const bf16* __restrict__ bias,
                   bf16* __restrict__ out, long ldo, float* __restrict__ part) {
  constexpr int WN = 4 / WK;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wk = wid % WK, wn = wid / WK;
  const int nb0 = blockIdx.x * 16 * NT * WN;
  const int n0 = nb0 + wn * 16 * NT;
  const int nchunks = K / 128;
  const int S = gridDim.y * WK;
  const int s_idx = blockIdx.y * WK + wk;
  const int c0 = (int)(((long)nchunks * s_idx) / S), c1 = (int)(((long)nchunks * (s_idx + 1)) / S);

  f32x4 acc[NT][MT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[NT][4], b0[MT][4], a1[NT][4], b1[MT][4];
  int c = c0;
  if (c < c1) skinny_load<MT, NT>(W, X, ldw, ldx, n0, c, lane, M, a0, b0);
  // Two named register sets (runtime-indexed arrays would go to scratch: rule 20).
  while (c < c1) {
    if (c + 1 < c1) skinny_load<MT, NT>(W, X, ldw, ldx, n0, c + 1, lane, M, a1, b1);
    skinny_mma<MT, NT>(a0, b0, acc);
    ++c;
    if (c >= c1) break;
    if (c + 1 < c1) skinny_load<MT, NT>(W, X, ldw, ldx, n0, c + 1, lane, M, a0, b0);
    skinny_mma<MT, NT>(a1, b1, acc);
    ++c;
  }

  // Cross-wave reduction through LDS: red[wave][t][mt][i][lane], summed over the WK waves.
  constexpr int E = NT * MT * 4 * 64;
  __shared__ float red[4 * E];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wid * E + ((t * MT + mt) * 4 + i) * 64 + lane] = acc[t][mt][i];
  __syncthreads();

  const bool silu_epi = epi == EPI_SILU;
  for (int idx = threadIdx.x; idx < WN * E; idx += kSkThreads) {
    const int vn = idx / E, e = idx % E;
    const int l = e & 63, i = (e >> 6) & 3, tm = e >> 8;
    const int t = tm / MT, mt = tm % MT;
    const int m = 16 * mt + (l & 15);
    if (m >= M) continue;
    const int nw0 = nb0 + vn * 16 * NT;
    const int n = nw0 + 16 * t + (l >> 4) * 4 + i;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < WK; ++k) v += red[(vn * WK + k) * E + e];
    if (part) {
      part[(long)blockIdx.y * M * N + (long)m * N + n] = v;
    } else if (silu_epi) {
      if (t & 1) continue;  // the gate tile's thread combines with its up partner
      const int eu = e + MT * 4 * 64;  // same (mt, i, lane), tile t + 1
      float u = 0.f;
#pragma unroll
      for (int k = 0; k < WK; ++k) u += red[(vn * WK + k) * E + eu];
      const int f = nw0 / 2 + 16 * (t / 2) + (l >> 4) * 4 + i;
      store_out(out, ldo, m, f, silu(v) * u);
    } else {
      store_out(out, ldo, m, n, epi == EPI_BIAS ? v + bf2f(bias[n]) : v);
    }
  }
}

// ---------------------------------------------------------------------------------------
// LDS-tiled GEMM
// ---------------------------------------------------------------------------------------
constexpr int kTileThreads = 256;
constexpr int kBK = 64;

// Loads per wave per stage for a ROWS x 64 tile: every wave issues the same count (small
// tiles re-issue a piece another wave also loads: identical bytes to the same LDS address),
// so one compile-time `vmcnt` count is valid for every wave.
template <int ROWS>
constexpr int stage_loads() { return (ROWS / 8 + 3) / 4; }

// `nt`: stream the operand with the non-temporal policy (aux = 2) — for weights that exactly
// one workgroup reads once (decode, a single M tile): issued->landed ~18 % shorter and 5-10 %
// per decode layer on MI355X (MI355X_MICROARCH.md 'nt-weights'); never for re-read panels.
// PACKED: `src` is a weight in the K-tile-blocked layout [N/256][K/64][256][64] (pack_w256):
// a 256-row x 64-column block is 32 KiB of contiguous memory, so a 128-row stage reads 16 KiB
// in one run instead of 128 runs of 128 B one row pitch apart; `ld` then carries K.
template <int ROWS, bool GATHER = false, bool PACKED = false>
__device__ __forceinline__ void tile_stage(const bf16* __restrict__ src, long ld, int row0,
                                           int row_max, int k0, char* lds, int wid, int lane,
                                           const int* __restrict__ rows = nullptr, bool nt = false) {
  // ROWS x 64 bf16 = ROWS x 8 chunks of 16 B; one wave-instruction writes 8 rows (1 KiB).
  constexpr int kBlocks = ROWS / 8;
  constexpr int kInstr = stage_loads<ROWS>();
#pragma unroll
  for (int i = 0; i < kInstr; ++i) {
    int blk = i * 4 + wid;             // 8-row block index
    if (kBlocks % 4 != 0) blk %= kBlocks;
    const int row = blk * 8 + (lane >> 3);
    const int slot = lane & 7;
    const int chunk = slot ^ ((row >> 1) & 7);
    int gr = row0 + row;
    gr = gr < row_max ? gr : row_max - 1;
    if constexpr (GATHER) {
      if (rows) gr = rows[gr];   // grouped GEMM: row slot -> source token
    }
    const bf16* g = PACKED ? src + (((long)(gr >> 8) * (ld >> 6) + (k0 >> 6)) << 14) + (gr & 255) * 64 + chunk * 8
                           : src + (long)gr * ld + k0 + chunk * 8;
    if (nt)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)g, (lds_ptr_t)(lds + blk * 1024), 16, 0, 2);
    else
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)g, (lds_ptr_t)(lds + blk * 1024), 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ bf16x8 lds_frag(const char* lds, int row, int chunk) {
  const int slot = chunk ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + slot * 16);
}

// Epilogue of the tile and decode-ring GEMMs. W is their MFMA A operand, so the accumulators
// hold C^T: acc[i][j][r] = C[m = mw + 16i + (lane&15)][n = nw + 16j + 4(lane>>4) + r] — four
// consecutive columns per lane, stored as one 16-B slab write or one 8-B bf16 write.
// `pslab`: this workgroup's split-K slab from row m0 on (nullptr: apply the epilogue).
// `rsc`: RMSNorm row scale of a consumer GEMM (RowScale, ss == nullptr: none), applied to the
// accumulators first, so split-K slabs, the bias and the SiLU all see the normalised rows.
template <int TI, int TJ>
__device__ __forceinline__ void tile_epilogue(const f32x4 (&acc)[TI][TJ], int mw, int nw, int lane,
                                              int M, int N, int epi, const bf16* __restrict__ bias,
                                              bf16* __restrict__ out, long ldo, float* __restrict__ pslab,
                                              int m0, const RowScale& rsc) {
  const int lr = lane & 15, lc = 4 * (lane >> 4);
  const auto rs = slab_rsrc(pslab, pslab ? (long)(M - m0) * N * 4 : 0);
  const bool vec = (ldo & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0;
  float sc[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i) sc[i] = 1.f;
  if (rsc.ss != nullptr) {
    // sum of the row's partial sums of squares: the 4 lanes of a row (lane >> 4) take every
    // 4th group of 4 chunks as 16-B loads, all in flight together, then two shuffles (a norm
    // norm leaves a chunk per 1024 columns, but a serial loop of dependent loads over many
    // chunks cost ~20 us per consumer GEMM); chunks % 4 != 0: one chunk per lane and step
    const int q = lane >> 4, nc = rsc.chunks;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int m = min(mw + 16 * i + lr, M - 1);
      const float* sp = rsc.ss + (long)m * nc;
      float t = 0.f;
      if ((nc & 3) == 0) {
#pragma unroll 4
        for (int c = 4 * q; c < nc; c += 16) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(sp + c);
          t += (v[0] + v[1]) + (v[2] + v[3]);
        }
      } else {
        for (int c = q; c < nc; c += 4) t += sp[c];
      }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      sc[i] = rsqrtf(t * rsc.inv_dim + rsc.eps);
    }
  }
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int m = mw + 16 * i + lr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int n = nw + 16 * j + lc;
      if (pslab) {
        store_slab4(rs, ((m - m0) * N + n) * 4, acc[i][j] * sc[i]);
      } else if (epi == EPI_SILU || epi == EPI_SILU_GATE) {
        if constexpr (TJ % 2 == 0) {   // gate/up 16-row groups pair up inside the wave
          if (j & 1) continue;
          f32x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = silu(acc[i][j][r] * sc[i]) * (acc[i][j + 1][r] * sc[i]);
          const int f = nw / 2 + 16 * (j / 2) + lc;
          if (epi == EPI_SILU_GATE) {   // the 4 columns share an expert (gF % 16 == 0)
            const float g = rsc.gate[(long)m * rsc.gld + rsc.ge0 + f / rsc.gF];
#pragma unroll
            for (int r = 0; r < 4; ++r) h[r] = bf2f(f2bf(h[r])) * g;
          }
          store_out4(out, ldo, m, f, h, vec);
        }
      } else {
        f32x4 v = acc[i][j] * sc[i];
        if (epi == EPI_BIAS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bf2f(bias[n + r]);
        }
        store_out4(out, ldo, m, n, v, vec);
      }
    }
  }
}

// STAGES-deep glds pipeline: K-tiles kt+1 .. kt+STAGES-1 stay in flight (LDS-DMA) while the
// MFMAs consume tile kt. Each iteration waits with a COUNTED vmcnt (only tile kt must have
// landed) and a raw s_barrier (a __syncthreads() would drain every in-flight DMA:
// cdna_hip_programming.md §5 "Pipelining across barriers"); the buffer refilled in an
// iteration is the one every wave finished reading in the previous iteration (WAR safe).
//
// GROUPED (MoE expert GEMM, K13): blockIdx.x indexes a device-built tile list
// gtiles[i] = {expert, first row slot, end row slot} (count in *gcount; excess workgroups
// exit), blockIdx.z the N tile; the expert selects W + expert * w_estride and A rows are
// gathered through grows[slot] (nullptr: slots are rows). Output rows are row slots.
template <int BM, int BN, int WMW, int STAGES, bool GROUPED = false, bool PACKW = false>
__global__ void __launch_bounds__(kTileThreads)
gemm_tile_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                 int M, int N, int K, int epi, const bf16* __restrict__ bias,
                 bf16* __restrict__ out, long ldo, float* __restrict__ part,
                 const int* __restrict__ grows = nullptr,
                 const int4* __restrict__ gtiles = nullptr, const int* __restrict__ gcount = nullptr,
                 long w_estride = 0, RowScale rsc = RowScale{nullptr, 0, 0.f, 0.f}) {
  constexpr int WNW = 4 / WMW;                // waves along M x waves along N
  constexpr int WM = BM / WMW, WN = BN / WNW; // per-wave output tile
  constexpr int TI = WM / 16, TJ = WN / 16;  // MFMA tiles per wave
  constexpr int A_BYTES = BM * kBK * 2, B_BYTES = BN * kBK * 2;
  constexpr int LPW = stage_loads<BM>() + stage_loads<BN>();  // glds per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;  // one buffer = [A tile | B tile]

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WNW, wn = wid % WNW;
  int tile, m0, n0, ksplit = 0;
  const int m_slab = M;             // split-K slab row stride (grouped: all row slots)
  bool single = false;              // grouped: this expert has one row tile (W read once)
  if constexpr (GROUPED) {
    if ((int)blockIdx.x >= *gcount) return;
    const int4 info = gtiles[blockIdx.x];
    W += (long)info.x * w_estride;
    m0 = info.y;
    M = info.z;                     // rows [m0, M) of the permuted slot space
    single = info.w != 0;
    n0 = blockIdx.z * BN;
    tile = 0;
  } else {
    const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
    tile = xcd_remap((int)blockIdx.x, mtiles * ntiles);
    const int tn = tile / mtiles, tm = tile % mtiles;  // consecutive tiles share a W panel
    m0 = tm * BM;
    n0 = tn * BN;
  }
  ksplit = (int)blockIdx.y;
  const int nsplit = (int)gridDim.y;

  const int ktiles = K / kBK;
  const int kt0 = (int)(((long)ktiles * ksplit) / nsplit);
  const int kt1 = (int)(((long)ktiles * (ksplit + 1)) / nsplit);
  // each W byte read by one workgroup: stream it non-temporally
  const bool w_nt = (GROUPED ? single : M <= BM) && g_tile_w_nt;

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    if (kt0 + s < kt1) {
      char* b = smem + s * STAGE_BYTES;
      tile_stage<BM, GROUPED>(X, ldx, m0, M, (kt0 + s) * kBK, b, wid, lane, grows);
      tile_stage<BN, false, PACKW>(W, ldw, n0, N, (kt0 + s) * kBK, b + A_BYTES, wid, lane, nullptr, w_nt);
    }
  }
  int buf = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    // tiles issued after kt: min(STAGES - 2, kt1 - 1 - kt); wait until only those are pending
    const int after = min(STAGES - 2, kt1 - 1 - kt);
    if (STAGES >= 4 && after >= 2) vm_wait<(STAGES >= 4 ? 2 : 0) * LPW>();
    else if (STAGES >= 3 && after >= 1) vm_wait<LPW>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < kt1) {
      int nbuf = buf + STAGES - 1;
      if (nbuf >= STAGES) nbuf -= STAGES;
      char* nb = smem + nbuf * STAGE_BYTES;
      tile_stage<BM, GROUPED>(X, ldx, m0, M, (kt + STAGES - 1) * kBK, nb, wid, lane, grows);
      tile_stage<BN, false, PACKW>(W, ldw, n0, N, (kt + STAGES - 1) * kBK, nb + A_BYTES, wid, lane, nullptr, w_nt);
    }
    const char* As = smem + buf * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TI], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = lds_frag(As, wm * WM + 16 * i + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = lds_frag(Bs, wn * WN + 16 * j + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);   // C^T tile
    }
    if (++buf == STAGES) buf = 0;
  }
  tile_epilogue<TI, TJ>(acc, m0 + wm * WM, n0 + wn * WN, lane, M, N, epi, bias, out, ldo,
                        part ? part + (long)ksplit * m_slab * N + (long)m0 * N : nullptr, m0, rsc);
}

// ---------------------------------------------------------------------------------------
// Decode ring GEMM (kind 3; decode batches of 65-256 rows, e.g. TP2 replicas at 128 rows).
//
// Measured on MI355X (tools/exp_dec.py, N 57344 x K 8192): gemm_tile at BM = 128 streams
// weights at ~4.9-5.3 TB/s for ANY M (the time is flat in M: the kernel shape, not the
// arithmetic, is the limit), while 64-row tiles at two 4-wave workgroups per CU reach
// ~6.0 TB/s — but only for M <= 64 (a second row tile re-reads W through the per-CU load
// path: 3.9 TB/s at M = 128). The per-CU LDS-DMA stream scales with the number of waves
// issuing it, and X staged per K-tile competes with W for it. So this kernel:
//  * runs 8 waves per workgroup (NWM along M x NWN along N), one workgroup per CU;
//  * keeps X and W in separate LDS rings: X (L2-resident) needs 3 slots, W gets SW slots
//    (up to 160 KiB in all), so SW-1 weight K-tiles stream while the MFMAs consume tile kt;
//  * uses wide N tiles (BN up to 256: 224 makes N = 57344 exactly 256 tiles) so X is at most
//    half of the staged bytes at BM = 128.
// Issue order per iteration is W(kt+SW-1) then X(kt+2), so X(kt) is always the later of the
// two loads tile kt needs and one counted vmcnt covers both: LW + LX loads were issued after
// X(kt) in steady state; in the tail the wait is exact or conservative.
// ---------------------------------------------------------------------------------------
template <int ROWS, int NW>
constexpr int ring_loads() { return (ROWS / 8 + NW - 1) / NW; }

template <int ROWS, int NW>
__device__ __forceinline__ void ring_stage(const bf16* __restrict__ src, long ld, int row0, int row_max,
                                           int k0, char* lds, int wid, int lane, bool nt) {
  constexpr int kBlocks = ROWS / 8;   // 8-row blocks of 1 KiB; one wave-instruction each
#pragma unroll
  for (int i = 0; i < ring_loads<ROWS, NW>(); ++i) {
    int blk = i * NW + wid;
    if (kBlocks % NW != 0) blk %= kBlocks;   // surplus lanes re-load a block (same bytes)
    const int row = blk * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    int gr = row0 + row;
    gr = gr < row_max ? gr : row_max - 1;
    const bf16* g = src + (long)gr * ld + k0 + chunk * 8;
    if (nt)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)g, (lds_ptr_t)(lds + blk * 1024), 16, 0, 2);
    else
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)g, (lds_ptr_t)(lds + blk * 1024), 16, 0, 0);
  }
}

constexpr int kDecThreads = 512;

template <int BM, int BN, int NWM, int NWN, int SW>
__global__ void __launch_bounds__(kDecThreads)
gemm_dec_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                int M, int N, int K, int epi, const bf16* __restrict__ bias,
                bf16* __restrict__ out, long ldo, float* __restrict__ part, RowScale rsc) {
  constexpr int SX = 3, NW = NWM * NWN;
  static_assert(NW * 64 <= kDecThreads && SW >= SX, "decode ring configuration");
  constexpr int WM = BM / NWM, WN = BN / NWN;   // per-wave output block
  constexpr int TI = WM / 16, TJ = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "per-wave block must be whole MFMA tiles");
  constexpr int XB = BM * kBK * 2, WB = BN * kBK * 2;
  constexpr int LX = ring_loads<BM, NW>(), LW = ring_loads<BN, NW>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const xs = smem;
  char* const wsm = smem + SX * XB;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / NWN, wn = wid % NWN;
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int tile = xcd_remap((int)blockIdx.x, mtiles * ntiles);
  const int ksplit = (int)blockIdx.y;
  const int tn = tile / mtiles, tm = tile % mtiles;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nsplit = (int)gridDim.y;
  const int ktiles = K / kBK;
  const int kt0 = (int)(((long)ktiles * ksplit) / nsplit);
  const int kt1 = (int)(((long)ktiles * (ksplit + 1)) / nsplit);
  const bool w_nt = mtiles == 1 && g_tile_w_nt;   // each weight byte read by one workgroup

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue = the issue pattern of virtual iterations kt0-SW+1 .. kt0-1: W(kt0 .. kt0+SW-2)
  // and, lagging by SW-SX, X(kt0 .. kt0+1). Slot of K-tile t: (t - kt0) mod S.
#pragma unroll
  for (int v = 0; v < SW - 1; ++v) {
    if (kt0 + v < kt1) ring_stage<BN, NW>(W, ldw, n0, N, (kt0 + v) * kBK, wsm + v * WB, wid, lane, w_nt);
    const int xv = v - (SW - SX);
    if (xv >= 0 && kt0 + xv < kt1) ring_stage<BM, NW>(X, ldx, m0, M, (kt0 + xv) * kBK, xs + xv * XB, wid, lane, false);
  }
  int xslot = 0, wslot = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    // loads issued after X(kt): iteration kt-1's W(kt+SW-2) (if any) and X(kt+1) (if any)
    if (kt + SW - 2 < kt1) vm_wait<LW + LX>();
    else if (kt + 1 < kt1) vm_wait<LX>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // refill the slots every wave finished reading in iteration kt-1
    const int wfill = wslot == 0 ? SW - 1 : wslot - 1;
    const int xfill = xslot == 0 ? SX - 1 : xslot - 1;
    if (kt + SW - 1 < kt1) ring_stage<BN, NW>(W, ldw, n0, N, (kt + SW - 1) * kBK, wsm + wfill * WB, wid, lane, w_nt);
    if (kt + SX - 1 < kt1) ring_stage<BM, NW>(X, ldx, m0, M, (kt + SX - 1) * kBK, xs + xfill * XB, wid, lane, false);
    const char* As = xs + xslot * XB;
    const char* Bs = wsm + wslot * WB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = lds_frag(As, wm * WM + 16 * i + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const bf16x8 b = lds_frag(Bs, wn * WN + 16 * j + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
        for (int i = 0; i < TI; ++i) acc[i][j] = mfma16(b, af[i], acc[i][j]);   // C^T tile
      }
    }
    if (++xslot == SX) xslot = 0;
    if (++wslot == SW) wslot = 0;
  }
  tile_epilogue<TI, TJ>(acc, m0 + wm * WM, n0 + wn * WN, lane, M, N, epi, bias, out, ldo,
                        part ? part + (long)ksplit * M * N + (long)m0 * N : nullptr, m0, rsc);
}

// Prefill tiles are walked in GROUP_M super-rows inside each XCD's contiguous range, so the
// 32 CUs of an XCD share X and W panels in their L2.
constexpr int kBigGroupM = 8;

// ---------------------------------------------------------------------------------------
// 8-phase big-tile GEMM (prefill): 256x256 tile, BK = 64, two K-tile LDS buffers (128 KiB),
// 8 waves (2 along M x 4 along N, 128x64 outputs each) in two groups staggered by one barrier
// (group wr = 1 starts one s_barrier later), so on every SIMD one wave runs a 16-MFMA segment
// while its partner reads fragments and issues DMA (cdna_hip_programming.md §5 "The 256²
// 8-phase template", T3+T4+T5).
//
// A K-tile is consumed in 4 phases, one C-quadrant of the wave's 128x64 block each:
//   q0: rows 0-63 x cols 0-31   reads A-lo (8 ds_read_b128) + B-lo (4)
//   q1: rows 0-63 x cols 32-63  reads B-hi (4)            (A-lo kept in registers)
//   q2: rows 64-127 x cols 32-63 reads A-hi (8)           (B-hi kept)
//   q3: rows 64-127 x cols 0-31  no reads                 (A-hi, B-lo kept)
// so each of the K-tile's four half-tiles (A-lo = rows {0-63, 128-191}, A-hi = {64-127,
// 192-255}, B-lo = cols {0-31, 64-95, ...}, B-hi = the other 32-column groups; 16 KiB each) is
// read completely in ONE phase. Every phase issues one half-tile of DMA (2 glds per wave) into
// a half that was fully read (and retired by lgkmcnt(0) before a barrier every reader passed)
// in an earlier phase: K-tile k's halves go out at phases 4(k-2)+{2,3,4,5} (A-lo, B-lo, B-hi,
// A-hi), i.e. one phase after the same half of K-tile k-2 was read. The counted wait is in
// phase 4k only (the K-tile's last phase): vmcnt(6) leaves the 3 half-tiles issued after A-hi(k)
// in flight and retires all of K-tile k, which is read from phase 4k+1 on (one phase after the
// wait, behind a barrier both groups pass: the template's RAW rule). Raw s_barrier only: a
// __syncthreads() would drain the DMA in flight (§5 "Pipelining across barriers").
// The fragment schedule on top of that (the prefill kernel for every M > 256, plan kind 4):
//  * early LDS release: A-lo is the one half restaged one phase after its read, so only its
//    reads must retire before a phase's barrier (lgkmcnt(4) after A first, B last); every
//    other read completes inside the wave's own MFMA segment;
//  * lookahead: the A-lo fragments of K-tile k+1 are read in phase q3 of K-tile k (whose read
//    segment is otherwise empty), and its B-lo fragments right behind q3's MFMAs (b_lo(k)'s
//    last use), so q0 reads nothing and no read latency sits behind a barrier. A counted wait
//    in q2 retires this wave's A-lo / B-lo(k+1) DMA, and the barrier ending q2 of group 0 (=
//    the one starting q2's MFMAs of group 1) is passed by both groups before either reads;
//  * buffer-descriptor staging: the tile's A / B rows start at an SGPR base (the descriptor),
//    the K offset and the hi-half row shift ride in the scalar soffset (A-hi = A-lo + 64 rows,
//    B-hi = B-lo + 32 rows: the same XOR pattern, which depends on row bits 1-3 only), each lane
//    keeps 4 constant byte offsets, and A rows past M read as zeros instead of a clamped
//    re-read (VALU per K-tile 49 -> 24).
// 1.39-1.40 PF at M = 8192 on the 70B projections, +4.6-5.2 % over the schedule without the
// lookahead and descriptors (profiles/r4_gemm_prefill_la.log, r4_gemm_prefill_lb.log).
// Measured and dropped (profiles/r3_gemm_prefill_pmc.md, r4_gemm_prefill_{bal,lh}.log):
//  - the round-2 5-slot BK-32 ring kernel (8 waves, one 16x16x32 K-step per barrier):
//    2-7 % slower at M = 8192, within -3..+32 % at M = 256/512;
//  - one wave per SIMD, 4 waves x 128x128 per wave (hipBLASLt's shape: MT256x256x64, 256
//    threads): 32x32x16 with a 4/5-slot BK-32 glds ring 1.07-1.10 PF; 16x16x32 with buffer
//    loads to LDS and the second MFMA half deferred behind the next K-tile's reads 1.13-1.23
//    PF; the same with BK 64 in a 2-slot ring 1.00-1.12 PF (WAIT_ANY x3: one K-tile of lead
//    does not cover HBM latency). All at 49-52 % MFMA-busy cycles against hipBLASLt's 87 %;
//  - the 24 reads spread 6 / 6 / 6 / 6 over the four read segments (0.7-1.5 % slower), A-hi
//    read in q0's empty segment (1.5-2.8 % slower), and the plain / early-release-only
//    schedules (plan mt 0-3 of round 4).
// ---------------------------------------------------------------------------------------
constexpr int kB8Threads = 512;
constexpr int kB8LdsBytes = 2 * 2 * 256 * 128;   // 2 buffers x (A, B) x 256 rows x 128 B

// LDS row-block (8 rows x 128 B = 1 KiB) of the h-th DMA instruction of half-tile `half`
// (0 A-lo / 1 B-lo / 2 B-hi / 3 A-hi; h in 0..15: instruction 2*wave + {0,1}).
__device__ __forceinline__ int b8_block(int half, int h) {
  if (half == 0 || half == 3) {            // A: rows {0-63,128-191} (lo) or {64-127,192-255} (hi)
    const int base = half == 0 ? 0 : 8;
    return (h < 8 ? base + h : 16 + base + (h - 8));
  }
  // B: 32-row groups g (0..3) at rows 64g + (hi ? 32 : 0); 4 blocks per group
  const int g = h >> 2, b = h & 3;
  return g * 8 + (half == 2 ? 4 : 0) + b;
}

struct B8Dma {
  int a[2], b[2];
};

__device__ __forceinline__ B8Dma b8_dma_offsets(long ldx, long ldw, int wid, int lane) {
  B8Dma d;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ra = b8_block(0, 2 * wid + i) * 8 + (lane >> 3);
    const int rb = b8_block(1, 2 * wid + i) * 8 + (lane >> 3);
    d.a[i] = (int)((ra * ldx + (((lane & 7) ^ ((ra >> 1) & 7)) * 8)) * 2);
    d.b[i] = (int)((rb * ldw + (((lane & 7) ^ ((rb >> 1) & 7)) * 8)) * 2);
  }
  return d;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t b8_rsrc(const bf16* base, long rows, long ld) {
  const long bytes = rows * ld * 2;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}

__device__ __forceinline__ void b8_stage_buf(__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, long ldx,
                                             long ldw, int k0, char* buf, int half, int wid, const B8Dma& d) {
  const bool isA = half == 0 || half == 3;
  char* lds = buf + (isA ? 0 : 256 * 128);
  const int shift = half == 3 ? (int)(64 * ldx * 2) : half == 2 ? (int)(32 * ldw * 2) : 0;
  const int soff = k0 * 2 + shift;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = b8_block(half, 2 * wid + i);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? ra : rb, (lds_ptr_t)(lds + blk * 1024), 16, isA ? d.a[i] : d.b[i],
                                             soff, 0, 0);
  }
}

// GROUPED (MoE expert GEMM at prefill scale, K13): the M tiles are the entries of a device-built
// tile list gtiles[i] = {expert, first row slot, end row slot, -} (count in *gcount, up to
// `M` = the list's capacity; excess workgroups exit): the expert selects W + expert *
// w_estride, and the A rows of slot s are the token rows grows[s] (nullptr: slot s itself),
// gathered by per-lane LDS-DMA addresses (rows past the tile's end re-read its last row; their
// outputs are not stored). Output rows are slots. Consecutive list entries are mostly tiles of
// one expert, so the GROUP_M walk shares the expert's weight panels in an XCD's L2.
__device__ __forceinline__ void b8_stage_gather(const bf16* const (&arow)[4], int k0, char* buf, int half, int wid) {
  const int base = half == 3 ? 2 : 0;   // A-lo: pointers 0, 1; A-hi: 2, 3
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = b8_block(half, 2 * wid + i);
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(arow[base + i] + k0), (lds_ptr_t)(buf + blk * 1024), 16, 0, 0);
  }
}

template <bool GROUPED = false>
__global__ void __launch_bounds__(kB8Threads)
gemm_big8_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                 int M, int N, int K, int epi, const bf16* __restrict__ bias,
                 bf16* __restrict__ out, long ldo, float* __restrict__ part,
                 const int* __restrict__ grows = nullptr, const int4* __restrict__ gtiles = nullptr,
                 const int* __restrict__ gcount = nullptr, long w_estride = 0) {
  constexpr int BM = 256, BN = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;   // GROUPED: M = tile-list capacity x BM
  const int t = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int per_group = kBigGroupM * ntiles;
  const int grp = t / per_group, first_m = grp * kBigGroupM;
  const int gsize = min(mtiles - first_m, kBigGroupM);
  int m0 = (first_m + (t % per_group) % gsize) * BM;
  const int n0 = ((t % per_group) / gsize) * BN;
  const bf16* arow[4] = {};
  if constexpr (GROUPED) {
    const int ti = m0 / BM;
    if (ti >= *gcount) return;
    const int4 info = gtiles[ti];
    W += (long)info.x * w_estride;
    m0 = info.y;
    M = info.z;                    // rows [m0, M) of the slot space
    // this lane's A rows: the 4 row blocks it DMAs (A-lo: b8_block(0, 2 wid + i), A-hi: (3, ...))
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = b8_block(i < 2 ? 0 : 3, 2 * wid + (i & 1)) * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      int slot = m0 + row;
      slot = slot < M ? slot : M - 1;
      const long src = grows != nullptr ? grows[slot] : slot;
      arow[i] = X + src * ldx + chunk * 8;
    }
  }
  const int ktiles = K / 64;
  const int kt0 = (int)(((long)ktiles * blockIdx.y) / gridDim.y);
  const int kt1 = (int)(((long)ktiles * (blockIdx.y + 1)) / gridDim.y);
  const int nk = kt1 - kt0;   // >= 2 (host check)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto bufp = [&](int k) -> char* { return smem + (k & 1) * (2 * 256 * 128); };
  // descriptors at the tile's first A / B row (SGPRs), 4 per-lane offsets
  const auto rsa = b8_rsrc(X + (long)m0 * ldx, M - m0, ldx);
  const auto rsb = b8_rsrc(W + (long)n0 * ldw, N - n0, ldw);
  const B8Dma dma = b8_dma_offsets(ldx, ldw, wid, lane);
  auto stage = [&](int k, int half) {
    if (GROUPED && (half == 0 || half == 3))
      b8_stage_gather(arow, (kt0 + k) * 64, bufp(k), half, wid);
    else
      b8_stage_buf(rsa, rsb, ldx, ldw, (kt0 + k) * 64, bufp(k), half, wid, dma);
  };
  // prologue: all of K-tile 0, then A-lo, B-lo, B-hi of K-tile 1 (the load stream's order)
  stage(0, 0); stage(0, 1); stage(0, 2); stage(0, 3);
  stage(1, 0); stage(1, 1); stage(1, 2);
  vm_wait<6>();                          // K-tile 0 landed (this wave's part)
  __builtin_amdgcn_s_barrier();          // every wave's part
  if (wr == 1) __builtin_amdgcn_s_barrier();

  const int ar = wr * 128 + (lane & 15);  // A fragment row of block i: ar + 16 i
  const int bc = wc * 64 + (lane & 15);   // B fragment row (output column) of block j
  bf16x8 a_lo[4][2], a_hi[4][2], b_lo[2][2], b_hi[2][2];
  auto read_a_lo = [&](const char* As) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a_lo[i][ks] = lds_frag(As, ar + 16 * i, ks * 4 + (lane >> 4));
  };
  auto read_b_lo = [&](const char* Bs) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b_lo[j][ks] = lds_frag(Bs, bc + 16 * j, ks * 4 + (lane >> 4));
  };
  read_a_lo(bufp(0));
  read_b_lo(bufp(0) + 256 * 128);
  for (int k = 0; k < nk; ++k) {
    const char* As = bufp(k);
    const char* Bs = As + 256 * 128;
    const bool more = k + 1 < nk, more2 = k + 2 < nk;
    // ---- q0: (A-lo, B-lo read ahead); DMA A-hi(k+1)
    if (more) stage(k + 1, 3);
    asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(b_lo[j][ks], a_lo[i][ks], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- q1: read B-hi; DMA A-lo(k+2) (A-lo(k) was read in q3 of k-1)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b_hi[j][ks] = lds_frag(Bs, bc + 32 + 16 * j, ks * 4 + (lane >> 4));
    if (more2) stage(k + 2, 0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][2 + j] = mfma16(b_hi[j][ks], a_lo[i][ks], acc[i][2 + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- q2: read A-hi; DMA B-lo(k+2)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a_hi[i][ks] = lds_frag(As, ar + 64 + 16 * i, ks * 4 + (lane >> 4));
    if (more2) stage(k + 2, 1);
    // this wave's A-lo / B-lo(k+1) DMA retired (left in flight: B-hi, A-hi(k+1) and, while
    // K-tile k+2 exists, A-lo / B-lo(k+2))
    if (more2) vm_wait<8>();
    else if (more) vm_wait<4>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 + i][2 + j] = mfma16(b_hi[j][ks], a_hi[i][ks], acc[4 + i][2 + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- q3: read A-lo(k+1); DMA B-hi(k+2); retire K-tile k+1
    // a_lo(k) is dead since q1; q3's MFMAs use a_hi / b_lo. Unconditional (past the last K-tile
    // it reads the other buffer's stale image, never used), and pinned here: under a branch the
    // scheduler sank the reads behind q3's MFMAs and barrier, i.e. back into q0
    read_a_lo(bufp(k + 1));
    __builtin_amdgcn_sched_barrier(0);
    if (more2) stage(k + 2, 2);
    if (more2) vm_wait<6>();   // A-hi(k+1) and older landed; A-lo/B-lo/B-hi(k+2) fly
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 + i][j] = mfma16(b_lo[j][ks], a_hi[i][ks], acc[4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
    // B-lo(k+1) behind q3's MFMAs, so its latency is spent in the barrier and q0's read segment
    // instead of after q0's barrier (its DMA retired with q2's wait)
    read_b_lo(bufp(k + 1) + 256 * 128);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();   // re-align the groups' barrier counts
  tile_epilogue<8, 4>(acc, m0 + wr * 128, n0 + wc * 64, lane, M, N, epi, bias, out, ldo,
                      part ? part + (long)blockIdx.y * M * N + (long)m0 * N : nullptr, m0,
                      RowScale{nullptr, 0, 0.f, 0.f});
}

// ---------------------------------------------------------------------------------------
// One wave per SIMD, 256x256 tile (plan kind 6, "big4"): 4 waves in 2 x 2, each owning a 128 x
// 128 output block (8 x 8 mfma_16x16x32 accumulators, 256 registers: the AGPR half of the
// 512-register file a lone wave gets). Per K-tile (BK = 64) a wave reads 32 fragments (16 KiB
// of A and B rows) for 128 MFMAs: a third fewer LDS bytes per FLOP than big8's 128 x 64 wave
// tile, whose fragment reads plus DMA writes fill the LDS port.
// LDS (160 KiB, all of it): LDS-DMA rings of whole K-tile halves, 3 slots of A (activation
// rows) and 2 of B (weight rows), 32 KiB each: no staging registers (those pushed the allocator
// into moving accumulators every K-tile). A gets the deeper ring: an XCD's 32 resident tiles
// are 8 row tiles x 4 column tiles (GROUP_M walk), so A misses its L2 twice as often as B.
// One barrier per K-tile, between its two k-steps (ks):
//   ks 0 of K-tile t: MFMAs on the ks-0 fragments; read the ks-1 fragments of t; DMA A(t+2)
//     into A slot (t+2) % 3, which K-tile t-1 left before the previous barrier;
//   own DMA of A(t+1), B(t+1) retired (vmcnt 8: A(t+2) flies), lgkmcnt(0), s_barrier;
//   ks 1: MFMAs on the ks-1 fragments; read the ks-0 fragments of t+1; DMA B(t+2) into B slot
//     t % 2 — K-tile t's last reads (its ks-1 fragments) are before this barrier in every wave.
// Source order is the schedule: each k-step is 16 slots of {4 MFMAs, 1 fragment read, a DMA
// every other slot} fenced by sched_barrier(0) (cdna_hip_programming.md T19: left alone, the
// scheduler clusters the memory operations, and a lone wave has nothing to hide the stall
// behind). A lane's fragments of one (slot, ks) share one address VGPR (immediate offsets: 4
// VALU per K-tile). Branch-free: past the last K-tile the DMA re-reads it into a slot nobody
// reads any more (a guard made hipcc wait vmcnt(0) per slot: 3.5x slower).
// Measured (profiles/r5_gemm_big4/): 1.52-1.55 PF at M = 8192 on the Llama-3-70B projections
// against 1.39-1.47 for gemm_big8_kernel and 1.53-1.64 for hipBLASLt on the same box. Steps that
// got it there from 1.0 PF: LDS-DMA rings instead of register staging (no accumulator moves),
// one loop with no peeled iterations, one fragment read per slot (not two), the loop rotated to
// end on the barrier, A's DMA moved into ks 0, immediate-offset fragment addresses.
// ---------------------------------------------------------------------------------------
constexpr int kB4Threads = 256;
constexpr int kB4Slot = 256 * 128;                 // one operand half of a K-tile: 32 KiB
constexpr int kB4LdsBytes = 5 * kB4Slot;           // A slots 0-2, B slots 3-4: 160 KiB

__device__ __forceinline__ void b4_dma(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, voff, soff, 0, 0);
}

// GROUPED (MoE expert GEMM at prefill scale): as gemm_big8_kernel<true> — M tiles are the
// entries of the device tile list {expert, first row slot, end slot}, W is offset by the expert,
// A rows are gathered through grows[slot] by per-lane LDS-DMA offsets from X (rows past the
// tile's end re-read its last row; their outputs are not stored).
template <bool GROUPED = false>
__global__ void __launch_bounds__(kB4Threads) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_big4_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                 int M, int N, int K, int epi, const bf16* __restrict__ bias,
                 bf16* __restrict__ out, long ldo, float* __restrict__ part,
                 const int* __restrict__ grows = nullptr, const int4* __restrict__ gtiles = nullptr,
                 const int* __restrict__ gcount = nullptr, long w_estride = 0) {
  constexpr int BM = 256, BN = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // wave index in an SGPR: the DMA's LDS destinations (M0) and the fragment row bases are then
  // scalar (a VGPR wave index cost a readfirstlane + s_nop per DMA instruction)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int t = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int per_group = kBigGroupM * ntiles;
  const int grp = t / per_group, first_m = grp * kBigGroupM;
  const int gsize = min(mtiles - first_m, kBigGroupM);
  int m0 = (first_m + (t % per_group) % gsize) * BM;
  const int n0 = ((t % per_group) / gsize) * BN;
  if constexpr (GROUPED) {
    const int ti = m0 / BM;
    if (ti >= *gcount) return;
    const int4 info = gtiles[ti];
    W += (long)info.x * w_estride;
    m0 = info.y;
    M = info.z;                    // rows [m0, M) of the slot space
  }
  const int ktiles = K / 64;
  const int kt0 = (int)(((long)ktiles * blockIdx.y) / gridDim.y);
  const int kt1 = (int)(((long)ktiles * (blockIdx.y + 1)) / gridDim.y);
  const int nk = kt1 - kt0;   // >= 2 (host check)

  // DMA: instruction s (0..7) of wave w fills LDS row block 8 w + s (8 rows x 128 B, lane-
  // linear); lane L supplies row 8 (8 w + s) + (L >> 3) at the chunk lds_frag expects in
  // position L & 7: chunk = (L & 7) ^ ((row >> 1) & 7) = (L & 7) ^ ((L >> 4) + 4 (s & 1)) & 7
  const auto rsa = b8_rsrc(X + (long)m0 * ldx, M - m0, ldx);   // A rows past M read zeros
  const auto rsb = b8_rsrc(W + (long)n0 * ldw, N - n0, ldw);
  const int drow = 64 * wid + (lane >> 3);
  int va[2], vb[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int ch = (lane & 7) ^ (((lane >> 4) + 4 * e) & 7);
    va[e] = (int)((drow * ldx + ch * 8) * 2);
    vb[e] = (int)((drow * ldw + ch * 8) * 2);
  }
  int ga[8] = {};   // GROUPED: byte offsets from X of this lane's gathered rows (at its chunk)
  const auto rsx = b8_rsrc(X, 1L << 30, 1);
  if constexpr (GROUPED) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int slot = min(m0 + drow + 8 * q, M - 1);
      const long src = grows != nullptr ? grows[slot] : slot;
      ga[q] = (int)((src * ldx + (((lane & 7) ^ (((lane >> 4) + 4 * (q & 1)) & 7)) * 8)) * 2);
    }
  }
  auto dma_a = [&](int k, int slot, int s) {
    if constexpr (GROUPED)
      b4_dma(rsx, smem + slot * kB4Slot + (8 * wid + s) * 1024, ga[s], (kt0 + k) * 128);
    else
      b4_dma(rsa, smem + slot * kB4Slot + (8 * wid + s) * 1024, va[s & 1], (kt0 + k) * 128 + (int)(8 * s * ldx * 2));
  };
  auto dma_b = [&](int k, int slot, int s) {
    b4_dma(rsb, smem + (3 + slot) * kB4Slot + (8 * wid + s) * 1024, vb[s & 1], (kt0 + k) * 128 + (int)(8 * s * ldw * 2));
  };
  const int fr = lane & 15, fq = lane >> 4;
  // fragment idx 0-7: B rows (output columns) 16 idx, 8-15: A rows 16 (idx - 8), of k-step ks.
  // lds_frag's swizzle depends on row bits 1-3 = fr bits 1-3 only, so a lane's fragments of one
  // (slot, ks) share one VGPR address and differ by immediates of 2048 B (16 rows)
  int lo[2][2];   // [operand A / B][ks] lane byte offset inside a slot
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int ch = ((ks * 4 + fq) ^ ((fr >> 1) & 7)) * 16;
    lo[0][ks] = (wr * 128 + fr) * 128 + ch;
    lo[1][ks] = (wc * 128 + fr) * 128 + ch;
  }
  auto rd1 = [&](int sa_, int sb_, int ks, int idx, bf16x8 (&f)[16]) {
    const char* p = idx < 8 ? smem + (3 + sb_) * kB4Slot + lo[1][ks] + 2048 * idx
                            : smem + sa_ * kB4Slot + lo[0][ks] + 2048 * (idx - 8);
    f[idx] = *reinterpret_cast<const bf16x8*>(p);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // MFMA group n (0..15): output row block i = n / 2, column blocks 4 (n & 1) .. + 3
  auto mf4 = [&](int n, const bf16x8 (&f)[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = n >> 1, j = 4 * (n & 1) + q;
      acc[i][j] = mfma16(f[j], f[8 + i], acc[i][j]);
    }
  };
  bf16x8 f0[16], f1[16];   // all fragments of k-step 0 / k-step 1

  // prologue: A(0), B(0), A(1), B(1), A(2) (the ring's load order: B(t+2) then A(t+3))
#pragma unroll
  for (int s = 0; s < 8; ++s) dma_a(0, 0, s);
#pragma unroll
  for (int s = 0; s < 8; ++s) dma_b(0, 0, s);
#pragma unroll
  for (int s = 0; s < 8; ++s) dma_a(1, 1, s);
#pragma unroll
  for (int s = 0; s < 8; ++s) dma_b(1, 1, s);
  vm_wait<16>();                      // K-tile 0 landed (own part); A(1), B(1) fly
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int idx = 0; idx < 16; ++idx) rd1(0, 0, 0, idx, f0);

  // The loop is rotated so its back edge sits right after the barrier (the compiler puts a
  // conservative lgkmcnt(0) at a loop header: there it finds nothing outstanding): iteration k =
  // ks 1 of K-tile k, then ks 0 of K-tile k + 1, then the barrier; the last ks 1 is peeled.
  auto ks0 = [&](int k, int sa_, int sb_) {   // ks 0 of K-tile k: its ks-1 fragments read
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      mf4(n, f0);
      // A(k+2) into the slot K-tile k-1 left (its last reads precede the previous barrier)
      if (n & 1) dma_a(min(k + 2, nk - 1), sa_ == 0 ? 2 : sa_ - 1, n >> 1);
      rd1(sa_, sb_, 1, n, f1);
      __builtin_amdgcn_sched_barrier(0);
    }
    vm_wait<8>();                     // A(k+1), B(k+1) landed; A(k+2) may fly
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  auto ks1 = [&](int k, int sa_, int sb_, int sa1_) {   // ks 1 of K-tile k: next ks-0 read, DMA
    const int kb = min(k + 2, nk - 1);
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      mf4(n, f1);
      rd1(sa1_, sb_ ^ 1, 0, n, f0);
      if (n & 1) dma_b(kb, sb_, n >> 1);   // B(k+2) into the slot K-tile k just left
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int sa = 0;   // A slot of K-tile k (k % 3)
  ks0(0, 0, 0);
  for (int k = 0; k + 1 < nk; ++k) {
    const int sb = k & 1, sa1 = sa == 2 ? 0 : sa + 1;
    ks1(k, sa, sb, sa1);
    ks0(k + 1, sa1, sb ^ 1);
    sa = sa1;
  }
  ks1(nk - 1, sa, (nk - 1) & 1, sa == 2 ? 0 : sa + 1);
  vm_wait<0>();                       // no LDS-DMA may outlive the workgroup
  tile_epilogue<8, 8>(acc, m0 + wr * 128, n0 + wc * 128, lane, M, N, epi, bias, out, ldo,
                      part ? part + (long)blockIdx.y * M * N + (long)m0 * N : nullptr, m0,
                      RowScale{nullptr, 0, 0.f, 0.f});
}

// ---------------------------------------------------------------------------------------
// Mid-M GEMM (plan kind 5): the tensor-parallel shard projections at M = 128-512 rows (tp2-tp8
// decode at 64 sequences per GPU, large single-GPU batches), where a 256x256 tile grid leaves
// most of the 256 CUs idle (tp8 QKV at M = 512: 10 tiles) and the 4-wave tile kernel keeps the
// matrix pipe ~25 % busy (one wave per SIMD, every K-tile behind one barrier).
//
// 8 waves in two groups of 4 staggered by one s_barrier (big8's scheme): each wave owns a
// 64 x WN output block (WN = 64 for 256x128 / 128x256 tiles, 32 for 128x128), and every
// K-tile (BK = 64) is two k-steps of 32. Per k-step a wave has a READ segment (its A and B
// fragments of that k-step, TI + TJ ds_read_b128, and half of its share of the LDS-DMA) and an
// MFMA segment (TI x TJ mfma_16x16x32). Group 1 runs one barrier behind group 0, so on every
// SIMD one wave's MFMA segment overlaps its partner's read segment:
//     global segment:  4k     4k+1   4k+2   4k+3   (k = K-tile)
//     group 0:         R0(k)  M0(k)  R1(k)  M1(k)
//     group 1:         M1(k-1) R0(k) M0(k)  R1(k)
// LDS: two rings of K-tile images (128-B rows, XOR-swizzled like lds_frag): SX slots of the
// activation rows X (BM x 64, mostly L2 hits: short latency) and SW >= SX slots of the weight
// rows W (BN x 64, streamed from HBM: the deep one). Iteration k issues X(k + SX - 1) in its
// first read segment and W(k + SW - 1) in its second, each into the slot of K-tile k - 1,
// whose last reader (group 1's R1(k-1), global segment 4k-1) retired its reads (lgkmcnt(0))
// before the barrier opening segment 4k. RAW: K-tile k+1 is first read in global segment 4k+4
// (group 0's R0(k+1)), so every wave retires its own DMA of K-tile k+1 before the barrier that
// closes segment 4k+3: group 0 at the end of M1(k), group 1 at the end of R1(k); the counted
// wait leaves exactly the loads issued after the later of X(k+1) / W(k+1) in flight (counted
// at run time near the tail, where the load stream thins out).
// DMA through buffer descriptors based at the tile's first row (A rows past M read zeros);
// weights streamed non-temporally when one row tile covers M (each byte read by one workgroup).
// Grid: 1-D, split-major then N-tile then M-tile, XCD-remapped, so an XCD's consecutive
// workgroups share a weight panel (and K range) across the M tiles in its L2.
// Measured (profiles/r5_gemm): one ring of whole K-tiles (SX = SW = 3) kept the matrix pipe
// 29 % busy on the tp8 down projection at M = 512, the waves parked on the DMA wait (SQ_WAIT_ANY
// 35 %) with 75 % L2 hits: the weight stream's latency, not the MFMA or LDS issue, bounds it.
// ---------------------------------------------------------------------------------------
constexpr int kMidThreads = 512;

template <int BM, int BN, int SX, int SW>
struct MidCfg {
  static constexpr int WM = 64;                          // wave rows
  static constexpr int WN = (BM * BN) / (8 * WM);        // wave columns: 8 waves cover the tile
  static constexpr int WGN = BN / WN, WGM = BM / WM;     // wave grid
  static constexpr int TI = WM / 16, TJ = WN / 16;
  static constexpr int XB = BM * 128, WB = BN * 128;     // bytes per X / W slot
  static constexpr int LX = BM / 64, LW = BN / 64;       // DMA instructions per wave per K-tile
  static constexpr int LDS = SX * XB + SW * WB;
  static_assert(WGM * WGN == 8 && WN % 16 == 0, "mid tile shape");
  static_assert(SX >= 2 && SW >= SX, "mid rings");
  static_assert(LDS <= 160 * 1024, "mid rings exceed the LDS");
};

// One 1-KiB LDS-DMA block through a buffer descriptor (a __device__ helper: the builtin's LDS
// address-space cast inside the kernel template's lambda left the template uninstantiable on
// the host side, i.e. no launch stub was emitted)
template <int AUX>
__device__ __forceinline__ void mid_dma1(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, voff, soff, 0, AUX);
}

// s_waitcnt vmcnt(n) for a run-time n (the count is an immediate): a jump over constants;
// n above the largest case waits for less than allowed, i.e. is clamped to a safe (longer) wait
__device__ __forceinline__ void vm_wait_dyn(int n) {
  switch (n) {
    case 0: vm_wait<0>(); break;   case 1: vm_wait<1>(); break;   case 2: vm_wait<2>(); break;
    case 3: vm_wait<3>(); break;   case 4: vm_wait<4>(); break;   case 5: vm_wait<5>(); break;
    case 6: vm_wait<6>(); break;   case 7: vm_wait<7>(); break;   case 8: vm_wait<8>(); break;
    case 9: vm_wait<9>(); break;   case 10: vm_wait<10>(); break; case 11: vm_wait<11>(); break;
    case 12: vm_wait<12>(); break; case 13: vm_wait<13>(); break; case 14: vm_wait<14>(); break;
    case 15: vm_wait<15>(); break; case 16: vm_wait<16>(); break; case 17: vm_wait<17>(); break;
    case 18: vm_wait<18>(); break; case 19: vm_wait<19>(); break; case 20: vm_wait<20>(); break;
    case 21: vm_wait<21>(); break; case 22: vm_wait<22>(); break; case 23: vm_wait<23>(); break;
    default: vm_wait<24>(); break;
  }
}

template <int BM, int BN, int SX, int SW, bool PK = false>
__global__ void __launch_bounds__(kMidThreads)
gemm_mid8_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                 int M, int N, int K, int epi, const bf16* __restrict__ bias,
                 bf16* __restrict__ out, long ldo, float* __restrict__ part, int nsplit,
                 RowScale rsc) {
  using C = MidCfg<BM, BN, SX, SW>;
  constexpr int TI = C::TI, TJ = C::TJ, LX = C::LX, LW = C::LW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const xs = smem;
  char* const wsm = smem + SX * C::XB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int grp = wid >> 2;
  const int wm = wid / C::WGN, wn = wid % C::WGN;
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int t = xcd_remap((int)blockIdx.x, mtiles * ntiles * nsplit);
  const int tm = t % mtiles, tn = (t / mtiles) % ntiles, ksplit = t / (mtiles * ntiles);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = K / kBK;
  const int kt0 = (int)(((long)ktiles * ksplit) / nsplit);
  const int nk = (int)(((long)ktiles * (ksplit + 1)) / nsplit) - kt0;

  // DMA: wave w moves the 1-KiB blocks w, w + 8, ... of an X / W slot (BM / 8, BN / 8 blocks)
  const auto rsa = b8_rsrc(X + (long)m0 * ldx, M - m0, ldx);
  // PK: W in the K-tile-blocked layout [N/256][K/64][256][64] (pack_w256): the tile's BN rows
  // lie in one 256-row block (BN divides 256), a row is 128 B and a K-tile 32 KiB further on
  const long wpitch = PK ? 64 : ldw;
  const auto rsb = PK ? b8_rsrc(W + ((long)(n0 >> 8) * K << 8) + (n0 & 255) * 64, 1, (long)K * 256 - (n0 & 255) * 64)
                      : b8_rsrc(W + (long)n0 * ldw, N - n0, ldw);
  const bool wnt = mtiles == 1 && g_tile_w_nt;
  int vx[LX], vw[LW];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int row = (wid + 8 * i) * 8 + (lane >> 3);
    vx[i] = (int)((row * ldx + (((lane & 7) ^ ((row >> 1) & 7)) * 8)) * 2);
  }
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int row = (wid + 8 * i) * 8 + (lane >> 3);
    vw[i] = (int)((row * wpitch + (((lane & 7) ^ ((row >> 1) & 7)) * 8)) * 2);
  }
  auto dma_x = [&](int k) {
    char* s = xs + (k % SX) * C::XB;
    const int soff = (kt0 + k) * kBK * 2;
#pragma unroll
    for (int i = 0; i < LX; ++i) mid_dma1<0>(rsa, s + (wid + 8 * i) * 1024, vx[i], soff);
  };
  auto dma_w = [&](int k) {
    char* s = wsm + (k % SW) * C::WB;
    const int soff = (kt0 + k) * (PK ? 256 * kBK * 2 : kBK * 2);
    if (wnt) {
#pragma unroll
      for (int i = 0; i < LW; ++i) mid_dma1<2>(rsb, s + (wid + 8 * i) * 1024, vw[i], soff);
    } else {
#pragma unroll
      for (int i = 0; i < LW; ++i) mid_dma1<0>(rsb, s + (wid + 8 * i) * 1024, vw[i], soff);
    }
  };
  // Loads issued (in order X(j + SX - 1), W(j + SW - 1) per iteration j; the prologue is the
  // virtual iterations 1 - SW .. -1) after the later of X(k+1) / W(k+1): what may stay in
  // flight once K-tile k+1 must have landed (k = -1: the prologue's wait for K-tile 0).
  auto after = [&](int k) {
    const int kt = k + 1;
    const int jx = kt - SX + 1, jw = kt - SW + 1;   // iterations that issued X(kt), W(kt)
    int n = 0;
    if (jw == jx) {   // SW == SX: W(kt) is the later one
      // nothing else of iteration jx after it
    } else if (kt + SW - SX < nk) {
      n += LW;        // W(jx + SW - 1) of the same iteration, behind X(kt)
    }
    for (int j = jx + 1; j <= k; ++j) {
      if (j + SX - 1 < nk) n += LX;
      if (j + SW - 1 < nk) n += LW;
    }
    return n;
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue = virtual iterations 1-SW .. -1: W(0 .. SW-2), X(0 .. SX-2) in issue order
#pragma unroll
  for (int v = 1 - SW; v <= -1; ++v) {
    if (v + SX - 1 >= 0 && v + SX - 1 < nk) dma_x(v + SX - 1);
    if (v + SW - 1 < nk) dma_w(v + SW - 1);
  }
  vm_wait_dyn(after(-1));
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();

  const int ar = wm * C::WM + (lane & 15), bc = wn * C::WN + (lane & 15);
  bf16x8 af[TI], bfr[TJ];
  for (int k = 0; k < nk; ++k) {
    const char* As = xs + (k % SX) * C::XB;
    const char* Bs = wsm + (k % SW) * C::WB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // ---- read segment: this k-step's fragments; X(k + SX - 1) / W(k + SW - 1) DMA
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = lds_frag(As, ar + 16 * i, ks * 4 + (lane >> 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = lds_frag(Bs, bc + 16 * j, ks * 4 + (lane >> 4));
      if (ks == 0) {
        if (k + SX - 1 < nk) dma_x(k + SX - 1);
      } else {
        if (k + SW - 1 < nk) dma_w(k + SW - 1);
        if (grp == 1) vm_wait_dyn(after(k));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // ---- MFMA segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);   // C^T tile
      __builtin_amdgcn_s_setprio(0);
      if (ks == 1 && grp == 0) vm_wait_dyn(after(k));
      __builtin_amdgcn_s_barrier();
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // re-align the groups' barrier counts
  tile_epilogue<TI, TJ>(acc, m0 + wm * C::WM, n0 + wn * C::WN, lane, M, N, epi, bias, out, ldo,
                        part ? part + (long)ksplit * M * N + (long)m0 * N : nullptr, m0, rsc);
}

// ---------------------------------------------------------------------------------------
// Host dispatch
// ---------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------
// Mid-M one-wave-per-SIMD GEMM (plan kind 7, "mid4"): big4's structure on 128x128 / 256x128 /
// 128x256 tiles for the TP-shard and large-batch decode projections (M = 128-512), where
// split-K fills the chip and each workgroup walks only 8-30 K-tiles. 4 waves in 2 x 2, each
// owning a (BM/2) x (BN/2) block; per K-tile a wave runs TI x TJ MFMAs per k-step in slots of 4
// (sched_barrier-fenced, fragment reads and LDS-DMA spread over the slots); LDS-DMA rings of SA
// activation and SB weight K-tiles (the whole 160 KiB: up to 5 weight K-tiles of lead for the
// HBM stream); one barrier per K-tile; the loop rotated to end on it (see gemm_big4_kernel).
// The DMA wait count at the barrier follows the fixed issue order
//   prologue A(0), B(0), A(1 .. SA-2), B(1 .. SB-1); iteration t: A(t+SA-1) in k-step 0,
//   B(t+SB) in k-step 1
// and is computed per iteration (scalar), exact in the first iterations as in the steady state.
// ---------------------------------------------------------------------------------------
constexpr int kMid4Threads = 256;

template <int BM, int BN, int SA, int SB>
struct Mid4Cfg {
  static constexpr int WM = BM / 2, WN = BN / 2, TI = WM / 16, TJ = WN / 16;
  static constexpr int NS = TI * TJ / 4;            // MFMA slots per k-step
  static constexpr int NF = TI + TJ;                // fragments per k-step
  static constexpr int NA = BM / 32, NB = BN / 32;  // DMA instructions per thread per K-tile
  static constexpr int ASLOT = BM * 128, BSLOT = BN * 128;
  static constexpr int LDS = SA * ASLOT + SB * BSLOT;
  static_assert(TJ % 4 == 0 && NA % 2 == 0 && NB % 2 == 0, "mid4 tile shape");
  static_assert(SA >= 2 && SB >= 2 && LDS <= 160 * 1024, "mid4 rings");
};

template <int BM, int BN, int SA, int SB, bool PK = false>
__global__ void __launch_bounds__(kMid4Threads) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_mid4_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                 int M, int N, int K, int epi, const bf16* __restrict__ bias,
                 bf16* __restrict__ out, long ldo, float* __restrict__ part, RowScale rsc) {
  using C = Mid4Cfg<BM, BN, SA, SB>;
  constexpr int TI = C::TI, TJ = C::TJ, NS = C::NS, NF = C::NF, NA = C::NA, NB = C::NB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int t = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int per_group = kBigGroupM * ntiles;
  const int grp = t / per_group, first_m = grp * kBigGroupM;
  const int gsize = min(mtiles - first_m, kBigGroupM);
  const int m0 = (first_m + (t % per_group) % gsize) * BM;
  const int n0 = ((t % per_group) / gsize) * BN;
  const int ktiles = K / 64;
  const int kt0 = (int)(((long)ktiles * blockIdx.y) / gridDim.y);
  const int kt1 = (int)(((long)ktiles * (blockIdx.y + 1)) / gridDim.y);
  const int nk = kt1 - kt0;   // >= 1 (host check)

  // DMA: instruction s of wave w fills LDS row block NA w + s (A; NB w + s for B), 8 rows x
  // 128 B lane-linear, lane L supplying row 8 (block) + (L >> 3) at lds_frag's swizzled chunk
  // (L & 7) ^ ((L >> 4) + 4 (s & 1)) & 7 (NA, NB even)
  const auto rsa = b8_rsrc(X + (long)m0 * ldx, M - m0, ldx);   // A rows past M read zeros
  // PK: W in the pack_w256 layout (see gemm_mid8_kernel): 128-B rows, 32-KiB K-tiles
  const long wpitch = PK ? 64 : ldw;
  const int kstep = PK ? 256 * 128 : 128;
  const auto rsb = PK ? b8_rsrc(W + ((long)(n0 >> 8) * K << 8) + (n0 & 255) * 64, 1, (long)K * 256 - (n0 & 255) * 64)
                      : b8_rsrc(W + (long)n0 * ldw, N - n0, ldw);
  int va[2], vb[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int ch = (lane & 7) ^ (((lane >> 4) + 4 * e) & 7);
    va[e] = (int)(((8 * NA * wid + (lane >> 3)) * ldx + ch * 8) * 2);
    vb[e] = (int)(((8 * NB * wid + (lane >> 3)) * wpitch + ch * 8) * 2);
  }
  char* const bbase = smem + SA * C::ASLOT;
  auto dma_a = [&](int k, int slot, int s) {
    b4_dma(rsa, smem + slot * C::ASLOT + (NA * wid + s) * 1024, va[s & 1], (kt0 + k) * 128 + (int)(8 * s * ldx * 2));
  };
  auto dma_b = [&](int k, int slot, int s) {
    b4_dma(rsb, bbase + slot * C::BSLOT + (NB * wid + s) * 1024, vb[s & 1], (kt0 + k) * kstep + (int)(8 * s * wpitch * 2));
  };
  const int fr = lane & 15, fq = lane >> 4;
  int lo[2][2];   // [A / B][ks] lane byte offset inside a slot (fragments differ by 2048 B)
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int ch = ((ks * 4 + fq) ^ ((fr >> 1) & 7)) * 16;
    lo[0][ks] = (wr * C::WM + fr) * 128 + ch;
    lo[1][ks] = (wc * C::WN + fr) * 128 + ch;
  }
  // fragment idx 0 .. TJ-1: B (output columns 16 idx), TJ .. NF-1: A (rows 16 (idx - TJ))
  auto rd1 = [&](int sa_, int sb_, int ks, int idx, bf16x8 (&f)[NF]) {
    const char* p = idx < TJ ? bbase + sb_ * C::BSLOT + lo[1][ks] + 2048 * idx
                             : smem + sa_ * C::ASLOT + lo[0][ks] + 2048 * (idx - TJ);
    f[idx] = *reinterpret_cast<const bf16x8*>(p);
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mf4 = [&](int n, const bf16x8 (&f)[NF]) {   // slot n: row block i, 4 column blocks
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = n / (TJ / 4), j = 4 * (n % (TJ / 4)) + q;
      acc[i][j] = mfma16(f[j], f[TJ + i], acc[i][j]);
    }
  };
  bf16x8 f0[NF], f1[NF];

  // issue-order bookkeeping (per-thread load counts, see the header)
  constexpr int P = (SA - 1) * NA + SB * NB;
  auto idx_a = [&](int j) {
    return j == 0 ? NA : j <= SA - 2 ? NA + NB + j * NA : P + (j - SA + 1) * (NA + NB) + NA;
  };
  auto idx_b = [&](int j) {
    return j == 0 ? NA + NB : j <= SB - 1 ? NA + NB + (SA - 2) * NA + j * NB : P + (j - SB) * (NA + NB) + NA + NB;
  };
#pragma unroll
  for (int s = 0; s < NA; ++s) dma_a(0, 0, s);
#pragma unroll
  for (int s = 0; s < NB; ++s) dma_b(0, 0, s);
#pragma unroll
  for (int j = 1; j <= SA - 2; ++j)
#pragma unroll
    for (int s = 0; s < NA; ++s) dma_a(min(j, nk - 1), j, s);
#pragma unroll
  for (int j = 1; j <= SB - 1; ++j)
#pragma unroll
    for (int s = 0; s < NB; ++s) dma_b(min(j, nk - 1), j, s);
  vm_wait<P - NA - NB>();            // K-tile 0 landed (own part)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int idx = 0; idx < NF; ++idx) rd1(0, 0, 0, idx, f0);

  auto ks0 = [&](int k, int sa_, int sb_) {   // k-step 0 of K-tile k; DMA A(k+SA-1); barrier
    const int ka = min(k + SA - 1, nk - 1), slot = sa_ == 0 ? SA - 1 : sa_ - 1;
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      mf4(n, f0);
#pragma unroll
      for (int q = n * NA / NS; q < (n + 1) * NA / NS; ++q) dma_a(ka, slot, q);
#pragma unroll
      for (int idx = n * NF / NS; idx < (n + 1) * NF / NS; ++idx) rd1(sa_, sb_, 1, idx, f1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // A(k+1), B(k+1) landed (own part): the loads issued after the later of them may fly
    const int total = P + k * (NA + NB) + NA;
    vm_wait_dyn(total - max(idx_a(k + 1), idx_b(k + 1)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  auto ks1 = [&](int k, int sa_, int sb_, int sa1_, int sb1_) {   // k-step 1; DMA B(k+SB)
    const int kb = min(k + SB, nk - 1);
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      mf4(n, f1);
#pragma unroll
      for (int idx = n * NF / NS; idx < (n + 1) * NF / NS; ++idx) rd1(sa1_, sb1_, 0, idx, f0);
#pragma unroll
      for (int q = n * NB / NS; q < (n + 1) * NB / NS; ++q) dma_b(kb, sb_, q);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int sa = 0, sb = 0;
  ks0(0, 0, 0);
  for (int k = 0; k + 1 < nk; ++k) {
    const int sa1 = sa == SA - 1 ? 0 : sa + 1, sb1 = sb == SB - 1 ? 0 : sb + 1;
    ks1(k, sa, sb, sa1, sb1);
    ks0(k + 1, sa1, sb1);
    sa = sa1;
    sb = sb1;
  }
  ks1(nk - 1, sa, sb, sa == SA - 1 ? 0 : sa + 1, sb == SB - 1 ? 0 : sb + 1);
  vm_wait<0>();                       // no LDS-DMA may outlive the workgroup
  tile_epilogue<TI, TJ>(acc, m0 + wr * C::WM, n0 + wc * C::WN, lane, M, N, epi, bias, out, ldo,
                        part ? part + (long)blockIdx.y * M * N + (long)m0 * N : nullptr, m0, rsc);
}

static int num_cus() { return 256; }

// Workspace layout: [kCounterBytes reserved head | SK x M x N f32 partials].
static float* splitk_part(float* ws) { return ws + kCounterBytes / sizeof(float); }



template <int MT, int NT, int WK>
static void run_skinny(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                       int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk,
                       hipStream_t stream) {
  dim3 grid(N / (16 * NT * (4 / WK)), sk);
  gemm_skinny_kernel<MT, NT, WK><<<grid, kSkThreads, 0, stream>>>(
      X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, sk > 1 ? splitk_part(ws) : nullptr);
}

static void init_nt_policy() {
  static bool done = false;
  if (done) return;
  done = true;
  const int zero = 0;
  const char* e = getenv("BFLY_GEMM_NT_WEIGHTS");
  if (e && e[0] == '0') (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tile_w_nt), &zero, sizeof(int));
}

template <int BM, int BN, int WMW, int STAGES, bool PACKW = false>
static void run_tile(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                     int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk,
                     hipStream_t stream, const RowScale& rsc) {
  init_nt_policy();
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const size_t lds = (size_t)STAGES * (BM + BN) * kBK * 2;
  const dim3 grid(tiles, sk);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once per kernel
  if (!attr_set && lds > 65536) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tile_kernel<BM, BN, WMW, STAGES, false, PACKW>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  gemm_tile_kernel<BM, BN, WMW, STAGES, false, PACKW><<<grid, kTileThreads, lds, stream>>>(
      X, ldx, W, PACKW ? (long)K : ldw, M, N, K, epi, bias, out, ldo, sk > 1 ? splitk_part(ws) : nullptr,
      nullptr, nullptr, nullptr, 0, rsc);
}

template <int BM, int BN, int NWM, int NWN, int SW>
static void run_dec(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                    int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk,
                    hipStream_t stream, const RowScale& rsc) {
  init_nt_policy();
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  constexpr size_t lds = (size_t)(3 * BM + SW * BN) * kBK * 2;
  static_assert(lds <= 160 * 1024, "decode GEMM rings exceed the 160 KiB LDS");
  static bool attr_set = false;
  if (!attr_set && lds > 65536) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_dec_kernel<BM, BN, NWM, NWN, SW>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const dim3 grid(tiles, sk);
  gemm_dec_kernel<BM, BN, NWM, NWN, SW><<<grid, NWM * NWN * 64, lds, stream>>>(
      X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, sk > 1 ? splitk_part(ws) : nullptr, rsc);
}

static void run_big8(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                     int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big8_kernel<false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kB8LdsBytes);
    attr = true;
  }
  const int tiles = ((M + 255) / 256) * (N / 256);
  dim3 grid(tiles, sk);
  float* part = sk > 1 ? splitk_part(ws) : nullptr;
  gemm_big8_kernel<false><<<grid, kB8Threads, kB8LdsBytes, stream>>>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, part);
}

static void run_big4(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                     int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big4_kernel<false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kB4LdsBytes);
    attr_set = true;
  }
  dim3 grid(((M + 255) / 256) * (N / 256), sk);
  float* part = sk > 1 ? splitk_part(ws) : nullptr;
  gemm_big4_kernel<false><<<grid, kB4Threads, kB4LdsBytes, stream>>>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, part);
}

template <int BM, int BN, int SA, int SB, bool PK = false>
static void run_mid4(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K, int epi,
                     const bf16* bias, bf16* out, long ldo, float* ws, int sk, hipStream_t stream,
                     const RowScale& rsc) {
  using C = Mid4Cfg<BM, BN, SA, SB>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mid4_kernel<BM, BN, SA, SB, PK>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr_set = true;
  }
  dim3 grid(((M + BM - 1) / BM) * (N / BN), sk);
  float* part = sk > 1 ? splitk_part(ws) : nullptr;
  gemm_mid4_kernel<BM, BN, SA, SB, PK><<<grid, kMid4Threads, C::LDS, stream>>>(X, ldx, W, ldw, M, N, K, epi, bias,
                                                                         out, ldo, part, rsc);
}

template <int BM, int BN, int SX, int SW, bool PK = false>
static void run_mid8(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K, int epi,
                     const bf16* bias, bf16* out, long ldo, float* ws, int sk, hipStream_t stream,
                     const RowScale& rsc) {
  init_nt_policy();
  constexpr size_t lds = (size_t)MidCfg<BM, BN, SX, SW>::LDS;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mid8_kernel<BM, BN, SX, SW, PK>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  gemm_mid8_kernel<BM, BN, SX, SW, PK><<<tiles * sk, kMidThreads, lds, stream>>>(
      X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, sk > 1 ? splitk_part(ws) : nullptr, sk, rsc);
}

// Plan selection, from the tools/bench_gemm.py sweep on MI355X (Llama-3-70B TP1/TP8 shapes,
// weights streamed from HBM): the LDS-tiled kernel with a small BM and split-K beats the
// register-streaming skinny kernel for every M >= 8 (e.g. down-proj M=64: 90 us = 5.2 TB/s vs
// 186 us) and ties or beats hipBLASLt; the skinny kernel stays for M <= 4 (GEMV regime).
// Split-K is sized so the grid has ~448 workgroups (1.75 per CU) with >= 4 K-tiles each.
// Measured plan table (tools/gen_gemm_table.py from the profiles/gemm_tune_*.json sweeps of
// tools/bench_gemm.py --sweep on MI355X): the fastest plan per model projection shape and
// token-count bucket (entries exist only where the sweep beat the heuristic by > 3%).
struct TunedPlan { int N, K, M, kind, mt, nt, wk, bm, bn, sk; };
static const TunedPlan kTuned[] = {
#include "gemm_tuned.inc"
};

static GemmPlan plan_gemm_heuristic(int M, int N, int K);

static bool tuned_enabled() {   // BFLY_GEMM_TUNED=0: heuristic plans only (A/B runs)
  static const bool on = [] {
    const char* e = getenv("BFLY_GEMM_TUNED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// BFLY_GEMM_PLAN="N,K,Mbucket:kind,mt,nt,wk,bm,bn,sk;..." forces plans for whole-model A/B runs
// (a shape's plan measured inside the decode step, where the neighbouring kernels and the
// cache state differ from an isolated sweep). Parsed once.
struct PlanOverride { int N, K, M; GemmPlan p; };
static const std::vector<PlanOverride>& plan_overrides() {
  static const std::vector<PlanOverride> v = [] {
    std::vector<PlanOverride> out;
    const char* e = getenv("BFLY_GEMM_PLAN");
    if (!e) return out;
    std::string s(e);
    size_t pos = 0;
    while (pos < s.size()) {
      size_t end = s.find(';', pos);
      if (end == std::string::npos) end = s.size();
      PlanOverride o{};
      if (sscanf(s.substr(pos, end - pos).c_str(), "%d,%d,%d:%d,%d,%d,%d,%d,%d,%d", &o.N, &o.K, &o.M, &o.p.kind,
                 &o.p.mt, &o.p.nt, &o.p.wk, &o.p.bm, &o.p.bn, &o.p.sk) == 10)
        out.push_back(o);
      pos = end + 1;
    }
    return out;
  }();
  return v;
}

GemmPlan plan_gemm(int M, int N, int K) {
  if (!plan_overrides().empty()) {
    static const int kB[] = {1, 16, 32, 64, 128, 256, 512};
    int bucket = 0;
    for (int b : kB)
      if (b >= M) { bucket = b; break; }
    for (const PlanOverride& o : plan_overrides())
      if (o.N == N && o.K == K && o.M == bucket) return o.p;
  }
  if (!tuned_enabled()) return plan_gemm_heuristic(M, N, K);
  // token-count buckets of the sweep: M uses the entry of its bucket, or the heuristic plan
  // when the sweep found nothing better there
  static const int kBuckets[] = {1, 16, 32, 64, 128, 256, 512};
  int bucket = 0;
  for (int b : kBuckets)
    if (b >= M) { bucket = b; break; }
  if (bucket == 0) return plan_gemm_heuristic(M, N, K);
  for (const TunedPlan& t : kTuned)
    if (t.N == N && t.K == K && t.M == bucket)   // 256x256 entries (swept on big8) run big4:
      return t.kind == 4 ? GemmPlan{6, 0, 0, 0, 256, 256, t.sk}   // >= big8 at every swept M / sk
                         : GemmPlan{t.kind, t.mt, t.nt, t.wk, t.bm, t.bn, t.sk};
  return plan_gemm_heuristic(M, N, K);
}

static GemmPlan plan_gemm_heuristic(int M, int N, int K) {
  GemmPlan p{};
  const int target = 448;
  const bool skinny_ok = K % 128 == 0 && N % 128 == 0;
  // register-streaming kernel: GEMV-like M, and short-K shapes (row-parallel projections
  // after TP splits K) where the LDS pipeline cannot fill before the K loop ends
  if (skinny_ok && (M <= 4 || (M <= 64 && K <= 1024))) {
    p.kind = 0;
    p.mt = (M + 15) / 16;
    const bool long_k = K > 4096;
    p.nt = M <= 4 ? (long_k ? 4 : 2) : 2;   // even: the SiLU epilogue pairs gate/up groups
    p.wk = long_k ? 2 : 4;
    const int blocks = N / (16 * p.nt * (4 / p.wk));
    int sk = 1;
    const int nchunks = K / 128;
    while (long_k && blocks * sk < target && sk * 2 * p.wk <= nchunks && sk < 16) sk *= 2;
    p.sk = sk;
    return p;
  }
  if (M > 256 && N % 256 == 0 && K % 64 == 0) {
    // prefill / large batch: the 256x256 one-wave-per-SIMD tile (gemm_big4_kernel: 1.52-1.55
    // PF at M = 8192 on the 70B projections, 6-10 % over the 8-phase gemm_big8_kernel and ahead
    // of it at M = 256-2048 too, profiles/r5_gemm_big4/); split K only when the tile grid cannot
    // fill the 256 CUs
    p.kind = 6;
    p.mt = 0;
    p.bm = p.bn = 256;
    const int tiles = ((M + 255) / 256) * (N / 256);
    int sk = 1;
    while (tiles * sk < 256 && K / 64 >= sk * 2 * 8 && sk < 8) sk *= 2;
    p.sk = sk;
    return p;
  }
  p.kind = 1;
  p.mt = M >= 512 ? 2 : 3;   // tile plans: `mt` = pipeline depth (K-tiles in flight + 1)
  if (M <= 16) { p.bm = 16; p.wk = 1; }
  else if (M <= 32) { p.bm = 32; p.wk = 1; }
  else if (M <= 64) { p.bm = 64; p.wk = 2; }
  else { p.bm = 128; p.wk = 2; }
  p.bn = 128;
  const int tiles = ((M + p.bm - 1) / p.bm) * (N / p.bn);
  int sk = 1;
  const int ktiles = K / kBK;
  while (tiles * sk < target && sk * 2 * 4 <= ktiles && sk < 16) sk *= 2;
  p.sk = sk;
  return p;
}

static size_t plan_ws_bytes(const GemmPlan& p, int M, int N) {
  return p.sk > 1 ? kCounterBytes + (size_t)p.sk * M * N * sizeof(float) : 0;
}

// Enough for the tuned plan and for the heuristic plan it may fall back to (below).
size_t gemm_workspace_bytes(int M, int N, int K) {
  const size_t a = plan_ws_bytes(plan_gemm(M, N, K), M, N);
  const size_t b = plan_ws_bytes(plan_gemm_heuristic(M, N, K), M, N);
  return a > b ? a : b;
}

// `dry`: validate only (the plan is supported for this shape/epilogue) without launching.
static int run_plan(const GemmPlan& p, const bf16* X, long ldx, const bf16* W, long ldw, int M,
                    int N, int K, int epi, const bf16* bias, bf16* out, long ldo, float* ws,
                    hipStream_t stream, bool dry = false, bool defer = false,
                    const RowScale* rs = nullptr, bool packed = false) {
  const RowScale rsc = rs ? *rs : RowScale{nullptr, 0, 0.f, 0.f};
  if (rs != nullptr && p.kind != 1 && p.kind != 3 && p.kind != 5 && p.kind != 7) return -4;   // row scale: tile / ring / mid epilogues
  if (epi == EPI_SILU_GATE && (p.kind != 1 || p.sk != 1)) return -4;   // gate: tile epilogue, no slabs
  // packed (pack_w256) weights: the tile plans mark it with nt = 1, the mid-M kernels take it here
  if (packed && p.kind != 5 && p.kind != 7) return -5;
  if (p.kind == 4) {
    // 8-phase big tile: every split needs >= 2 K-tiles of 64
    if (N % 256 != 0 || K % 64 != 0 || K / 64 < 2 * p.sk) return -1;
    if (!dry) run_big8(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream);
  } else if (p.kind == 7) {
    // mid-M one-wave-per-SIMD tile: plan {7, SA (activation ring), SB (weight ring), 0, BM, BN, sk}
    if (N % p.bn != 0 || K % 64 != 0 || K / 64 < p.sk) return -1;
    bool done = false;
#define MID4_CASE(BM_, BN_, SA_, SB_)                                                               \
  if (!done && p.bm == BM_ && p.bn == BN_ && p.mt == SA_ && p.nt == SB_) {                          \
    if (!dry && packed) run_mid4<BM_, BN_, SA_, SB_, true>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    else if (!dry) run_mid4<BM_, BN_, SA_, SB_>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    done = true;                                                                                   \
  }
    MID4_CASE(128, 128, 4, 6) MID4_CASE(128, 128, 3, 7) MID4_CASE(128, 128, 2, 8)
    MID4_CASE(256, 128, 3, 4) MID4_CASE(256, 128, 2, 6) MID4_CASE(128, 256, 4, 3) MID4_CASE(128, 256, 2, 4)
#undef MID4_CASE
    if (!done) return -2;
  } else if (p.kind == 6) {
    // one-wave-per-SIMD 256x256 tile: every split needs >= 2 K-tiles of 64
    if (N % 256 != 0 || K % 64 != 0 || K / 64 < 2 * p.sk) return -1;
    if (!dry) run_big4(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream);

  } else if (p.kind == 5) {
    // mid-M 8-wave staggered GEMM: plan {5, SW (weight ring), SX (activation ring; 0 = SW), 0,
    // BM, BN, sk}
    if (N % p.bn != 0 || K % kBK != 0 || K / kBK < p.sk) return -1;
    if (epi == EPI_SILU && p.bn * p.bm / 512 % 32 != 0) return -1;
    const int sx = p.nt > 0 ? p.nt : p.mt;
    bool done = false;
#define MID_CASE(BM_, BN_, SX_, SW_)                                                              \
  if (!done && p.bm == BM_ && p.bn == BN_ && sx == SX_ && p.mt == SW_) {                           \
    if (!dry && packed) run_mid8<BM_, BN_, SX_, SW_, true>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    else if (!dry) run_mid8<BM_, BN_, SX_, SW_>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    done = true;                                                                                   \
  }
    MID_CASE(256, 128, 3, 3) MID_CASE(256, 128, 2, 6) MID_CASE(256, 128, 3, 4)
    MID_CASE(128, 256, 3, 3) MID_CASE(128, 256, 2, 4)
    MID_CASE(128, 128, 4, 4) MID_CASE(128, 128, 3, 3) MID_CASE(128, 128, 3, 6) MID_CASE(128, 128, 2, 8)
    MID_CASE(128, 128, 2, 2)   // 64 KiB: two workgroups per CU
#undef MID_CASE
    if (!done) return -2;
  } else if (p.kind == 3) {
    // decode ring GEMM: plan {3, SW (weight ring depth), waves, waves along M, BM, BN, sk}
    if (N % p.bn != 0 || K % kBK != 0 || K / kBK < p.sk * 2) return -1;
    const int nwn = p.wk > 0 ? p.nt / p.wk : 0;
    if (epi == EPI_SILU && (nwn <= 0 || (p.bn / nwn) % 32 != 0)) return -1;
    bool done = false;
#define DEC_CASE(BM_, BN_, NWM_, NWN_, SW_)                                                      \
  if (!done && p.bm == BM_ && p.bn == BN_ && p.wk == NWM_ && p.nt == NWM_ * NWN_ && p.mt == SW_) { \
    if (!dry) run_dec<BM_, BN_, NWM_, NWN_, SW_>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    done = true;                                                                                 \
  }
    DEC_CASE(128, 224, 8, 1, 4) DEC_CASE(128, 224, 8, 1, 3) DEC_CASE(128, 256, 8, 1, 3)
    DEC_CASE(128, 256, 4, 2, 3) DEC_CASE(128, 128, 8, 1, 5) DEC_CASE(128, 128, 4, 2, 5)
    DEC_CASE(128, 160, 8, 1, 4) DEC_CASE(128, 80, 8, 1, 6) DEC_CASE(128, 64, 8, 1, 8)
    DEC_CASE(128, 64, 4, 2, 8) DEC_CASE(64, 128, 4, 2, 6) DEC_CASE(64, 256, 4, 2, 4)
    DEC_CASE(64, 224, 4, 1, 4) DEC_CASE(64, 160, 4, 2, 5) DEC_CASE(64, 64, 4, 2, 8)
#undef DEC_CASE
    if (!done) return -2;
  } else if (p.kind == 0) {
    if (K % 128 != 0 || M > 16 * p.mt) return -1;
    if (N % (16 * p.nt * (4 / p.wk)) != 0) return -1;
    if (epi == EPI_SILU && p.nt % 2 != 0) return -1;
    if (p.sk > 1 && N / (16 * p.nt * (4 / p.wk)) > kSplitCounters) return -1;
    bool done = false;
#define SK_CASE(MT_, NT_, WK_)                                                                   \
  if (!done && p.mt == MT_ && p.nt == NT_ && p.wk == WK_) {                                       \
    if (!dry) run_skinny<MT_, NT_, WK_>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream); \
    done = true;                                                                                  \
  }
#define SK_WK(MT_, NT_) SK_CASE(MT_, NT_, 1) SK_CASE(MT_, NT_, 2) SK_CASE(MT_, NT_, 4)
    SK_WK(1, 1) SK_WK(1, 2) SK_WK(1, 4) SK_WK(2, 1) SK_WK(2, 2) SK_WK(2, 4)
    SK_WK(3, 2) SK_WK(4, 1) SK_WK(4, 2) SK_WK(4, 4)
#undef SK_WK
#undef SK_CASE
    if (!done) return -2;
  } else if (p.kind == 1 && p.nt == 1) {
    // tile plan over a K-tile-blocked weight (pack_w256 layout): 16 / 32 / 64-row tiles of 128 /
    // 256 columns (the packed layout only changes the weight stage's addresses, so every decode
    // tile the row-major table picks, down to the B = 1 bucket, has its packed twin)
    if (N % 256 != 0 || K % 64 != 0 || (p.bm != 16 && p.bm != 32 && p.bm != 64) || (p.bn != 128 && p.bn != 256) ||
        K / kBK < p.sk)
      return -1;
    if (p.sk > 1 && (long)((M + p.bm - 1) / p.bm) * (N / p.bn) > kSplitCounters) return -1;
    bool done = false;
    const int st = p.mt > 0 ? p.mt : 2;
#define TLP_CASE(BM_, BN_, WMW_, ST_)                                                                 \
  if (!done && p.bm == BM_ && p.bn == BN_ && p.wk == WMW_ && st == ST_) {                             \
    if (!dry) run_tile<BM_, BN_, WMW_, ST_, true>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    done = true;                                                                                      \
  }
#define TLP_ST(BM_, BN_, WMW_) TLP_CASE(BM_, BN_, WMW_, 2) TLP_CASE(BM_, BN_, WMW_, 3) TLP_CASE(BM_, BN_, WMW_, 4)
    TLP_ST(16, 128, 1) TLP_ST(16, 256, 1) TLP_ST(32, 128, 1) TLP_ST(32, 256, 1)
    TLP_ST(64, 128, 1) TLP_ST(64, 128, 2) TLP_ST(64, 256, 1) TLP_ST(64, 256, 2)
#undef TLP_ST
#undef TLP_CASE
    if (!done) return -2;
  } else {
    if (N % p.bn != 0 || K % kBK != 0) return -1;
    if (p.sk > 1 && (long)((M + p.bm - 1) / p.bm) * (N / p.bn) > kSplitCounters) return -1;
    bool done = false;
    const int st = p.mt > 0 ? p.mt : 2;   // tile plans reuse `mt` as the pipeline depth
#define TL_CASE(BM_, BN_, WMW_, ST_)                                                            \
  if (!done && p.bm == BM_ && p.bn == BN_ && p.wk == WMW_ && st == ST_) {                       \
    if (!dry) run_tile<BM_, BN_, WMW_, ST_>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream, rsc); \
    done = true;                                                                                \
  }
#define TL_ST(BM_, BN_, WMW_) TL_CASE(BM_, BN_, WMW_, 2) TL_CASE(BM_, BN_, WMW_, 3) TL_CASE(BM_, BN_, WMW_, 4)
    TL_ST(16, 128, 1) TL_ST(16, 256, 1) TL_ST(32, 128, 1) TL_ST(32, 256, 1)
    TL_ST(64, 128, 1) TL_ST(64, 128, 2) TL_ST(64, 256, 1) TL_ST(64, 256, 2)
    TL_ST(128, 128, 2) TL_ST(128, 256, 2)
    // CU-balanced decode tiles: N/224 or N/160 tiles x split-K land on exactly 256 workgroups
    // for the Llama-3-70B projections (gate/up 57344 = 256 x 224, QKV 10240 = 64 x 160)
    TL_ST(64, 224, 4) TL_ST(64, 160, 4)
#undef TL_ST
#undef TL_CASE
    if (!done) return -2;
  }
  if (p.sk > 1 && !dry && !defer) {
    const int nout = epi == EPI_SILU ? N / 2 : N;
    long total = (long)M * nout;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    gemm_splitk_reduce_kernel<<<grid, 256, 0, stream>>>(splitk_part(ws), p.sk, M, N, epi, bias,
                                                         out, ldo);
  }
  return 0;
}

int launch_gemm_plan(const GemmPlan& p, const bf16* X, long ldx, const bf16* W, long ldw, int M,
                     int N, int K, int epi, const bf16* bias, bf16* out, long ldo, float* ws,
                     size_t ws_bytes, hipStream_t stream) {
  if (M <= 0) return 0;
  if (p.sk > 1 && (ws == nullptr || ws_bytes < kCounterBytes + (size_t)p.sk * M * N * sizeof(float)))
    return -3;
  return run_plan(p, X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, stream);
}

// The plan for this call: the tuned/heuristic plan, or the heuristic one when a table entry
// measured for another epilogue cannot run this one (e.g. odd skinny NT with SiLU).
static GemmPlan select_plan(int M, int N, int K, int epi) {
  GemmPlan p = plan_gemm(M, N, K);
  if (run_plan(p, nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr, 0, nullptr, nullptr, true) != 0)
    p = plan_gemm_heuristic(M, N, K);
  return p;
}

int gemm_rowscale_check(int M, int N, int K, int epi) {
  if (M <= 0) return 0;
  const RowScale probe{nullptr, 0, 0.f, 0.f};
  return run_plan(select_plan(M, N, K, epi), nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr, 0,
                  nullptr, nullptr, true, false, &probe);
}

// Grouped expert GEMM (MoE): BM x 128 tile (BM = 64 or 128 rows per expert tile, chosen by
// the caller from the expected rows per expert), 3-stage pipeline; grid = (max tiles, sk,
// N / 128) with the device tile list deciding which workgroups run. sk > 1 splits K and
// writes f32 slabs part[sk][slots][N] (consumed by moe_combine_slabs: the split-K reduce is
// fused into the weighted combine) — decode-sized expert batches otherwise leave most CUs
// idle on the down projection (N = hidden: 32 column tiles per expert tile).
template <int BM>
static int launch_grouped_bm(const bf16* X, long ldx, const bf16* W, long ldw, long w_estride, int N,
                             int K, int epi, const int* rows, const int4* tiles, const int* count,
                             int max_tiles, int slots, int sk, float* part, bf16* out, long ldo,
                             hipStream_t stream) {
  constexpr int BN = 128, WMW = 2, ST = 3;
  const size_t lds = (size_t)ST * (BM + BN) * kBK * 2;
  static bool attr_set = false;
  if (!attr_set && lds > 65536) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tile_kernel<BM, BN, WMW, ST, true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  dim3 grid(max_tiles, sk, N / BN);
  gemm_tile_kernel<BM, BN, WMW, ST, true><<<grid, kTileThreads, lds, stream>>>(
      X, ldx, W, ldw, slots, N, K, epi, nullptr, out, ldo, sk > 1 ? part : nullptr, rows,
      tiles, count, w_estride);
  return 0;
}

int launch_gemm_grouped(const bf16* X, long ldx, const bf16* W, long ldw, long w_estride, int N,
                        int K, int epi, const int* rows, const int4* tiles, const int* count,
                        int max_tiles, bf16* out, long ldo, hipStream_t stream, int bm, int slots,
                        int sk, float* part) {
  if (N % 128 != 0 || K % kBK != 0 || max_tiles <= 0) return -1;
  if (epi != EPI_NONE && epi != EPI_SILU) return -1;
  if (sk < 1 || sk > K / kBK || (sk > 1 && (part == nullptr || epi != EPI_NONE || slots <= 0))) return -2;
  if (bm == 256) {
    // prefill-scale expert batches: a 256x256 tile over the tile list, no split
    if (N % 256 != 0 || K / 64 < 2 || sk != 1) return -2;
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big8_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kB8LdsBytes);
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big4_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kB4LdsBytes);
      attr = true;
    }
    dim3 grid(max_tiles * (N / 256), 1);
    // the SwiGLU gate/up GEMM on big4, the down projection on big8: Mixtral 8x7B at 32k routed
    // rows, gate/up 6.02-6.04 vs 6.35-6.40 ms, down 3.64-3.66 vs 3.19-3.20 ms
    // (profiles/r5_gemm_big4/grouped_moe_per_gemm.log)
    if (epi == EPI_SILU)
      gemm_big4_kernel<true><<<grid, kB4Threads, kB4LdsBytes, stream>>>(
          X, ldx, W, ldw, max_tiles * 256, N, K, epi, nullptr, out, ldo, nullptr, rows, tiles, count, w_estride);
    else
      gemm_big8_kernel<true><<<grid, kB8Threads, kB8LdsBytes, stream>>>(
          X, ldx, W, ldw, max_tiles * 256, N, K, epi, nullptr, out, ldo, nullptr, rows, tiles, count, w_estride);
    return 0;
  }
  if (bm == 128)
    return launch_grouped_bm<128>(X, ldx, W, ldw, w_estride, N, K, epi, rows, tiles, count, max_tiles,
                                  slots, sk, part, out, ldo, stream);
  if (bm == 64)
    return launch_grouped_bm<64>(X, ldx, W, ldw, w_estride, N, K, epi, rows, tiles, count, max_tiles,
                                 slots, sk, part, out, ldo, stream);
  return -3;
}

int gemm_check(int M, int N, int K, int epi) {
  if (M <= 0) return 0;
  return run_plan(select_plan(M, N, K, epi), nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr,
                  0, nullptr, nullptr, true);
}

int launch_gemm_deferred(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                         bf16* out, long ldo, float* ws, size_t ws_bytes, hipStream_t stream,
                         const RowScale* rs) {
  if (M <= 0) return 1;
  GemmPlan p = select_plan(M, N, K, EPI_NONE);
  if (p.sk > 1 && (ws == nullptr || ws_bytes < kCounterBytes + (size_t)p.sk * M * N * sizeof(float)))
    p.sk = 1;
  const bool defer = p.sk > 1;
  const int rc = run_plan(p, X, ldx, W, ldw, M, N, K, EPI_NONE, nullptr, out, ldo, ws, stream,
                          false, defer, rs);
  if (rc != 0) return rc;
  return defer ? p.sk : 1;
}

size_t gemm_slab_offset_floats() { return kCounterBytes / sizeof(float); }

void launch_splitk_reduce(const float* part, int sk, int M, int N, bf16* out, long ldo,
                          hipStream_t stream) {
  long total = (long)M * N;
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  gemm_splitk_reduce_kernel<<<grid, 256, 0, stream>>>(part, sk, M, N, EPI_NONE, nullptr, out, ldo);
}

int launch_gemm(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K, int epi,
                const bf16* bias, bf16* out, long ldo, float* ws, size_t ws_bytes,
                hipStream_t stream, const RowScale* rs) {
  if (M <= 0) return 0;
  GemmPlan p = select_plan(M, N, K, epi);
  if (p.sk > 1 && (ws == nullptr || ws_bytes < kCounterBytes + (size_t)p.sk * M * N * sizeof(float)))
    p.sk = 1;
  return run_plan(p, X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, stream, false, false, rs);
}

// Decode GEMM over a K-tile-blocked copy of the weight (layout [N/256][K/64][256][64], made
// once by the engine when HBM allows, models/transformer.pack_decode_weights): the plan the
// row-major weight would run (16 / 32 / 64-row tiles and the mid-M kernels of kinds 5 / 7, with
// their split-K; EPI_SILU_GATE: the gate plan) on the packed copy. Each 128-row weight stage is then one 16 KiB run of memory instead of 128
// runs of 128 B a row pitch apart: the Llama-3-70B gate/up GEMM at M = 64 in 145 against
// 158 us, bitwise the same result (tools/packed_probe.py). Returns < 0 (nothing launched)
// when the plan for this shape is not such a tile plan: the caller then uses the row-major
// weight. `dry`: only report whether it applies.
// Packed-weight plans that differ from the row-major table's (tools/packed_probe.py --sweep,
// isolated, weights rotating through HBM; profiles/r6_packed/sweep_m64.jsonl): kind -1 = keep
// this shape on the row-major weight (its row-major plan is faster than any packed one).
struct PackedTuned { int N, K, M; GemmPlan p; };
static const PackedTuned kPackedTuned[] = {
    {8192, 8192, 64, {1, 3, 1, 2, 64, 128, 4}},   // 70B O: 29.3 us vs 32.7 (row-major table plan, split-K 8)
    {4096, 4096, 1, {-1, 0, 0, 0, 0, 0, 0}},      // 8B O: row-major 13.7 us vs 14.2 packed at M = 64;
    {4096, 4096, 16, {-1, 0, 0, 0, 0, 0, 0}},     // packing O / down measured 1-2 % slower per step
    {4096, 4096, 32, {-1, 0, 0, 0, 0, 0, 0}},     // at B = 1 (kinds_b1_ab.log)
    {4096, 4096, 64, {-1, 0, 0, 0, 0, 0, 0}},
};

int launch_gemm_packed(const bf16* X, long ldx, const bf16* Wp, int M, int N, int K, int epi, bf16* out,
                       long ldo, hipStream_t stream, const RowScale* rs, bool dry, float* ws, size_t ws_bytes,
                       bool defer) {
  if (M <= 0) return dry ? 0 : 1;
  if (N % 256 != 0 || K % 64 != 0) return -1;
  GemmPlan p = plan_gemm(M, N, K);
  if (tuned_enabled() && plan_overrides().empty() && epi != EPI_SILU_GATE) {
    static const int kB[] = {1, 16, 32, 64, 128, 256, 512};
    int bucket = 0;
    for (int b : kB)
      if (b >= M) { bucket = b; break; }
    for (const PackedTuned& t : kPackedTuned)
      if (t.N == N && t.K == K && t.M == bucket) {
        if (t.p.kind < 0) return -2;
        if (run_plan(t.p, nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr, 0, nullptr, nullptr, true) == 0)
          p = t.p;
        break;
      }
  }
  if (epi != EPI_SILU_GATE &&
      run_plan(p, nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr, 0, nullptr, nullptr, true) != 0)
    p = plan_gemm_heuristic(M, N, K);
  if (epi == EPI_SILU_GATE &&
      run_plan(p, nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr, 0, nullptr, nullptr, true) != 0) {
    const int bm = M <= 16 ? 16 : M <= 32 ? 32 : M <= 64 ? 64 : 128;
    p = GemmPlan{1, 3, 0, bm <= 32 ? 1 : 2, bm, 128, 1};
  }
  // mid-M kernels (kinds 5 / 7): their weight DMA takes the packed layout as a template flag
  const bool mid = (p.kind == 5 || p.kind == 7) && (p.bn == 128 || p.bn == 256);
  if (!mid && (p.kind != 1 || (p.bm != 16 && p.bm != 32 && p.bm != 64) || (p.bn != 128 && p.bn != 256))) return -2;
  if (!dry && p.sk > 1 && (ws == nullptr || ws_bytes < kCounterBytes + (size_t)p.sk * M * N * sizeof(float)))
    return -3;
  if (!mid) p.nt = 1;
  if (dry)
    return run_plan(p, nullptr, 0, nullptr, 0, M, N, K, epi, nullptr, nullptr, 0, nullptr, nullptr, true, false,
                    nullptr, mid);
  const bool d = defer && p.sk > 1;
  const int rc = run_plan(p, X, ldx, Wp, K, M, N, K, epi, nullptr, out, ldo, ws, stream, false, d, rs, mid);
  if (rc != 0) return rc;
  return d ? p.sk : 1;     // split count of slabs left in the workspace (deferred), else 1
}

// The dense MoE decode path's gate/up GEMM with the routing weight in its epilogue: one launch
// and one pass over the [M, E * ffn] activation fewer per MoE layer (Mixtral 8x7B B = 64:
// moe_gate_scale was 6.5 us per layer, profiles/r5_moe/mixtral_prefill_decode_trace.md). The
// expert GEMM is a weight stream over >= 1792 column tiles, so the tile plan never splits K.
int launch_gemm_silu_gate(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                          bf16* out, long ldo, const float* gates, int gld, int ge0, int gF,
                          hipStream_t stream) {
  if (M <= 0) return 0;
  if (gates == nullptr || gF <= 0 || gF % 16 != 0 || (N / 2) % gF != 0) return -5;
  GemmPlan p = plan_gemm(M, N, K);
  if (run_plan(p, nullptr, 0, nullptr, 0, M, N, K, EPI_SILU_GATE, nullptr, nullptr, 0, nullptr, nullptr, true) != 0) {
    const int bm = M <= 16 ? 16 : M <= 32 ? 32 : M <= 64 ? 64 : 128;
    p = GemmPlan{1, 3, 0, bm <= 32 ? 1 : 2, bm, 128, 1};
  }
  RowScale rs{nullptr, 0, 0.f, 0.f};
  rs.gate = gates;
  rs.gld = gld;
  rs.ge0 = ge0;
  rs.gF = gF;
  return run_plan(p, X, ldx, W, ldw, M, N, K, EPI_SILU_GATE, nullptr, out, ldo, nullptr, stream, false, false, &rs);
}

}  // namespace bfly
