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
//    K permutation: lane group g = lane>>4 loads 64 contiguous bytes (4 sub-steps) of a row
//    per 128-wide K chunk: physical k = 32g + 8s + j for sub-step s, element j. The same map is
//    used for both operands, so every product pairs matching k.
//  * gemm_tile (M > 64, prefill / large-batch decode): BMx128x64 LDS-tiled, 4 waves (2x2),
//    both operands staged global->LDS by global_load_lds_dwordx4 (no VGPR round trip) into
//    two buffers (load of tile t+1 overlaps MFMAs on tile t), XOR-swizzled LDS image
//    (slot = chunk ^ ((row >> 1) & 7), applied on the per-lane SOURCE address because the
//    DMA writes lane-linearly; rule 21) which makes every ds_read_b128 lane group hit 16
//    distinct bank slots; bijective XCD-aware tile remap (T1).
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// ---------------------------------------------------------------------------------------
// Epilogue helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void store_out(bf16* out, long ldo, int m, int n, float v) {
  out[(long)m * ldo + n] = f2bf(v);
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

// ---------------------------------------------------------------------------------------
// Skinny (decode) GEMM
// ---------------------------------------------------------------------------------------
constexpr int kSkThreads = 256;

template <int MT, int NT>
__device__ __forceinline__ void skinny_load(const bf16* __restrict__ W, const bf16* __restrict__ X,
                                            long ldw, long ldx, int n0, int kc, int lane, int M,
                                            bf16x8 (&a)[NT][4], bf16x8 (&b)[MT][4]) {
  const int g = lane >> 4, r = lane & 15;
  const long kofs = (long)kc * 128 + 32 * g;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(W + (long)(n0 + 16 * t + r) * ldw + kofs);
#pragma unroll
    for (int s = 0; s < 4; ++s) a[t][s] = ld_nt(p + s);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int m = 16 * mt + r;
    m = m < M ? m : M - 1;
    const bf16x8* p = reinterpret_cast<const bf16x8*>(X + (long)m * ldx + kofs);
#pragma unroll
    for (int s = 0; s < 4; ++s) b[mt][s] = p[s];
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

template <int MT, int NT>
__global__ void __launch_bounds__(kSkThreads)
gemm_skinny_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                   int M, int N, int K, int epi, const bf16* __restrict__ bias,
                   bf16* __restrict__ out, long ldo, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16 * NT;
  const int nchunks = K / 128;
  const int S = gridDim.y * 4;
  const int s_idx = blockIdx.y * 4 + wid;
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

  // Cross-wave reduction through LDS: red[wave][t][mt][i][lane].
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
  for (int e = threadIdx.x; e < E; e += kSkThreads) {
    const int l = e & 63, i = (e >> 6) & 3, tm = e >> 8;
    const int t = tm / MT, mt = tm % MT;
    const int m = 16 * mt + (l & 15);
    if (m >= M) continue;
    const int n = n0 + 16 * t + (l >> 4) * 4 + i;
    const float v = red[e] + red[E + e] + red[2 * E + e] + red[3 * E + e];
    if (part) {
      part[(long)blockIdx.y * M * N + (long)m * N + n] = v;
    } else if (silu_epi) {
      if (t & 1) continue;  // the gate tile's thread combines with its up partner
      const int eu = e + MT * 4 * 64;  // same (mt, i, lane), tile t + 1
      const float u = red[eu] + red[E + eu] + red[2 * E + eu] + red[3 * E + eu];
      const int f = n0 / 2 + 16 * (t / 2) + (l >> 4) * 4 + i;
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

template <int ROWS>
__device__ __forceinline__ void tile_stage(const bf16* __restrict__ src, long ld, int row0,
                                           int row_max, int k0, char* lds, int wid, int lane) {
  // ROWS x 64 bf16 = ROWS x 8 chunks of 16 B; one wave-instruction writes 8 rows (1 KiB).
  constexpr int kInstr = ROWS / 32;  // per wave (4 waves)
#pragma unroll
  for (int i = 0; i < kInstr; ++i) {
    const int blk = i * 4 + wid;             // 8-row block index
    const int row = blk * 8 + (lane >> 3);
    const int slot = lane & 7;
    const int chunk = slot ^ ((row >> 1) & 7);
    int gr = row0 + row;
    gr = gr < row_max ? gr : row_max - 1;
    const bf16* g = src + (long)gr * ld + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)g, (lds_ptr_t)(lds + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 lds_frag(const char* lds, int row, int chunk) {
  const int slot = chunk ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + slot * 16);
}

template <int BM, int BN>
__global__ void __launch_bounds__(kTileThreads)
gemm_tile_kernel(const bf16* __restrict__ X, long ldx, const bf16* __restrict__ W, long ldw,
                 int M, int N, int K, int epi, const bf16* __restrict__ bias,
                 bf16* __restrict__ out, long ldo, float* __restrict__ part) {
  constexpr int WM = BM / 2, WN = BN / 2;    // per-wave output tile
  constexpr int TI = WM / 16, TJ = WN / 16;  // MFMA tiles per wave
  constexpr int A_BYTES = BM * kBK * 2, B_BYTES = BN * kBK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;  // one buffer = [A tile | B tile]

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int tile = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int tn = tile / mtiles, tm = tile % mtiles;  // consecutive tiles share a W panel
  const int m0 = tm * BM, n0 = tn * BN;

  const int ktiles = K / kBK;
  const int kt0 = (int)(((long)ktiles * blockIdx.y) / gridDim.y);
  const int kt1 = (int)(((long)ktiles * (blockIdx.y + 1)) / gridDim.y);

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    tile_stage<BM>(X, ldx, m0, M, kt0 * kBK, smem, wid, lane);
    tile_stage<BN>(W, ldw, n0, N, kt0 * kBK, smem + A_BYTES, wid, lane);
  }
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < kt1) {
      char* nb = smem + (cur ^ 1) * STAGE_BYTES;
      tile_stage<BM>(X, ldx, m0, M, (kt + 1) * kBK, nb, wid, lane);
      tile_stage<BN>(W, ldw, n0, N, (kt + 1) * kBK, nb + A_BYTES, wid, lane);
    }
    const char* As = smem + cur * STAGE_BYTES;
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
        for (int j = 0; j < TJ; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }

  // Epilogue: acc[i][j][r] = C[m = m0 + wm*WM + 16i + (lane>>4)*4 + r][n = n0 + wn*WN + 16j + (lane&15)]
#pragma unroll
  for (int i = 0; i < TI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WM + 16 * i + (lane >> 4) * 4 + r;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int n = n0 + wn * WN + 16 * j + (lane & 15);
        const float v = acc[i][j][r];
        if (part) {
          part[(long)blockIdx.y * M * N + (long)m * N + n] = v;
        } else if (epi == EPI_SILU) {
          if (j & 1) continue;
          const float u = acc[i][j + 1][r];
          const int f = (n0 + wn * WN) / 2 + 16 * (j / 2) + (lane & 15);
          store_out(out, ldo, m, f, silu(v) * u);
        } else {
          store_out(out, ldo, m, n, epi == EPI_BIAS ? v + bf2f(bias[n]) : v);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Host dispatch
// ---------------------------------------------------------------------------------------
static int num_cus() { return 256; }

template <int MT, int NT>
static void run_skinny(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                       int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk,
                       hipStream_t stream) {
  dim3 grid(N / (16 * NT), sk);
  gemm_skinny_kernel<MT, NT><<<grid, kSkThreads, 0, stream>>>(
      X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, sk > 1 ? ws : nullptr);
}

template <int BM, int BN>
static void run_tile(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                     int epi, const bf16* bias, bf16* out, long ldo, float* ws, int sk,
                     hipStream_t stream) {
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const size_t lds = 2 * (BM + BN) * kBK * 2;
  dim3 grid(tiles, sk);
  gemm_tile_kernel<BM, BN><<<grid, kTileThreads, lds, stream>>>(
      X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, sk > 1 ? ws : nullptr);
}

GemmPlan plan_gemm(int M, int N, int K) {
  GemmPlan p{};
  const int target = 2 * num_cus();  // workgroups wanted in flight
  if (M <= 64 && K % 128 == 0) {
    p.kind = 0;
    p.mt = (M + 15) / 16;
    p.nt = (p.mt <= 2 && N % 32 == 0) ? 2 : 1;
    const int blocks = N / (16 * p.nt);
    int sk = 1;
    const int nchunks = K / 128;
    while (blocks * sk < target && sk * 2 * 4 <= nchunks && sk < 16) sk *= 2;
    p.sk = sk;
  } else {
    p.kind = 1;
    p.bm = M <= 64 ? 64 : 128;
    p.bn = 128;
    const int tiles = ((M + p.bm - 1) / p.bm) * (N / p.bn);
    int sk = 1;
    const int ktiles = K / kBK;
    while (tiles * sk < num_cus() && sk * 2 * 4 <= ktiles && sk < 16) sk *= 2;
    p.sk = sk;
  }
  return p;
}

size_t gemm_workspace_bytes(int M, int N, int K) {
  const GemmPlan p = plan_gemm(M, N, K);
  return p.sk > 1 ? (size_t)p.sk * M * N * sizeof(float) : 0;
}

int launch_gemm(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K, int epi,
                const bf16* bias, bf16* out, long ldo, float* ws, size_t ws_bytes,
                hipStream_t stream) {
  if (M <= 0) return 0;
  GemmPlan p = plan_gemm(M, N, K);
  if (p.sk > 1 && (ws == nullptr || ws_bytes < (size_t)p.sk * M * N * sizeof(float))) p.sk = 1;
  if (p.kind == 0) {
    if (epi == EPI_SILU && p.nt == 1) p.nt = 2;  // SILU pairs gate/up tiles inside a wave
    if (N % (16 * p.nt) != 0) return -1;
#define SK_CASE(MT_, NT_) \
  if (p.mt == MT_ && p.nt == NT_) run_skinny<MT_, NT_>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream)
    SK_CASE(1, 1); SK_CASE(1, 2); SK_CASE(2, 1); SK_CASE(2, 2);
    SK_CASE(3, 1); SK_CASE(3, 2); SK_CASE(4, 1); SK_CASE(4, 2);
#undef SK_CASE
  } else {
    if (N % p.bn != 0 || K % kBK != 0) return -1;
    if (p.bm == 64) run_tile<64, 128>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream);
    else run_tile<128, 128>(X, ldx, W, ldw, M, N, K, epi, bias, out, ldo, ws, p.sk, stream);
  }
  if (p.sk > 1) {
    const int nout = epi == EPI_SILU ? N / 2 : N;
    long total = (long)M * nout;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    gemm_splitk_reduce_kernel<<<grid, 256, 0, stream>>>(ws, p.sk, M, N, epi, bias, out, ldo);
  }
  return 0;
}

}  // namespace bfly
