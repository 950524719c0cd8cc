// Layout probes: tiny kernels that expose the hardware operand/accumulator maps the real
// kernels rely on (MFMA fragment layouts, ds_read_b64_tr_b16 gather), so a layout assumption
// is checked against exact integer data on the device instead of inferred from a failing
// kernel (cdna_hip_programming.md §3: "check the map with exact integer data").
#include "bfly_common.h"
#include "bfly_kernels.h"

namespace bfly {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4* lds_s4_ptr_p;

// probe 0: ds_read_b64_tr_b16. LDS holds a [64][128] int16 image, element (r, c) = r*128 + c,
// stored plainly (no swizzle). Lane l supplies address (row = 4*(l>>4) + ((l&15)>>2),
// col = 4*(l&3)); out[l*4 + j] = element j returned to lane l.
// probe 1: mfma_f32_32x32x16_bf16 with A[i][k] = i*16 + k + 1 (rows 0..31, k 0..15) and
// B[k][j] = (k == j % 16) ? 1 : 0 ... written as plain integers so D is exact; lane l passes
// A[row l&31][k = 8(l>>5)+j] and B[k = 8(l>>5)+j][col l&31]; out[l*16 + r] = D register r.
__global__ void probe_kernel(int which, float* out) {
  __shared__ __attribute__((aligned(16))) short lds[64 * 128];
  const int l = threadIdx.x;
  if (which == 0) {
    for (int i = l; i < 64 * 128; i += 64) lds[i] = (short)i;
    __syncthreads();
    const int row = 4 * (l >> 4) + ((l & 15) >> 2), col = 4 * (l & 3);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr_p)(lds + row * 128 + col));
    for (int j = 0; j < 4; ++j) out[l * 4 + j] = (float)v[j];
  } else if (which == 3 || which == 4) {
    // the prefill kernel's V addressing on its swizzled image: element (r, c) = r (which 3)
    // or c (which 4); dt = 0, kt = 0, s = 0. out[l*8 + j] = element j (lo 0..3, hi 4..7).
    for (int i = l; i < 64 * 128; i += 64) {
      const int r = i / 128, c = i % 128, ch = c / 8;
      const int off = (r * 256 + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)))) / 2 + (c % 8);
      lds[off] = (short)(which == 3 ? r : c);
    }
    __syncthreads();
    const int tq = (l & 15) >> 2, tp = l & 3, tg = (l >> 4) & 1, hi = l >> 5;
    const int ch = 2 * tg + (tp >> 1);
    const int krow = 4 * hi + tq;
    auto off = [](int row, int c) { return row * 256 + 16 * (c ^ (((row & 3) << 2) | ((row >> 2) & 3))); };
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr_p)((char*)lds + off(krow, ch) + 8 * (tp & 1)));
    s16x4 h4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr_p)((char*)lds + off(krow + 8, ch) + 8 * (tp & 1)));
    for (int j = 0; j < 4; ++j) { out[l * 8 + j] = (float)lo[j]; out[l * 8 + 4 + j] = (float)h4[j]; }
  } else if (which == 1 || which == 2) {
    // mfma_f32_32x32x16_bf16 C/D map: which 1: A[i][k] = i, B = 1 -> D[i][j] = 16 i;
    // which 2: A = 1, B[k][j] = j -> D[i][j] = 16 j. out[l*16 + r] = D register r.
    bf16x8 a, b;
    const int r = l & 31;
    for (int j = 0; j < 8; ++j) {
      a[j] = (bf16)(float)(which == 1 ? r : 1);
      b[j] = (bf16)(float)(which == 1 ? 1 : r);
    }
    f32x16 acc = {};
    acc = mfma32(a, b, acc);
    for (int i = 0; i < 16; ++i) out[l * 16 + i] = acc[i];
  }
}

void launch_probe(int which, float* out, hipStream_t stream) {
  probe_kernel<<<1, 64, 0, stream>>>(which, out);
}

}  // namespace bfly
