// torch.ops.bfly.* registrations for the HIP kernels in csrc/kernels.
//
// Every op validates shapes/dtypes/strides on the host (a bad shape must never reach a
// kernel: a GPU fault can reset every GPU of the host) and launches on the current HIP stream
// without allocating or synchronising, so whole decode steps can be captured in a hipGraph
// (torch.cuda.CUDAGraph on ROCm). Ops write into caller-provided outputs ("out" style): the
// engine owns static buffers, which is what graph replay needs.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "bfly_kernels.h"

namespace {

using at::Tensor;

// torch on ROCm exposes HIP devices as device type 'cuda'; the masquerading stream is the
// one torch.cuda.current_stream() returns (so ops order correctly with torch's own kernels).
inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

inline bfly::bf16* bf(const Tensor& t) { return reinterpret_cast<bfly::bf16*>(t.data_ptr()); }

#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_INNER(t) TORCH_CHECK((t).stride(-1) == 1, #t " must have unit inner stride")
#define CHECK_ALIGN16(t) \
  TORCH_CHECK(reinterpret_cast<uintptr_t>((t).data_ptr()) % 16 == 0, #t " must be 16-B aligned")
// paged KV caches: bf16, or FP8 e4m3 (torch.float8_e4m3fn) for the optional FP8 KV cache
#define CHECK_KV(k, v)                                                                          \
  TORCH_CHECK(((k).scalar_type() == at::kBFloat16 || (k).scalar_type() == at::kFloat8_e4m3fn) && \
                  (v).scalar_type() == (k).scalar_type(),                                       \
              "KV caches must both be bf16 or both float8_e4m3fn")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")

void rms_norm(const Tensor& x, const Tensor& w, double eps, Tensor& out,
              const c10::optional<Tensor>& residual) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "rms_norm expects 2-D x/out");
  CHECK_INNER(x); CHECK_INNER(out); CHECK_ALIGN16(x); CHECK_ALIGN16(out);
  const int rows = x.size(0), dim = x.size(1);
  TORCH_CHECK(dim % 8 == 0 && dim <= 16384, "rms_norm: dim must be a multiple of 8, <= 16384");
  TORCH_CHECK(w.numel() == dim && w.is_contiguous(), "rms_norm: weight shape");
  TORCH_CHECK(out.size(0) == rows && out.size(1) == dim, "rms_norm: out shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "rms_norm: row strides % 8");
  bfly::bf16* res = nullptr;
  if (residual.has_value()) {
    const Tensor& r = *residual;
    CHECK_BF16(r);
    TORCH_CHECK(r.is_contiguous() && r.size(0) == rows && r.size(1) == dim, "rms_norm: residual");
    res = bf(r);
  }
  c10::DeviceGuard g(x.device());
  bfly::launch_rmsnorm(bf(x), x.stride(0), res, bf(w), bf(out), out.stride(0), rows, dim,
                       (float)eps, res != nullptr, cur_stream());
}

void layer_norm(const Tensor& x, const Tensor& w, const Tensor& b, double eps, Tensor& out,
                const c10::optional<Tensor>& residual) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(b); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && out.is_contiguous(), "layer_norm: 2-D contiguous");
  const int rows = x.size(0), dim = x.size(1);
  TORCH_CHECK(dim % 8 == 0 && dim <= 16384, "layer_norm: dim");
  TORCH_CHECK(w.numel() == dim && b.numel() == dim, "layer_norm: params");
  bfly::bf16* res = nullptr;
  if (residual.has_value()) {
    TORCH_CHECK(residual->is_contiguous() && residual->sizes() == x.sizes(), "layer_norm: residual");
    res = bf(*residual);
  }
  c10::DeviceGuard g(x.device());
  bfly::launch_layernorm(bf(x), res, bf(w), bf(b), bf(out), rows, dim, (float)eps, res != nullptr,
                         cur_stream());
}

void rope_kv(Tensor& qkv, const Tensor& positions, const Tensor& cos_t, const Tensor& sin_t,
             int64_t num_q_heads, int64_t num_kv_heads, const c10::optional<Tensor>& slots,
             const c10::optional<Tensor>& k_cache, const c10::optional<Tensor>& v_cache,
             const c10::optional<Tensor>& partial) {
  CHECK_GPU(qkv); CHECK_BF16(qkv);
  TORCH_CHECK(qkv.dim() == 2 && qkv.is_contiguous(), "rope_kv: qkv must be 2-D contiguous");
  const int T = qkv.size(0);
  const int H = num_q_heads + 2 * num_kv_heads;
  TORCH_CHECK(qkv.size(1) % H == 0, "rope_kv: row length not divisible by heads");
  const int D = qkv.size(1) / H;
  TORCH_CHECK(D == 128 || D == 64, "rope_kv: head_dim must be 64 or 128");
  CHECK_I32(positions);
  TORCH_CHECK(positions.numel() == T && positions.is_contiguous(), "rope_kv: positions");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat, "rope_kv: f32 tables");
  TORCH_CHECK(cos_t.is_contiguous() && sin_t.is_contiguous() && cos_t.size(-1) == D / 2 &&
                  sin_t.sizes() == cos_t.sizes(), "rope_kv: table shape [max_pos, D/2]");
  const int* sl = nullptr;
  void *kc = nullptr, *vc = nullptr;
  int BS = 1, fp8 = 0;
  if (slots.has_value()) {
    CHECK_I32(*slots);
    TORCH_CHECK(slots->numel() == T, "rope_kv: slots");
    TORCH_CHECK(k_cache.has_value() && v_cache.has_value(), "rope_kv: caches required with slots");
    const Tensor& K = *k_cache;
    const Tensor& V = *v_cache;
    CHECK_KV(K, V);
    TORCH_CHECK(K.dim() == 4 && K.is_contiguous() && K.size(1) == num_kv_heads && K.size(3) == D,
                "rope_kv: k_cache must be [blocks, Hkv, BS, D]");
    TORCH_CHECK(V.dim() == 4 && V.is_contiguous() && V.size(1) == num_kv_heads && V.size(2) == D &&
                    V.size(3) == K.size(2) && V.size(0) == K.size(0),
                "rope_kv: v_cache must be [blocks, Hkv, D, BS]");
    sl = slots->data_ptr<int>();
    kc = K.data_ptr();
    vc = V.data_ptr();
    BS = K.size(2);
    fp8 = K.scalar_type() == at::kFloat8_e4m3fn;
  }
  const float* part = nullptr;
  int sk = 0;
  if (partial.has_value()) {
    const Tensor& P = *partial;
    TORCH_CHECK(P.scalar_type() == at::kFloat && P.dim() == 3 && P.is_contiguous() && P.size(1) == T &&
                    P.size(2) == qkv.size(1), "rope_kv: partial slabs must be [sk, T, row] f32");
    part = P.data_ptr<float>();
    sk = P.size(0);
  }
  c10::DeviceGuard g(qkv.device());
  bfly::launch_rope_kv(bf(qkv), T, num_q_heads, num_kv_heads, D, positions.data_ptr<int>(),
                       cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), sl, kc, vc, BS,
                       cur_stream(), part, sk, fp8);
}

void kv_append(const Tensor& k, const Tensor& v, const Tensor& slots, Tensor& k_cache,
               Tensor& v_cache) {
  CHECK_GPU(k); CHECK_BF16(k); CHECK_BF16(v); CHECK_I32(slots);
  TORCH_CHECK(k.dim() == 3 && v.dim() == 3 && k.sizes() == v.sizes(), "kv_append: [T, Hkv, D]");
  TORCH_CHECK(k.stride(2) == 1 && k.stride(1) == k.size(2) && v.stride(2) == 1 &&
                  v.stride(1) == v.size(2), "kv_append: rows must be dense over heads");
  const int T = k.size(0), Hkv = k.size(1), D = k.size(2);
  TORCH_CHECK(D == 128 || D == 64, "kv_append: head_dim");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D, "kv_append: k_cache");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(2) == D, "kv_append: v_cache");
  TORCH_CHECK(slots.numel() == T, "kv_append: slots");
  CHECK_KV(k_cache, v_cache);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous(), "kv_append: caches must be contiguous");
  c10::DeviceGuard g(k.device());
  bfly::launch_kv_append(bf(k), k.stride(0), bf(v), v.stride(0), slots.data_ptr<int>(),
                         k_cache.data_ptr(), v_cache.data_ptr(), T, Hkv, D, k_cache.size(2), cur_stream(),
                         k_cache.scalar_type() == at::kFloat8_e4m3fn);
}

void silu_mul(const Tensor& gu, Tensor& out, int64_t interleave) {
  CHECK_GPU(gu); CHECK_BF16(gu); CHECK_BF16(out);
  TORCH_CHECK(gu.is_contiguous() && out.is_contiguous(), "silu_mul: contiguous");
  const int ffn = out.size(-1);
  TORCH_CHECK(gu.size(-1) == 2 * ffn && ffn % 8 == 0, "silu_mul: shapes");
  TORCH_CHECK(interleave == 0 || (interleave % 8 == 0 && ffn % interleave == 0), "silu_mul: interleave");
  const long rows = out.numel() / ffn;
  TORCH_CHECK(gu.numel() == rows * 2 * ffn, "silu_mul: rows");
  c10::DeviceGuard g(gu.device());
  bfly::launch_silu_mul(bf(gu), bf(out), rows, ffn, interleave, cur_stream());
}

void gelu(const Tensor& x, Tensor& out) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(out);
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel() &&
                  x.numel() % 8 == 0, "gelu: shapes");
  c10::DeviceGuard g(x.device());
  bfly::launch_gelu(bf(x), bf(out), x.numel(), cur_stream());
}

void add(const Tensor& a, const Tensor& b, Tensor& out) {
  CHECK_GPU(a); CHECK_BF16(a); CHECK_BF16(b); CHECK_BF16(out);
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && out.is_contiguous() &&
                  a.numel() == b.numel() && a.numel() == out.numel() && a.numel() % 8 == 0,
              "add: shapes");
  c10::DeviceGuard g(a.device());
  bfly::launch_add(bf(a), bf(b), bf(out), a.numel(), cur_stream());
}

void init_hash(Tensor& out, int64_t grow0, int64_t gcol0, int64_t gcols, int64_t seed, double amp) {
  CHECK_GPU(out); CHECK_BF16(out);
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1, "init_hash: 2-D with unit inner stride");
  c10::DeviceGuard g(out.device());
  bfly::launch_init_hash(bf(out), out.size(0), out.size(1), out.stride(0), grow0, gcol0, gcols,
                         (uint32_t)seed, (float)amp, cur_stream());
}

void embed(const Tensor& ids, const Tensor& table, Tensor& out, int64_t vstart) {
  CHECK_GPU(ids); CHECK_I32(ids); CHECK_BF16(table); CHECK_BF16(out);
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous() && out.is_contiguous(), "embed: layout");
  const int T = ids.numel(), dim = table.size(1);
  TORCH_CHECK(dim % 8 == 0 && out.numel() == (long)T * dim, "embed: shapes");
  c10::DeviceGuard g(ids.device());
  bfly::launch_embed(ids.data_ptr<int>(), bf(table), bf(out), T, dim, vstart, table.size(0),
                     cur_stream());
}

// zero a device buffer with the runtime's fill (no torch elementwise kernel in a trace)
void zero_(Tensor& t) {
  CHECK_GPU(t);
  TORCH_CHECK(t.is_contiguous(), "zero_: contiguous tensors only");
  c10::DeviceGuard g(t.device());
  if (t.numel() > 0)
    TORCH_CHECK(hipMemsetAsync(t.data_ptr(), 0, t.numel() * t.element_size(), cur_stream()) == hipSuccess,
                "zero_: hipMemsetAsync failed");
}

// fill a 4-byte-element device buffer with one 32-bit pattern (runtime memset, no torch kernel)
void fill32_(Tensor& t, int64_t value) {
  CHECK_GPU(t);
  TORCH_CHECK(t.is_contiguous() && t.element_size() == 4, "fill32_: contiguous 4-byte elements");
  c10::DeviceGuard g(t.device());
  if (t.numel() > 0)
    TORCH_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(t.data_ptr()), (int)value, t.numel(),
                                  cur_stream()) == hipSuccess, "fill32_: hipMemsetD32Async failed");
}

void gather_rows(const Tensor& src, const Tensor& idx, Tensor& out) {
  CHECK_GPU(src); CHECK_GPU(idx); CHECK_GPU(out);
  TORCH_CHECK(src.dim() == 2 && out.dim() == 2 && src.stride(1) == 1 && out.stride(1) == 1, "gather_rows: 2-D rows");
  TORCH_CHECK(src.scalar_type() == out.scalar_type() && src.size(1) == out.size(1), "gather_rows: row types");
  TORCH_CHECK(idx.dim() == 1 && idx.is_contiguous() && idx.numel() == out.size(0) &&
              (idx.scalar_type() == at::kInt || idx.scalar_type() == at::kLong), "gather_rows: idx");
  const long es = src.element_size();
  TORCH_CHECK((src.size(1) * es) % 4 == 0 && (src.stride(0) * es) % 4 == 0 && (out.stride(0) * es) % 4 == 0,
              "gather_rows: rows must be whole 4-byte words");
  c10::DeviceGuard g(src.device());
  bfly::launch_gather_rows(src.data_ptr(), src.stride(0) * es / 4, idx.data_ptr(), idx.scalar_type() == at::kLong,
                           out.data_ptr(), out.stride(0) * es / 4, (int)(src.size(1) * es / 4), out.size(0),
                           src.size(0), cur_stream());
}

void sample_pack(const Tensor& scores, const Tensor& ids, Tensor& pair) {
  CHECK_GPU(scores); CHECK_GPU(ids); CHECK_I32(ids);
  TORCH_CHECK(scores.scalar_type() == at::kFloat && pair.scalar_type() == at::kFloat && scores.is_contiguous() &&
              ids.is_contiguous() && pair.is_contiguous() && pair.numel() == 2 * scores.numel() &&
              ids.numel() == scores.numel(), "sample_pack: shapes");
  c10::DeviceGuard g(scores.device());
  bfly::launch_sample_pack(scores.data_ptr<float>(), ids.data_ptr<int>(), pair.data_ptr<float>(), scores.numel(),
                           cur_stream());
}

void sample_merge(const Tensor& allp, Tensor& out) {
  CHECK_GPU(allp); CHECK_I32(out);
  TORCH_CHECK(allp.scalar_type() == at::kFloat && allp.is_contiguous() && allp.dim() == 3 && allp.size(2) == 2 &&
              out.is_contiguous() && out.numel() == allp.size(1), "sample_merge: shapes");
  c10::DeviceGuard g(allp.device());
  bfly::launch_sample_merge(allp.data_ptr<float>(), allp.size(0), allp.size(1), out.data_ptr<int>(), cur_stream());
}

void sample(const Tensor& logits, const c10::optional<Tensor>& temps,
            const c10::optional<Tensor>& seeds, int64_t vstart, Tensor& out_ids,
            Tensor& out_scores, Tensor& workspace, const c10::optional<Tensor>& thresh,
            bool check_finite) {
  CHECK_GPU(logits); CHECK_BF16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) % 8 == 0, "sample: logits");
  CHECK_ALIGN16(logits);
  const int rows = logits.size(0), V = logits.size(1);
  CHECK_I32(out_ids);
  TORCH_CHECK(out_ids.numel() == rows && out_scores.numel() == rows &&
                  out_scores.scalar_type() == at::kFloat, "sample: outputs");
  TORCH_CHECK(workspace.scalar_type() == at::kLong &&
                  workspace.numel() >= (long)rows * bfly::kSampleMaxChunks, "sample: workspace");
  const float* tp = nullptr;
  const long* sp = nullptr;
  if (temps.has_value()) {
    TORCH_CHECK(temps->scalar_type() == at::kFloat && temps->numel() == rows, "sample: temps");
    tp = temps->data_ptr<float>();
  }
  if (seeds.has_value()) {
    TORCH_CHECK(seeds->scalar_type() == at::kLong && seeds->numel() == rows, "sample: seeds");
    sp = seeds->data_ptr<int64_t>();
  }
  const float* thp = nullptr;
  if (thresh.has_value()) {
    TORCH_CHECK(thresh->scalar_type() == at::kFloat && thresh->numel() == rows && thresh->is_contiguous(),
                "sample: thresh [rows] f32");
    thp = thresh->data_ptr<float>();
  }
  c10::DeviceGuard g(logits.device());
  bfly::launch_sample(bf(logits), logits.stride(0), rows, V, vstart, tp, sp,
                      reinterpret_cast<uint64_t*>(workspace.data_ptr()), out_ids.data_ptr<int>(),
                      out_scores.data_ptr<float>(), cur_stream(), thp, check_finite ? 1 : 0);
}

// Exact top-k / top-p radix select (sample.hip). `ws` is one zeroed f32 buffer holding
// state [rows, 8] | smax [rows] (int32 bits) | hist [rows, 512].
struct TkpViews { float* state; int* smax; float* hist; };
TkpViews tkp_views(Tensor& ws, int rows) {
  CHECK_GPU(ws);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= (long)rows * (8 + 1 + 512),
              "tkp: workspace must be f32 [rows * 521] contiguous");
  float* b = ws.data_ptr<float>();
  return {b, reinterpret_cast<int*>(b + rows * 8), b + rows * 9};
}

void check_tkp_logits(const Tensor& logits, const Tensor& temps) {
  CHECK_GPU(logits); CHECK_BF16(logits); CHECK_ALIGN16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) % 8 == 0, "tkp: logits");
  TORCH_CHECK(temps.scalar_type() == at::kFloat && temps.is_contiguous() && temps.numel() == logits.size(0),
              "tkp: temps [rows] f32");
}

void tkp_begin(const Tensor& logits, const Tensor& temps, const Tensor& top_k, const Tensor& top_p, Tensor& ws) {
  check_tkp_logits(logits, temps);
  const int rows = logits.size(0);
  CHECK_I32(top_k);
  TORCH_CHECK(top_k.numel() == rows && top_k.is_contiguous(), "tkp_begin: top_k [rows] int32");
  TORCH_CHECK(top_p.scalar_type() == at::kFloat && top_p.numel() == rows && top_p.is_contiguous(),
              "tkp_begin: top_p [rows] f32");
  TkpViews v = tkp_views(ws, rows);
  c10::DeviceGuard g(logits.device());
  bfly::launch_tkp_begin(bf(logits), logits.stride(0), rows, logits.size(1), temps.data_ptr<float>(),
                         top_k.data_ptr<int>(), top_p.data_ptr<float>(), v.state, v.smax, cur_stream());
}

void tkp_pass(const Tensor& logits, const Tensor& temps, Tensor& ws, int64_t pass, int64_t phase) {
  check_tkp_logits(logits, temps);
  TORCH_CHECK(pass >= 0 && pass < 4 && (phase == 0 || phase == 1), "tkp_pass: pass 0-3, phase 0/1");
  const int rows = logits.size(0);
  TkpViews v = tkp_views(ws, rows);
  c10::DeviceGuard g(logits.device());
  bfly::launch_tkp_pass(bf(logits), logits.stride(0), rows, logits.size(1), temps.data_ptr<float>(), v.state,
                        v.smax, v.hist, (int)pass, (int)phase, cur_stream());
}

void tkp_select(const Tensor& top_p, Tensor& ws, int64_t rows, int64_t pass, int64_t phase) {
  CHECK_GPU(top_p);
  TORCH_CHECK(top_p.scalar_type() == at::kFloat && top_p.numel() == rows && top_p.is_contiguous(),
              "tkp_select: top_p [rows] f32");
  TORCH_CHECK(pass >= 0 && pass < 4 && (phase == 0 || phase == 1), "tkp_select: pass 0-3, phase 0/1");
  TkpViews v = tkp_views(ws, rows);
  c10::DeviceGuard g(top_p.device());
  bfly::launch_tkp_select(top_p.data_ptr<float>(), v.state, v.hist, rows, (int)pass, (int)phase, cur_stream());
}

void tkp_final(Tensor& ws, int64_t rows, Tensor& thresh) {
  TORCH_CHECK(thresh.scalar_type() == at::kFloat && thresh.numel() == rows && thresh.is_contiguous(),
              "tkp_final: thresh [rows] f32");
  TkpViews v = tkp_views(ws, rows);
  c10::DeviceGuard g(ws.device());
  bfly::launch_tkp_final(v.state, rows, thresh.data_ptr<float>(), cur_stream());
}

int64_t gemm_workspace_size(int64_t M, int64_t N, int64_t K) {
  return (int64_t)bfly::gemm_workspace_bytes(M, N, K);
}

std::vector<int64_t> gemm_plan(int64_t M, int64_t N, int64_t K) {
  const bfly::GemmPlan p = bfly::plan_gemm(M, N, K);
  return {p.kind, p.mt, p.nt, p.bm, p.bn, p.sk, p.wk};
}

void gemm(const Tensor& x, const Tensor& w, Tensor& out, const c10::optional<Tensor>& bias,
          int64_t epilogue, const c10::optional<Tensor>& workspace) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm: 2-D operands");
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm: K mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm: row strides % 8");
  TORCH_CHECK(K % 64 == 0, "gemm: K must be a multiple of 64, got ", K);
  TORCH_CHECK(N % 128 == 0, "gemm: N must be a multiple of 128, got ", N);
  const int nout = epilogue == bfly::EPI_SILU ? N / 2 : N;
  TORCH_CHECK(out.size(0) == M && out.size(1) == nout, "gemm: out shape");
  const bfly::bf16* bp = nullptr;
  if (epilogue == bfly::EPI_BIAS) {
    TORCH_CHECK(bias.has_value() && bias->numel() == N, "gemm: bias required");
    CHECK_BF16(*bias);
    bp = bf(*bias);
  }
  float* ws = nullptr;
  size_t ws_bytes = 0;
  if (workspace.has_value()) {
    ws = reinterpret_cast<float*>(workspace->data_ptr());
    ws_bytes = workspace->numel() * workspace->element_size();
  }
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm(bf(x), x.stride(0), bf(w), w.stride(0), M, N, K, epilogue, bp,
                                   bf(out), out.stride(0), ws, ws_bytes, cur_stream());
  TORCH_CHECK(rc == 0, "gemm: unsupported shape M=", M, " N=", N, " K=", K, " (rc=", rc, ")");
}

// out[M, N/2] = moe_gate_scale(silu(gate) * up): the dense MoE decode gate/up GEMM over the
// concatenated local experts with the routing weights gates[M, E] applied in its epilogue.
void gemm_silu_gate(const Tensor& x, const Tensor& w, Tensor& out, const Tensor& gates, int64_t e0,
                    int64_t num_local) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_GPU(gates);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm_silu_gate: 2-D operands");
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 128 == 0, "gemm_silu_gate: shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_silu_gate: row strides % 8");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N / 2, "gemm_silu_gate: out shape");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.dim() == 2 && gates.is_contiguous() &&
                  gates.size(0) == M, "gemm_silu_gate: gates [M, E] f32");
  TORCH_CHECK(num_local > 0 && (N / 2) % num_local == 0 && e0 >= 0 && e0 + num_local <= gates.size(1),
              "gemm_silu_gate: experts");
  const int F = (N / 2) / num_local;
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm_silu_gate(bf(x), x.stride(0), bf(w), w.stride(0), M, N, K, bf(out),
                                             out.stride(0), gates.data_ptr<float>(), (int)gates.size(1),
                                             (int)e0, F, cur_stream());
  TORCH_CHECK(rc == 0, "gemm_silu_gate: unsupported shape M=", M, " N=", N, " K=", K, " F=", F, " (rc=", rc, ")");
}

static bfly::RowScale row_scale(const Tensor& ssp, double eps, int M, int K);

// Decode GEMM over the K-tile-blocked copy `wp` ([N/256][K/64][256][64] viewed as [N, K]) of a
// weight; optional RMSNorm row scale (ssp, eps) and MoE gate (gates, e0, num_local: epilogue 3).
// Returns 0 when it ran, < 0 when the shape's plan has no packed form (nothing launched).
int64_t gemm_packed(const Tensor& x, const Tensor& wp, Tensor& out, int64_t epilogue,
                    const c10::optional<Tensor>& ssp, double eps, const c10::optional<Tensor>& gates,
                    int64_t e0, int64_t num_local, const c10::optional<Tensor>& workspace, bool defer) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(wp); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && wp.dim() == 2 && out.dim() == 2 && wp.is_contiguous(), "gemm_packed: operands");
  CHECK_INNER(x); CHECK_INNER(out); CHECK_ALIGN16(x); CHECK_ALIGN16(wp);
  const int M = x.size(0), K = x.size(1), N = wp.size(0);
  TORCH_CHECK(wp.size(1) == K && x.stride(0) % 8 == 0, "gemm_packed: shape");
  const bool silu = epilogue == bfly::EPI_SILU || epilogue == bfly::EPI_SILU_GATE;
  TORCH_CHECK(epilogue != bfly::EPI_BIAS, "gemm_packed: no bias epilogue");
  TORCH_CHECK(out.size(0) == M && out.size(1) == (silu ? N / 2 : N), "gemm_packed: out shape");
  bfly::RowScale rs{nullptr, 0, 0.f, 0.f};
  if (ssp.has_value()) rs = row_scale(*ssp, eps, M, K);
  if (epilogue == bfly::EPI_SILU_GATE) {
    TORCH_CHECK(gates.has_value() && gates->scalar_type() == at::kFloat && gates->dim() == 2 &&
                    gates->is_contiguous() && gates->size(0) == M, "gemm_packed: gates [M, E] f32");
    TORCH_CHECK(num_local > 0 && (N / 2) % num_local == 0 && e0 + num_local <= gates->size(1), "gemm_packed: experts");
    rs.gate = gates->data_ptr<float>();
    rs.gld = (int)gates->size(1);
    rs.ge0 = (int)e0;
    rs.gF = (int)((N / 2) / num_local);
    if (rs.gF % 16 != 0) return -5;
  }
  const bool any = ssp.has_value() || epilogue == bfly::EPI_SILU_GATE;
  float* ws = nullptr;
  size_t ws_bytes = 0;
  if (workspace.has_value()) {
    TORCH_CHECK(workspace->scalar_type() == at::kFloat && workspace->is_contiguous(), "gemm_packed: workspace");
    ws = workspace->data_ptr<float>();
    ws_bytes = workspace->numel() * 4;
  }
  c10::DeviceGuard g(x.device());
  return bfly::launch_gemm_packed(bf(x), x.stride(0), bf(wp), M, N, K, (int)epilogue, bf(out), out.stride(0),
                                  cur_stream(), any ? &rs : nullptr, false, ws, ws_bytes, defer);
}

// 0 when the plan for (M, N, K, epilogue) has a packed-weight form (launch_gemm_packed dry run)
int64_t gemm_packed_check(int64_t M, int64_t N, int64_t K, int64_t epilogue) {
  return bfly::launch_gemm_packed(nullptr, 0, nullptr, (int)M, (int)N, (int)K, (int)epilogue, nullptr, 0, nullptr,
                                  nullptr, true);
}

// Benchmark / tuning entry: run an explicit plan [kind, mt, nt, wk, bm, bn, sk].
void gemm_with_plan(const Tensor& x, const Tensor& w, Tensor& out, std::vector<int64_t> plan,
                    int64_t epilogue, const c10::optional<Tensor>& workspace,
                    const c10::optional<Tensor>& bias) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2 && plan.size() == 7, "gemm_with_plan: args");
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm_with_plan: K mismatch");
  const int nout = epilogue == bfly::EPI_SILU ? N / 2 : N;
  TORCH_CHECK(out.size(0) == M && out.size(1) == nout, "gemm_with_plan: out shape");
  bfly::GemmPlan p{};
  p.kind = plan[0]; p.mt = plan[1]; p.nt = plan[2]; p.wk = plan[3]; p.bm = plan[4]; p.bn = plan[5]; p.sk = plan[6];
  float* ws = nullptr;
  size_t ws_bytes = 0;
  if (workspace.has_value()) {
    ws = reinterpret_cast<float*>(workspace->data_ptr());
    ws_bytes = workspace->numel() * workspace->element_size();
  }
  const bfly::bf16* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(epilogue == bfly::EPI_BIAS && bias->numel() == N && bias->is_contiguous(), "gemm_with_plan: bias");
    CHECK_BF16(*bias);
    bp = bf(*bias);
  }
  TORCH_CHECK(epilogue != bfly::EPI_BIAS || bp != nullptr, "gemm_with_plan: bias epilogue needs a bias");
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm_plan(p, bf(x), x.stride(0), bf(w), w.stride(0), M, N, K, epilogue,
                                        bp, bf(out), out.stride(0), ws, ws_bytes, cur_stream());
  TORCH_CHECK(rc == 0, "gemm_with_plan: plan rejected (rc=", rc, ")");
}

// GEMM whose split-K reduce is left to the consumer: returns the split count (slabs in the
// workspace) or 1 (out written).
int64_t gemm_deferred(const Tensor& x, const Tensor& w, Tensor& out, Tensor& workspace) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm_deferred: 2-D operands");
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 128 == 0, "gemm_deferred: shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_deferred: row strides % 8");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N && out.is_contiguous(), "gemm_deferred: out");
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.is_contiguous(), "gemm_deferred: workspace");
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm_deferred(bf(x), x.stride(0), bf(w), w.stride(0), M, N, K, bf(out),
                                            out.stride(0), workspace.data_ptr<float>(),
                                            workspace.numel() * 4, cur_stream());
  TORCH_CHECK(rc > 0, "gemm_deferred: unsupported shape M=", M, " N=", N, " K=", K, " (rc=", rc, ")");
  return rc;
}

// RMSNorm row scale of a consumer GEMM: ssp [M, chunks] f32 partial sums of squares written by
// rms_norm_rows for X = x * g rows of width K.
static bfly::RowScale row_scale(const Tensor& ssp, double eps, int M, int K) {
  CHECK_GPU(ssp);
  TORCH_CHECK(ssp.scalar_type() == at::kFloat && ssp.dim() == 2 && ssp.is_contiguous() && ssp.size(0) == M,
              "row scale: ssp must be [M, chunks] f32");
  return bfly::RowScale{ssp.data_ptr<float>(), (int)ssp.size(1), 1.f / (float)K, (float)eps};
}

// gemm() with the consumer RMSNorm row scale (X rows = x * g of rms_norm_rows)
void gemm_rs(const Tensor& x, const Tensor& w, Tensor& out, const c10::optional<Tensor>& bias,
             int64_t epilogue, const c10::optional<Tensor>& workspace, const Tensor& ssp, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm_rs: 2-D operands");
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 128 == 0, "gemm_rs: shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_rs: row strides % 8");
  const int nout = epilogue == bfly::EPI_SILU ? N / 2 : N;
  TORCH_CHECK(out.size(0) == M && out.size(1) == nout, "gemm_rs: out shape");
  const bfly::bf16* bp = nullptr;
  if (epilogue == bfly::EPI_BIAS) {
    TORCH_CHECK(bias.has_value() && bias->numel() == N, "gemm_rs: bias required");
    CHECK_BF16(*bias);
    bp = bf(*bias);
  }
  float* ws = nullptr;
  size_t ws_bytes = 0;
  if (workspace.has_value()) {
    ws = reinterpret_cast<float*>(workspace->data_ptr());
    ws_bytes = workspace->numel() * workspace->element_size();
  }
  const bfly::RowScale rs = row_scale(ssp, eps, M, K);
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm(bf(x), x.stride(0), bf(w), w.stride(0), M, N, K, epilogue, bp,
                                   bf(out), out.stride(0), ws, ws_bytes, cur_stream(), &rs);
  TORCH_CHECK(rc == 0, "gemm_rs: unsupported plan M=", M, " N=", N, " K=", K, " (rc=", rc, ")");
}

int64_t gemm_deferred_rs(const Tensor& x, const Tensor& w, Tensor& out, Tensor& workspace, const Tensor& ssp,
                         double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemm_deferred_rs: 2-D operands");
  CHECK_INNER(x); CHECK_INNER(w); CHECK_INNER(out);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && K % 64 == 0 && N % 128 == 0, "gemm_deferred_rs: shape");
  TORCH_CHECK(x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "gemm_deferred_rs: row strides % 8");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N && out.is_contiguous(), "gemm_deferred_rs: out");
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.is_contiguous(), "gemm_deferred_rs: workspace");
  const bfly::RowScale rs = row_scale(ssp, eps, M, K);
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm_deferred(bf(x), x.stride(0), bf(w), w.stride(0), M, N, K, bf(out),
                                            out.stride(0), workspace.data_ptr<float>(),
                                            workspace.numel() * 4, cur_stream(), &rs);
  TORCH_CHECK(rc > 0, "gemm_deferred_rs: unsupported plan M=", M, " N=", N, " K=", K, " (rc=", rc, ")");
  return rc;
}

// Row-split add + RMSNorm for a row-scaling consumer GEMM: out = x * w (un-normalised),
// ssp [rows, chunks] = per-chunk sums of squares. x: bf16 [rows, dim] or f32 slabs [sk, rows, dim].
void rms_norm_rows(const Tensor& x, const Tensor& w, Tensor& out, Tensor& ssp,
                   const c10::optional<Tensor>& residual) {
  CHECK_GPU(x); CHECK_BF16(w); CHECK_BF16(out);
  const bool slabs = x.scalar_type() == at::kFloat;
  TORCH_CHECK(slabs ? (x.dim() == 3 && x.is_contiguous()) : (x.dim() == 2 && x.scalar_type() == at::kBFloat16),
              "rms_norm_rows: x must be bf16 [rows, dim] or f32 slabs [sk, rows, dim]");
  const int sk = slabs ? x.size(0) : 0;
  const int rows = x.size(x.dim() - 2), dim = x.size(x.dim() - 1);
  TORCH_CHECK(dim % 8 == 0 && w.numel() == dim && w.is_contiguous(), "rms_norm_rows: dim / weight");
  if (!slabs) {
    CHECK_INNER(x); CHECK_ALIGN16(x);
    TORCH_CHECK(x.stride(0) % 8 == 0, "rms_norm_rows: row stride % 8");
  }
  TORCH_CHECK(out.is_contiguous() && out.size(0) == rows && out.size(1) == dim, "rms_norm_rows: out");
  TORCH_CHECK(ssp.scalar_type() == at::kFloat && ssp.is_contiguous() && ssp.dim() == 2 && ssp.size(0) == rows &&
                  ssp.size(1) == bfly::rmsnorm_rows_chunks(dim),
              "rms_norm_rows: ssp must be [rows, ", bfly::rmsnorm_rows_chunks(dim), "] f32");
  bfly::bf16* res = nullptr;
  if (residual.has_value()) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) == rows && residual->size(1) == dim,
                "rms_norm_rows: residual");
    res = bf(*residual);
  }
  c10::DeviceGuard g(out.device());
  const int rc = bfly::launch_rmsnorm_rows(slabs ? nullptr : bf(x), slabs ? 0 : x.stride(0), res, bf(w), bf(out),
                                           ssp.data_ptr<float>(), rows, dim, res != nullptr, cur_stream(),
                                           slabs ? x.data_ptr<float>() : nullptr, sk);
  TORCH_CHECK(rc == 0, "rms_norm_rows: launch failed (rc=", rc, ")");
}

void splitk_reduce(const Tensor& slabs, Tensor& out) {
  CHECK_GPU(slabs);
  TORCH_CHECK(slabs.scalar_type() == at::kFloat && slabs.dim() == 3 && slabs.is_contiguous(), "splitk_reduce: slabs [sk, M, N] f32");
  CHECK_BF16(out);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == slabs.size(1) && out.size(1) == slabs.size(2) && out.is_contiguous(), "splitk_reduce: out");
  c10::DeviceGuard g(out.device());
  bfly::launch_splitk_reduce(slabs.data_ptr<float>(), slabs.size(0), slabs.size(1), slabs.size(2), bf(out),
                             out.stride(0), cur_stream());
}

void rms_norm_partial(const Tensor& slabs, const Tensor& w, double eps, Tensor& out,
                      const c10::optional<Tensor>& residual) {
  CHECK_GPU(slabs);
  TORCH_CHECK(slabs.scalar_type() == at::kFloat && slabs.dim() == 3 && slabs.is_contiguous(), "rms_norm_partial: slabs [sk, rows, dim]");
  const int sk = slabs.size(0), rows = slabs.size(1), dim = slabs.size(2);
  CHECK_BF16(w); CHECK_BF16(out);
  TORCH_CHECK(dim % 8 == 0 && dim <= 16384 && w.numel() == dim, "rms_norm_partial: dim");
  TORCH_CHECK(out.is_contiguous() && out.size(0) == rows && out.size(1) == dim, "rms_norm_partial: out");
  bfly::bf16* res = nullptr;
  if (residual.has_value()) {
    CHECK_BF16(*residual);
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) == rows && residual->size(1) == dim, "rms_norm_partial: residual");
    res = bf(*residual);
  }
  c10::DeviceGuard g(out.device());
  bfly::launch_rmsnorm(nullptr, dim, res, bf(w), bf(out), dim, rows, dim, (float)eps, res != nullptr,
                       cur_stream(), slabs.data_ptr<float>(), sk);
}

// rms_norm_partial + MoE routing of the normalised rows (router_w [E, dim], E = 4 or 8)
void rms_norm_partial_route(const Tensor& slabs, const Tensor& w, double eps, Tensor& out, Tensor& residual,
                            const Tensor& router_w, int64_t top_k, Tensor& gates, Tensor& topk_ids, Tensor& topk_w) {
  CHECK_GPU(slabs);
  TORCH_CHECK(slabs.scalar_type() == at::kFloat && slabs.dim() == 3 && slabs.is_contiguous(), "rms_norm_partial_route: slabs");
  const int sk = slabs.size(0), rows = slabs.size(1), dim = slabs.size(2);
  CHECK_BF16(w); CHECK_BF16(out); CHECK_BF16(residual); CHECK_BF16(router_w);
  TORCH_CHECK(dim % 8 == 0 && w.numel() == dim, "rms_norm_partial_route: dim");
  TORCH_CHECK(out.is_contiguous() && out.size(0) == rows && out.size(1) == dim, "rms_norm_partial_route: out");
  TORCH_CHECK(residual.is_contiguous() && residual.size(0) == rows && residual.size(1) == dim, "rms_norm_partial_route: residual");
  const int E = router_w.size(0);
  TORCH_CHECK(router_w.dim() == 2 && router_w.is_contiguous() && router_w.size(1) == dim, "rms_norm_partial_route: router_w");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.is_contiguous() && gates.size(0) == rows && gates.size(1) == E,
              "rms_norm_partial_route: gates");
  TORCH_CHECK(topk_ids.scalar_type() == at::kInt && topk_w.scalar_type() == at::kFloat && topk_ids.is_contiguous() &&
                  topk_w.is_contiguous() && topk_ids.size(0) == rows && topk_ids.size(1) == top_k &&
                  topk_w.size(0) == rows && topk_w.size(1) == top_k, "rms_norm_partial_route: topk");
  c10::DeviceGuard g(out.device());
  const int rc = bfly::launch_rmsnorm_route(slabs.data_ptr<float>(), sk, bf(residual), bf(w), bf(out), rows, dim,
                                            (float)eps, true, bf(router_w), E, (int)top_k, gates.data_ptr<float>(),
                                            topk_ids.data_ptr<int>(), topk_w.data_ptr<float>(), cur_stream());
  TORCH_CHECK(rc == 0, "rms_norm_partial_route: unsupported (E=", E, ", dim=", dim, ", rc=", rc, ")");
}

int64_t rms_norm_route_ok(int64_t E, int64_t dim) { return (E == 4 || E == 8) && dim % 8 == 0 && dim <= 16384 ? 1 : 0; }

int64_t attn_decode_splits(int64_t max_ctx, int64_t part_tokens) {
  return bfly::attn_decode_splits(max_ctx, part_tokens);
}

int64_t attn_decode_part_tokens(int64_t B, int64_t Hkv, int64_t max_ctx) {
  return bfly::attn_decode_part_tokens(B, Hkv, max_ctx);
}

void attn_decode(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache,
                 const Tensor& block_tables, const Tensor& ctx_lens, double scale,
                 int64_t max_ctx, int64_t part_tokens, Tensor& out,
                 const c10::optional<Tensor>& part_o, const c10::optional<Tensor>& part_ml) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_KV(k_cache, v_cache); CHECK_BF16(out);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == q.size(2), "attn_decode: q [B, Hq, D]");
  const int B = q.size(0), Hq = q.size(1), D = q.size(2);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous(), "attn_decode: caches");
  const int Hkv = k_cache.size(1), BS = k_cache.size(2);
  TORCH_CHECK(k_cache.size(3) == D && v_cache.size(2) == D && v_cache.size(3) == BS, "attn_decode: cache dims");
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)B * Hq * D, "attn_decode: out");
  CHECK_I32(block_tables); CHECK_I32(ctx_lens);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && block_tables.stride(1) == 1,
              "attn_decode: block_tables");
  TORCH_CHECK(ctx_lens.numel() >= B, "attn_decode: ctx_lens");
  TORCH_CHECK((long)block_tables.size(1) * BS >= max_ctx, "attn_decode: block table too narrow for max_ctx");
  if (part_tokens <= 0) part_tokens = bfly::attn_decode_part_tokens(B, Hkv, max_ctx);
  const int nsplit = bfly::attn_decode_splits(max_ctx, part_tokens);
  float *po = nullptr, *pml = nullptr;
  if (nsplit > 1) {
    TORCH_CHECK(part_o.has_value() && part_ml.has_value(), "attn_decode: partial buffers required");
    TORCH_CHECK(part_o->numel() >= (long)B * Hkv * nsplit * 16 * D, "attn_decode: part_o too small");
    TORCH_CHECK(part_ml->numel() >= (long)B * Hkv * nsplit * 16 * 2, "attn_decode: part_ml too small");
    po = part_o->data_ptr<float>();
    pml = part_ml->data_ptr<float>();
  }
  c10::DeviceGuard g(q.device());
  const int rc = bfly::launch_attn_decode(bf(q), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                          block_tables.data_ptr<int>(), block_tables.stride(0),
                                          ctx_lens.data_ptr<int>(), B, Hq, Hkv, D, BS, (float)scale,
                                          max_ctx, part_tokens, bf(out), po, pml, cur_stream(),
                                          k_cache.scalar_type() == at::kFloat8_e4m3fn);
  TORCH_CHECK(rc == 0, "attn_decode: unsupported configuration (rc=", rc, ")");
}

// Chunked prefill over the paged cache (attention_paged.hip): q [T, Hq, D] rows grouped per
// sequence by cu_q, positions [T] their absolute positions, tables [nseq, max_blocks].
void attn_prefill_paged(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& tables,
                        const Tensor& cu_q, const Tensor& positions, int64_t max_q, double scale, Tensor& out) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_KV(k_cache, v_cache); CHECK_BF16(out);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == q.size(2), "attn_prefill_paged: q [T, Hq, D]");
  TORCH_CHECK(out.dim() == 3 && out.sizes() == q.sizes() && out.stride(2) == 1 && out.stride(1) == out.size(2),
              "attn_prefill_paged: out like q");
  const int Hq = q.size(1), D = q.size(2);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous(), "attn_prefill_paged: caches");
  const int Hkv = k_cache.size(1), BS = k_cache.size(2);
  TORCH_CHECK(k_cache.size(3) == D && v_cache.size(2) == D && v_cache.size(3) == BS, "attn_prefill_paged: cache dims");
  CHECK_I32(tables); CHECK_I32(cu_q); CHECK_I32(positions);
  const int nseq = cu_q.numel() - 1;
  TORCH_CHECK(tables.dim() == 2 && tables.size(0) >= nseq && tables.stride(1) == 1, "attn_prefill_paged: tables");
  TORCH_CHECK(positions.numel() >= q.size(0) && cu_q.is_contiguous() && positions.is_contiguous(),
              "attn_prefill_paged: positions / cu_q");
  c10::DeviceGuard g(q.device());
  const int rc = bfly::launch_attn_prefill_paged(bf(q), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                                 tables.data_ptr<int>(), tables.stride(0), cu_q.data_ptr<int>(),
                                                 positions.data_ptr<int>(), nseq, (int)max_q, Hq, Hkv, D, BS,
                                                 (float)scale, bf(out), out.stride(0), cur_stream(),
                                                 k_cache.scalar_type() == at::kFloat8_e4m3fn);
  TORCH_CHECK(rc == 0, "attn_prefill_paged: unsupported configuration (rc=", rc, ")");
}

void attn_prefill(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& cu_seqlens,
                  int64_t max_seqlen, double scale, bool causal, Tensor& out,
                  const c10::optional<Tensor>& cu_seqlens_k, const c10::optional<Tensor>& lse) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_BF16(out);
  for (const Tensor* t : {&q, &k, &v, (const Tensor*)&out})
    TORCH_CHECK(t->dim() == 3 && t->stride(2) == 1 && t->stride(1) == t->size(2) && t->stride(0) % 8 == 0,
                "attn_prefill: [T, H, D] with dense heads");
  const int Hq = q.size(1), Hkv = k.size(1), D = q.size(2);
  TORCH_CHECK(k.size(2) == D && v.size(2) == D && v.size(1) == Hkv, "attn_prefill: dims");
  TORCH_CHECK(out.size(1) == Hq && out.size(2) == D && out.size(0) == q.size(0), "attn_prefill: out");
  CHECK_I32(cu_seqlens);
  const int nseq = cu_seqlens.numel() - 1;
  const int* cuk = nullptr;
  if (cu_seqlens_k.has_value()) {   // keys from another chunk (context-parallel ring step)
    CHECK_I32(*cu_seqlens_k);
    TORCH_CHECK(cu_seqlens_k->numel() == nseq + 1 && cu_seqlens_k->is_contiguous(), "attn_prefill: cu_seqlens_k");
    TORCH_CHECK(!causal, "attn_prefill: separate key offsets are only defined for non-causal attention");
    cuk = cu_seqlens_k->data_ptr<int>();
  }
  float* lp = nullptr;
  if (lse.has_value()) {
    CHECK_GPU(*lse);
    TORCH_CHECK(lse->scalar_type() == at::kFloat && lse->is_contiguous() && lse->numel() == q.size(0) * Hq,
                "attn_prefill: lse [T, Hq] f32");
    lp = lse->data_ptr<float>();
  }
  c10::DeviceGuard g(q.device());
  const int rc = bfly::launch_attn_prefill(bf(q), q.stride(0), bf(k), k.stride(0), bf(v), v.stride(0),
                                           cu_seqlens.data_ptr<int>(), nseq, max_seqlen, Hq, Hkv, D,
                                           (float)scale, causal, bf(out), out.stride(0), cur_stream(),
                                           cuk, lp);
  TORCH_CHECK(rc == 0, "attn_prefill: unsupported configuration (rc=", rc, ")");
}

void attn_lse_merge(Tensor& acc_o, Tensor& acc_lse, const Tensor& o, const Tensor& lse) {
  CHECK_GPU(acc_o); CHECK_BF16(o);
  TORCH_CHECK(acc_o.scalar_type() == at::kFloat && acc_o.dim() == 3 && acc_o.is_contiguous() && acc_o.size(2) == 128,
              "attn_lse_merge: acc_o [T, H, 128] f32");
  const int T = acc_o.size(0), H = acc_o.size(1);
  TORCH_CHECK(acc_lse.scalar_type() == at::kFloat && acc_lse.is_contiguous() && acc_lse.numel() == (int64_t)T * H,
              "attn_lse_merge: acc_lse [T, H] f32");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (int64_t)T * H,
              "attn_lse_merge: lse [T, H] f32");
  TORCH_CHECK(o.dim() == 3 && o.size(0) == T && o.size(1) == H && o.size(2) == 128 && o.stride(2) == 1 &&
                  o.stride(1) == 128, "attn_lse_merge: o [T, H, 128] bf16 with dense heads");
  c10::DeviceGuard g(acc_o.device());
  const int rc = bfly::launch_attn_lse_merge(acc_o.data_ptr<float>(), acc_lse.data_ptr<float>(), bf(o), o.stride(0),
                                             lse.data_ptr<float>(), T, H, 128, cur_stream());
  TORCH_CHECK(rc == 0, "attn_lse_merge: rejected (", rc, ")");
}

void moe_route(const Tensor& x, const Tensor& wr, int64_t top_k, Tensor& gates, Tensor& topk_ids,
               Tensor& topk_w) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(wr);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "moe_route: x");
  TORCH_CHECK(wr.dim() == 2 && wr.is_contiguous() && wr.size(1) == x.size(1), "moe_route: router weight");
  const int T = x.size(0), H = x.size(1), E = wr.size(0);
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.is_contiguous() && gates.numel() == (long)T * E, "moe_route: gates");
  CHECK_I32(topk_ids);
  TORCH_CHECK(topk_ids.numel() == (long)T * top_k && topk_w.numel() == (long)T * top_k &&
                  topk_w.scalar_type() == at::kFloat, "moe_route: topk outputs");
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_moe_route(bf(x), x.stride(0), bf(wr), T, H, E, top_k, gates.data_ptr<float>(),
                                        topk_ids.data_ptr<int>(), topk_w.data_ptr<float>(), cur_stream());
  TORCH_CHECK(rc == 0, "moe_route: unsupported (E <= 64, k <= 8, H % 8 == 0)");
}

int64_t moe_max_tiles(int64_t TK, int64_t El, int64_t bm) { return bfly::moe_max_tiles(TK, El, (int)bm); }

// block counts (EP IPC receive buffer): rows form blocks of `bcap`; only the first bcnt[b] rows of
// block b are valid (device-resident counts, so no host sync)
static const int* block_counts(const c10::optional<Tensor>& bcnt, int64_t bcap, long rows, const char* what) {
  if (!bcnt.has_value()) return nullptr;
  CHECK_I32(*bcnt);
  TORCH_CHECK(bcap > 0 && rows % bcap == 0 && bcnt->numel() >= rows / bcap, what, ": block counts");
  return bcnt->data_ptr<int>();
}

void moe_align(const Tensor& topk_ids, int64_t e0, int64_t num_local, Tensor& rows, Tensor& slot_of,
               Tensor& tiles, Tensor& count, int64_t bm, const c10::optional<Tensor>& bcnt, int64_t bcap) {
  TORCH_CHECK(bm == 64 || bm == 128 || bm == 256, "moe_align: tile rows 64, 128 or 256");
  CHECK_GPU(topk_ids); CHECK_I32(topk_ids); CHECK_I32(rows); CHECK_I32(slot_of); CHECK_I32(tiles); CHECK_I32(count);
  TORCH_CHECK(topk_ids.dim() == 2 && topk_ids.is_contiguous(), "moe_align: topk_ids [T, k]");
  const int T = topk_ids.size(0), K = topk_ids.size(1);
  TORCH_CHECK(num_local > 0 && num_local <= 64, "moe_align: 1..64 local experts");
  TORCH_CHECK(rows.numel() >= (long)T * K && slot_of.numel() == (long)T * K, "moe_align: rows / slot_of size");
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 4 && tiles.is_contiguous() &&
                  tiles.size(0) >= bfly::moe_max_tiles(T * K, num_local, (int)bm), "moe_align: tiles [max_tiles, 4]");
  TORCH_CHECK(count.numel() == 1, "moe_align: count");
  c10::DeviceGuard g(topk_ids.device());
  const int* bc = block_counts(bcnt, bcap, T, "moe_align");
  const int rc = bfly::launch_moe_align(topk_ids.data_ptr<int>(), T, K, e0, num_local, (int)bm,
                                        rows.data_ptr<int>(), slot_of.data_ptr<int>(),
                                        reinterpret_cast<int4*>(tiles.data_ptr<int>()), count.data_ptr<int>(), cur_stream(),
                                        bc, (int)bcap);
  TORCH_CHECK(rc == 0, "moe_align: rejected (", rc, ")");
}

void moe_grouped_gemm(const Tensor& x, const Tensor& w, Tensor& out, const c10::optional<Tensor>& rows,
                      const Tensor& tiles, const Tensor& count, int64_t w_estride, int64_t n, int64_t k,
                      int64_t num_experts, int64_t epilogue, int64_t bm, const c10::optional<Tensor>& part) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_I32(tiles); CHECK_I32(count);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.size(1) >= k, "moe_grouped_gemm: x");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.stride(0) % 8 == 0, "moe_grouped_gemm: w");
  TORCH_CHECK(n % 128 == 0 && k % 64 == 0, "moe_grouped_gemm: N % 128, K % 64");
  TORCH_CHECK(epilogue == bfly::EPI_NONE || epilogue == bfly::EPI_SILU, "moe_grouped_gemm: epilogue");
  const long ldw = w.stride(0);
  const long last = (num_experts - 1) * w_estride + (n - 1) * ldw + k;
  TORCH_CHECK(num_experts > 0 && last <= w.numel(), "moe_grouped_gemm: expert slices exceed w");
  const int nout = epilogue == bfly::EPI_SILU ? n / 2 : n;
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) == nout, "moe_grouped_gemm: out");
  const int* rp = nullptr;
  if (rows.has_value()) {
    CHECK_I32(*rows);
    rp = rows->data_ptr<int>();
  } else {
    TORCH_CHECK(x.size(0) >= out.size(0), "moe_grouped_gemm: slot rows");
  }
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 4, "moe_grouped_gemm: tiles");
  int sk = 1;
  float* pp = nullptr;
  if (part.has_value()) {   // split-K: f32 slabs [sk][slots][n], reduced by moe_combine_slabs
    const Tensor& pt = *part;
    CHECK_GPU(pt);
    TORCH_CHECK(pt.scalar_type() == at::kFloat && pt.dim() == 3 && pt.is_contiguous() && pt.size(1) == out.size(0) &&
                    pt.size(2) == n && epilogue == bfly::EPI_NONE, "moe_grouped_gemm: part [sk, slots, n] f32");
    sk = (int)pt.size(0);
    pp = pt.data_ptr<float>();
  }
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_gemm_grouped(bf(x), x.stride(0), bf(w), ldw, w_estride, n, k, epilogue, rp,
                                           reinterpret_cast<const int4*>(tiles.data_ptr<int>()), count.data_ptr<int>(),
                                           tiles.size(0), bf(out), out.stride(0), cur_stream(), (int)bm,
                                           (int)out.size(0), sk, pp);
  TORCH_CHECK(rc == 0, "moe_grouped_gemm: rejected (", rc, ")");
}

void moe_combine(const Tensor& y, const Tensor& slot_of, const Tensor& topk_w, Tensor& out,
                 const c10::optional<Tensor>& bcnt, int64_t bcap) {
  CHECK_GPU(y); CHECK_BF16(y); CHECK_I32(slot_of); CHECK_BF16(out);
  TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.dim() == 2 && topk_w.is_contiguous(), "moe_combine: topk_w");
  const int T = topk_w.size(0), K = topk_w.size(1), H = out.size(1);
  TORCH_CHECK(slot_of.numel() == (long)T * K && out.size(0) == T && out.is_contiguous() && y.is_contiguous() &&
                  y.size(1) == H, "moe_combine: shapes");
  c10::DeviceGuard g(y.device());
  const int rc = bfly::launch_moe_combine(bf(y), slot_of.data_ptr<int>(), topk_w.data_ptr<float>(), T, K, H, bf(out),
                                          cur_stream(), block_counts(bcnt, bcap, T, "moe_combine"), (int)bcap);
  TORCH_CHECK(rc == 0, "moe_combine: H % 8");
}

void moe_combine_slabs(const Tensor& part, const Tensor& slot_of, const Tensor& topk_w, Tensor& out,
                       const c10::optional<Tensor>& bcnt, int64_t bcap) {
  CHECK_GPU(part); CHECK_I32(slot_of); CHECK_BF16(out);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.dim() == 3 && part.is_contiguous(), "moe_combine_slabs: part");
  TORCH_CHECK(topk_w.scalar_type() == at::kFloat && topk_w.dim() == 2 && topk_w.is_contiguous(), "moe_combine_slabs: topk_w");
  const int T = topk_w.size(0), K = topk_w.size(1), H = out.size(1);
  TORCH_CHECK(slot_of.numel() == (long)T * K && out.size(0) == T && out.is_contiguous() && part.size(2) == H &&
                  part.size(1) >= (long)T * K, "moe_combine_slabs: shapes");
  c10::DeviceGuard g(part.device());
  const int rc = bfly::launch_moe_combine_slabs(part.data_ptr<float>(), (int)part.size(0), part.size(1) * (long)H,
                                                slot_of.data_ptr<int>(), topk_w.data_ptr<float>(), T, K, H, bf(out),
                                                cur_stream(), block_counts(bcnt, bcap, T, "moe_combine_slabs"), (int)bcap);
  TORCH_CHECK(rc == 0, "moe_combine_slabs: H % 4");
}

void ep_pack(const Tensor& x, const Tensor& ids, const Tensor& w, const c10::optional<Tensor>& slots,
             int64_t experts_per_rank, int64_t ep, int64_t cap, Tensor& send, Tensor& meta, Tensor& slot) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_I32(ids); CHECK_BF16(send); CHECK_I32(slot);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "ep_pack: x [T, H] contiguous");
  const int T = x.size(0), H = x.size(1);
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) == T && ids.is_contiguous(), "ep_pack: ids [T, k]");
  const int K = ids.size(1);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == (long)T * K, "ep_pack: w [T, k] f32");
  TORCH_CHECK(cap >= T && send.is_contiguous() && send.size(0) == ep * cap && send.size(1) == H, "ep_pack: send [ep*cap, H]");
  TORCH_CHECK(meta.scalar_type() == at::kFloat && meta.is_contiguous() && meta.size(0) == ep * cap &&
                  meta.size(1) == 2 * K, "ep_pack: meta [ep*cap, 2k] f32");
  TORCH_CHECK(slot.is_contiguous() && slot.numel() == (long)T * ep, "ep_pack: slot [T, ep]");
  const int* sp = nullptr;
  if (slots.has_value()) {
    CHECK_I32(*slots);
    TORCH_CHECK(slots->numel() == T, "ep_pack: slots [T]");
    sp = slots->data_ptr<int>();
  }
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_ep_pack(bf(x), ids.data_ptr<int>(), w.data_ptr<float>(), sp, T, K, H,
                                      (int)experts_per_rank, (int)ep, (int)cap, bf(send), meta.data_ptr<float>(),
                                      slot.data_ptr<int>(), cur_stream());
  TORCH_CHECK(rc == 0, "ep_pack: rejected (", rc, ")");
}

void ep_combine(const Tensor& back, const Tensor& slot, Tensor& out) {
  CHECK_GPU(back); CHECK_BF16(back); CHECK_I32(slot); CHECK_BF16(out);
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && back.is_contiguous() && back.size(1) == out.size(1),
              "ep_combine: shapes");
  const int T = out.size(0);
  TORCH_CHECK(T == 0 || slot.numel() % T == 0, "ep_combine: slot [T, ep]");
  const int ep = T ? (int)(slot.numel() / T) : 2;
  c10::DeviceGuard g(back.device());
  const int rc = bfly::launch_ep_combine(bf(back), slot.data_ptr<int>(), T, out.size(1), ep, bf(out), cur_stream());
  TORCH_CHECK(rc == 0, "ep_combine: rejected (", rc, ")");
}

void moe_gate_scale(Tensor& h, const Tensor& gates, int64_t e0, int64_t num_local) {
  CHECK_GPU(h); CHECK_BF16(h);
  TORCH_CHECK(h.dim() == 2 && h.is_contiguous(), "moe_gate_scale: h");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.dim() == 2 && gates.is_contiguous() &&
                  gates.size(0) == h.size(0), "moe_gate_scale: gates");
  const int T = h.size(0), E = gates.size(1);
  TORCH_CHECK(h.size(1) % num_local == 0 && e0 + num_local <= E, "moe_gate_scale: experts");
  const int F = h.size(1) / num_local;
  TORCH_CHECK(F % 8 == 0, "moe_gate_scale: F % 8");
  c10::DeviceGuard g(h.device());
  bfly::launch_moe_gate_scale(bf(h), gates.data_ptr<float>(), T, E, e0, num_local, F, cur_stream());
}

void probe(int64_t which, Tensor& out) {
  CHECK_GPU(out);
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 64 * 16, "probe: out");
  c10::DeviceGuard g(out.device());
  bfly::launch_probe(which, out.data_ptr<float>(), cur_stream());
}

// ---- one-shot IPC all-reduce -------------------------------------------------------------
// Buffers are raw device pointers carried as int64 (they are shared with peer processes via
// hipIpc handles and live for the communicator's lifetime, outside torch's allocator).
int64_t car_alloc(int64_t bytes) {
  TORCH_CHECK(bytes > 0, "car_alloc: bytes");
  void* p = bfly::car_alloc((size_t)bytes);
  TORCH_CHECK(p != nullptr, "car_alloc: hipExtMallocWithFlags(uncached) failed");
  return reinterpret_cast<int64_t>(p);
}
void car_free(int64_t p) { bfly::car_free(reinterpret_cast<void*>(p)); }
Tensor car_ipc_handle(int64_t p) {
  Tensor h = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  TORCH_CHECK(bfly::car_ipc_handle(reinterpret_cast<void*>(p), h.data_ptr<uint8_t>()) == 0,
              "car_ipc_handle: hipIpcGetMemHandle failed");
  return h;
}
int64_t car_ipc_open(const Tensor& h) {
  TORCH_CHECK(h.scalar_type() == at::kByte && h.numel() == 64 && h.is_contiguous() && !h.is_cuda(),
              "car_ipc_open: expects a 64-byte CPU uint8 handle");
  void* p = bfly::car_ipc_open(h.data_ptr<uint8_t>());
  TORCH_CHECK(p != nullptr, "car_ipc_open: hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}
void car_ipc_close(int64_t p) { bfly::car_ipc_close(reinterpret_cast<void*>(p)); }
int64_t car_error(int64_t p) { return bfly::car_error(reinterpret_cast<const void*>(p)); }
void car_clear_error(int64_t p) {
  TORCH_CHECK(bfly::car_clear_error(reinterpret_cast<void*>(p)) == 0, "car_clear_error: hipMemset failed");
}

void custom_all_reduce(const Tensor& inp, Tensor& out, const c10::optional<Tensor>& residual,
                       const c10::optional<Tensor>& w, double eps, at::IntArrayRef bases,
                       int64_t rank, int64_t cap, const c10::optional<Tensor>& slabs,
                       bool two_shot, int64_t blocks) {
  CHECK_GPU(inp); CHECK_BF16(inp); CHECK_BF16(out);
  TORCH_CHECK(inp.dim() == 2 && inp.is_contiguous() && out.is_contiguous() &&
                  out.sizes() == inp.sizes(), "custom_all_reduce: 2-D contiguous, same shape");
  CHECK_ALIGN16(inp); CHECK_ALIGN16(out);
  const int world = (int)bases.size();
  TORCH_CHECK(world == 2 || world == 4 || world == 8, "custom_all_reduce: world must be 2, 4 or 8");
  TORCH_CHECK(rank >= 0 && rank < world, "custom_all_reduce: rank");
  const int rows = inp.size(0), dim = inp.size(1);
  TORCH_CHECK(dim % 8 == 0 && dim <= 16384, "custom_all_reduce: dim % 8 == 0 and <= 16384");
  TORCH_CHECK((int64_t)rows * dim * 2 <= cap, "custom_all_reduce: message larger than the buffer");
  bfly::ArPeers peers{};
  for (int i = 0; i < world; ++i) {
    TORCH_CHECK(bases[i] != 0, "custom_all_reduce: null peer buffer");
    peers.base[i] = reinterpret_cast<char*>(bases[i]);
  }
  peers.herr = bfly::health_words_device();
  bfly::bf16* res = nullptr;
  const bfly::bf16* wp = nullptr;
  if (residual.has_value()) {
    TORCH_CHECK(w.has_value(), "custom_all_reduce: norm weight required with residual");
    const Tensor& r = *residual;
    CHECK_BF16(r); CHECK_BF16((*w));
    TORCH_CHECK(r.is_contiguous() && r.sizes() == inp.sizes(), "custom_all_reduce: residual shape");
    TORCH_CHECK(w->numel() == dim && w->is_contiguous(), "custom_all_reduce: weight shape");
    TORCH_CHECK(out.data_ptr() != inp.data_ptr(), "custom_all_reduce: fused norm cannot run in place");
    res = bf(r);
    wp = bf(*w);
  }
  const float* sp = nullptr;
  int sk = 0;
  if (slabs.has_value()) {   // inp is then only the shape / output placeholder
    const Tensor& sl = *slabs;
    CHECK_GPU(sl);
    TORCH_CHECK(sl.scalar_type() == at::kFloat && sl.dim() == 3 && sl.is_contiguous() &&
                    sl.size(1) == rows && sl.size(2) == dim, "custom_all_reduce: slabs [sk, rows, dim] f32");
    CHECK_ALIGN16(sl);
    sp = sl.data_ptr<float>();
    sk = (int)sl.size(0);
  }
  c10::DeviceGuard g(inp.device());
  const int rc = bfly::launch_custom_allreduce(bf(inp), bf(out), res, wp, (float)eps, rows, dim,
                                               peers, world, (int)rank, cap, cur_stream(), sp, sk,
                                               two_shot, (int)blocks);
  TORCH_CHECK(rc == 0, "custom_all_reduce: launch rejected (", rc, ")");
}

// ---- byte-minimal EP dispatch over peer IPC buffers (allocated with car_alloc) ------------
static bfly::ArPeers ep_peers(at::IntArrayRef bases) {
  TORCH_CHECK(bases.size() == 2 || bases.size() == 4 || bases.size() == 8, "ep_ipc: 2, 4 or 8 ranks");
  bfly::ArPeers peers{};
  for (size_t i = 0; i < bases.size(); ++i) {
    TORCH_CHECK(bases[i] != 0, "ep_ipc: null peer buffer");
    peers.base[i] = reinterpret_cast<char*>(bases[i]);
  }
  peers.herr = bfly::health_words_device();
  return peers;
}

// Host-mapped health words (bfly_kernels.h): [kHealthCar] custom all-reduce and [kHealthEp]
// EP IPC flag-wait timeouts. health_init allocates them (eagerly, before any graph capture);
// reading them is a plain host load, safe from a poller thread while the GPU is busy or stuck.
bool health_init() { return bfly::health_words_device() != nullptr; }

// Read and reset the runtime's sticky last-error code: a failed stream capture leaves
// hipErrorStreamCaptureInvalidated behind, which the next checked launch would report as
// its own failure (ModelRunner clears it before falling back to eager decode).
int64_t hip_clear_error() { return (int64_t)hipGetLastError(); }

std::vector<int64_t> health_words() {
  return {(int64_t)bfly::health_word(bfly::kHealthCar), (int64_t)bfly::health_word(bfly::kHealthEp)};
}

void health_clear(int64_t word) { bfly::health_clear((int)word); }

std::vector<int64_t> ep_ipc_layout(int64_t ep, int64_t capmax, int64_t H, int64_t K) {
  const bfly::EpLayout L = bfly::ep_ipc_layout((int)ep, (int)capmax, (int)H, (int)K);
  return {L.x, L.ids, L.w, L.back, L.total};
}

// a [rows, cols] view of a region of this rank's IPC buffer (no ownership: the buffer lives as
// long as the EpIpc object that allocated it)
Tensor ep_ipc_view(int64_t ptr, int64_t offset, int64_t rows, int64_t cols, int64_t dtype, int64_t device) {
  const at::ScalarType st = dtype == 0 ? at::kBFloat16 : dtype == 1 ? at::kInt : at::kFloat;
  return at::from_blob(reinterpret_cast<char*>(ptr) + offset, {rows, cols},
                       at::TensorOptions().dtype(st).device(at::kCUDA, (int)device));
}

void ep_ipc_dispatch(const Tensor& x, const Tensor& ids, const Tensor& w, const c10::optional<Tensor>& slots,
                     int64_t experts_per_rank, int64_t capmax, at::IntArrayRef bases, int64_t rank, Tensor& slot) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_I32(ids); CHECK_I32(slot);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "ep_ipc_dispatch: x [T, H] contiguous");
  const int T = x.size(0), H = x.size(1), ep = (int)bases.size();
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) == T && ids.is_contiguous(), "ep_ipc_dispatch: ids [T, k]");
  const int K = ids.size(1);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == (long)T * K, "ep_ipc_dispatch: w");
  TORCH_CHECK(capmax >= T, "ep_ipc_dispatch: more tokens than the buffer's capacity");
  TORCH_CHECK(slot.is_contiguous() && slot.numel() == (long)T * ep, "ep_ipc_dispatch: slot [T, ep]");
  const int* sp = nullptr;
  if (slots.has_value()) {
    CHECK_I32(*slots);
    TORCH_CHECK(slots->numel() == T, "ep_ipc_dispatch: slots [T]");
    sp = slots->data_ptr<int>();
  }
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_ep_ipc_dispatch(bf(x), ids.data_ptr<int>(), w.data_ptr<float>(), sp, T, K, H,
                                              (int)experts_per_rank, ep, (int)capmax, ep_peers(bases), (int)rank,
                                              slot.data_ptr<int>(), cur_stream());
  TORCH_CHECK(rc == 0, "ep_ipc_dispatch: rejected (", rc, ")");
}

// Prefill-sized dispatch (T up to capmax; ep_ipc.hip launch_ep_ipc_dispatch_prefill)
void ep_ipc_dispatch_prefill(const Tensor& x, const Tensor& ids, const Tensor& w, int64_t experts_per_rank,
                             int64_t capmax, at::IntArrayRef bases, int64_t rank, Tensor& slot) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_I32(ids); CHECK_I32(slot);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "ep_ipc_dispatch_prefill: x [T, H] contiguous");
  const int T = x.size(0), H = x.size(1), ep = (int)bases.size();
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) == T && ids.is_contiguous(), "ep_ipc_dispatch_prefill: ids [T, k]");
  const int K = ids.size(1);
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == (long)T * K,
              "ep_ipc_dispatch_prefill: w");
  TORCH_CHECK(capmax >= T, "ep_ipc_dispatch_prefill: more tokens than the buffer's capacity");
  TORCH_CHECK(slot.is_contiguous() && slot.numel() == (long)T * ep, "ep_ipc_dispatch_prefill: slot [T, ep]");
  c10::DeviceGuard g(x.device());
  const int rc = bfly::launch_ep_ipc_dispatch_prefill(bf(x), ids.data_ptr<int>(), w.data_ptr<float>(), T, K, H,
                                                      (int)experts_per_rank, ep, (int)capmax, ep_peers(bases),
                                                      (int)rank, slot.data_ptr<int>(), cur_stream());
  TORCH_CHECK(rc == 0, "ep_ipc_dispatch_prefill: rejected (", rc, ")");
}

int64_t ep_ipc_counts_offset() { return bfly::ep_ipc_counts_offset(); }

void ep_ipc_wait(const Tensor& like, at::IntArrayRef bases, int64_t rank) {
  CHECK_GPU(like);
  c10::DeviceGuard g(like.device());
  const int rc = bfly::launch_ep_ipc_wait(ep_peers(bases), (int)bases.size(), (int)rank, cur_stream());
  TORCH_CHECK(rc == 0, "ep_ipc_wait: rejected (", rc, ")");
}

void ep_ipc_return(const Tensor& y, int64_t K, int64_t capmax, at::IntArrayRef bases, int64_t rank) {
  CHECK_GPU(y); CHECK_BF16(y);
  const int ep = (int)bases.size();
  TORCH_CHECK(y.dim() == 2 && y.is_contiguous() && y.size(0) == ep * capmax, "ep_ipc_return: y [ep*capmax, H]");
  c10::DeviceGuard g(y.device());
  const int rc = bfly::launch_ep_ipc_return(bf(y), y.size(1), (int)K, ep, (int)capmax, ep_peers(bases), (int)rank,
                                            cur_stream());
  TORCH_CHECK(rc == 0, "ep_ipc_return: rejected (", rc, ")");
}

void ep_ipc_combine(const Tensor& slot, int64_t K, int64_t capmax, at::IntArrayRef bases, int64_t rank, Tensor& out) {
  CHECK_GPU(out); CHECK_BF16(out); CHECK_I32(slot);
  const int T = out.size(0), ep = (int)bases.size();
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && slot.numel() == (long)T * ep, "ep_ipc_combine: shapes");
  c10::DeviceGuard g(out.device());
  const int rc = bfly::launch_ep_ipc_combine(slot.data_ptr<int>(), T, out.size(1), (int)K, ep, (int)capmax,
                                             ep_peers(bases), (int)rank, bf(out), cur_stream());
  TORCH_CHECK(rc == 0, "ep_ipc_combine: rejected (", rc, ")");
}

std::vector<int64_t> ep_ipc_stats(int64_t p) {
  long long v[2] = {0, 0};
  TORCH_CHECK(bfly::ep_ipc_stats(reinterpret_cast<const void*>(p), v) == 0, "ep_ipc_stats: hipMemcpy failed");
  return {v[0], v[1]};
}

}  // namespace

TORCH_LIBRARY(bfly, m) {
  m.def("rms_norm(Tensor x, Tensor w, float eps, Tensor(a!) out, Tensor(b!)? residual) -> ()");
  m.def("layer_norm(Tensor x, Tensor w, Tensor b, float eps, Tensor(a!) out, Tensor(b!)? residual) -> ()");
  m.def("rope_kv(Tensor(a!) qkv, Tensor positions, Tensor cos, Tensor sin, int num_q_heads, "
        "int num_kv_heads, Tensor? slots, Tensor(b!)? k_cache, Tensor(c!)? v_cache, Tensor? partial=None) -> ()");
  m.def("gemm_deferred(Tensor x, Tensor w, Tensor(a!) out, Tensor(b!) workspace) -> int");
  m.def("splitk_reduce(Tensor slabs, Tensor(a!) out) -> ()");
  m.def("rms_norm_partial(Tensor slabs, Tensor w, float eps, Tensor(a!) out, Tensor(b!)? residual) -> ()");
  m.def("rms_norm_partial_route(Tensor slabs, Tensor w, float eps, Tensor(a!) out, Tensor(b!) residual, Tensor router_w, "
        "int top_k, Tensor(c!) gates, Tensor(d!) topk_ids, Tensor(e!) topk_w) -> ()");
  m.def("rms_norm_route_ok(int E, int dim) -> int", &rms_norm_route_ok);
  m.def("gemm_slab_offset() -> int", []() -> int64_t { return (int64_t)bfly::gemm_slab_offset_floats(); });
  m.def("gemm_rs(Tensor x, Tensor w, Tensor(a!) out, Tensor? bias, int epilogue, Tensor(b!)? workspace, "
        "Tensor ssp, float eps) -> ()");
  m.def("gemm_deferred_rs(Tensor x, Tensor w, Tensor(a!) out, Tensor(b!) workspace, Tensor ssp, float eps) -> int");
  m.def("rms_norm_rows(Tensor x, Tensor w, Tensor(a!) out, Tensor(b!) ssp, Tensor(c!)? residual) -> ()");
  m.def("rms_norm_rows_chunks(int dim) -> int", [](int64_t dim) -> int64_t { return bfly::rmsnorm_rows_chunks(dim); });
  m.def("gemm_rowscale_check(int M, int N, int K, int epilogue) -> int",
        [](int64_t M, int64_t N, int64_t K, int64_t e) -> int64_t { return bfly::gemm_rowscale_check(M, N, K, e); });
  m.def("kv_append(Tensor k, Tensor v, Tensor slots, Tensor(a!) k_cache, Tensor(b!) v_cache) -> ()");
  m.def("silu_mul(Tensor gu, Tensor(a!) out, int interleave) -> ()");
  m.def("gelu(Tensor x, Tensor(a!) out) -> ()");
  m.def("add(Tensor a, Tensor b, Tensor(a!) out) -> ()");
  m.def("init_hash(Tensor(a!) out, int grow0, int gcol0, int gcols, int seed, float amp) -> ()");
  m.def("embed(Tensor ids, Tensor table, Tensor(a!) out, int vstart) -> ()");
  m.def("gather_rows(Tensor src, Tensor idx, Tensor(a!) out) -> ()");
  m.def("zero_(Tensor(a!) t) -> ()");
  m.def("fill32_(Tensor(a!) t, int value) -> ()");
  m.def("sample_pack(Tensor scores, Tensor ids, Tensor(a!) pair) -> ()");
  m.def("sample_merge(Tensor allp, Tensor(a!) out) -> ()");
  m.def("sample(Tensor logits, Tensor? temps, Tensor? seeds, int vstart, Tensor(a!) out_ids, "
        "Tensor(b!) out_scores, Tensor(c!) workspace, Tensor? thresh=None, bool check_finite=False) -> ()");
  m.def("tkp_begin(Tensor logits, Tensor temps, Tensor top_k, Tensor top_p, Tensor(a!) ws) -> ()");
  m.def("tkp_pass(Tensor logits, Tensor temps, Tensor(a!) ws, int pass_, int phase) -> ()");
  m.def("tkp_select(Tensor top_p, Tensor(a!) ws, int rows, int pass_, int phase) -> ()");
  m.def("tkp_final(Tensor(a!) ws, int rows, Tensor(b!) thresh) -> ()");
  m.def("gemm(Tensor x, Tensor w, Tensor(a!) out, Tensor? bias, int epilogue, Tensor(b!)? workspace) -> ()");
  m.def("gemm_silu_gate(Tensor x, Tensor w, Tensor(a!) out, Tensor gates, int e0, int num_local) -> ()");
  m.def("gemm_packed(Tensor x, Tensor wp, Tensor(a!) out, int epilogue, Tensor? ssp=None, float eps=0.0, "
        "Tensor? gates=None, int e0=0, int num_local=1, Tensor(b!)? workspace=None, bool defer=False) -> int");
  m.def("gemm_packed_check(int M, int N, int K, int epilogue) -> int", &gemm_packed_check);
  m.def("gemm_with_plan(Tensor x, Tensor w, Tensor(a!) out, int[] plan, int epilogue, Tensor(b!)? workspace, "
        "Tensor? bias=None) -> ()");
  m.def("gemm_workspace_size(int M, int N, int K) -> int", &gemm_workspace_size);
  m.def("gemm_plan(int M, int N, int K) -> int[]", &gemm_plan);
  m.def("gemm_check(int M, int N, int K, int epilogue) -> int",
        [](int64_t M, int64_t N, int64_t K, int64_t e) -> int64_t { return bfly::gemm_check(M, N, K, e); });
  m.def("attn_decode_splits(int max_ctx, int part_tokens) -> int", &attn_decode_splits);
  m.def("attn_decode_part_tokens(int B, int Hkv, int max_ctx) -> int", &attn_decode_part_tokens);
  m.def("attn_decode(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor ctx_lens, "
        "float scale, int max_ctx, int part_tokens, Tensor(a!) out, Tensor(b!)? part_o, "
        "Tensor(c!)? part_ml) -> ()");
  m.def("moe_route(Tensor x, Tensor wr, int top_k, Tensor(a!) gates, Tensor(b!) topk_ids, Tensor(c!) topk_w) -> ()");
  m.def("moe_gate_scale(Tensor(a!) h, Tensor gates, int e0, int num_local) -> ()");
  m.def("moe_max_tiles(int tk, int num_local, int bm=64) -> int", &moe_max_tiles);
  m.def("moe_align(Tensor topk_ids, int e0, int num_local, Tensor(a!) rows, Tensor(b!) slot_of, Tensor(c!) tiles, "
        "Tensor(d!) count, int bm=64, Tensor? bcnt=None, int bcap=0) -> ()");
  m.def("moe_grouped_gemm(Tensor x, Tensor w, Tensor(a!) out, Tensor? rows, Tensor tiles, Tensor count, int w_estride, "
        "int n, int k, int num_experts, int epilogue, int bm=64, Tensor(b!)? part=None) -> ()");
  m.def("moe_combine(Tensor y, Tensor slot_of, Tensor topk_w, Tensor(a!) out, Tensor? bcnt=None, int bcap=0) -> ()");
  m.def("moe_combine_slabs(Tensor part, Tensor slot_of, Tensor topk_w, Tensor(a!) out, Tensor? bcnt=None, "
        "int bcap=0) -> ()");
  m.def("ep_ipc_dispatch_prefill(Tensor x, Tensor ids, Tensor w, int experts_per_rank, int capmax, int[] bases, "
        "int rank, Tensor(a!) slot) -> ()");
  m.def("ep_ipc_counts_offset() -> int", &ep_ipc_counts_offset);
  m.def("ep_pack(Tensor x, Tensor ids, Tensor w, Tensor? slots, int experts_per_rank, int ep, int cap, "
        "Tensor(a!) send, Tensor(b!) meta, Tensor(c!) slot) -> ()");
  m.def("ep_combine(Tensor back, Tensor slot, Tensor(a!) out) -> ()");
  m.def("probe(int which, Tensor(a!) out) -> ()");
  m.def("car_alloc(int bytes) -> int", &car_alloc);
  m.def("car_free(int ptr) -> ()", &car_free);
  m.def("car_ipc_handle(int ptr) -> Tensor", &car_ipc_handle);
  m.def("car_ipc_open(Tensor handle) -> int", &car_ipc_open);
  m.def("car_ipc_close(int ptr) -> ()", &car_ipc_close);
  m.def("car_error(int ptr) -> int", &car_error);
  m.def("car_clear_error(int ptr) -> ()", &car_clear_error);
  m.def("car_buffer_bytes(int cap) -> int", [](int64_t cap) -> int64_t { return bfly::car_buffer_bytes(cap); });
  m.def("custom_all_reduce(Tensor inp, Tensor(a!) out, Tensor(b!)? residual, Tensor? w, float eps, "
        "int[] bases, int rank, int cap, Tensor? slabs=None, bool two_shot=False, int blocks=128) -> ()");
  m.def("ep_ipc_layout(int ep, int capmax, int H, int K) -> int[]", &ep_ipc_layout);
  m.def("ep_ipc_view(int ptr, int offset, int rows, int cols, int dtype, int device) -> Tensor", &ep_ipc_view);
  m.def("ep_ipc_dispatch(Tensor x, Tensor ids, Tensor w, Tensor? slots, int experts_per_rank, int capmax, "
        "int[] bases, int rank, Tensor(a!) slot) -> ()");
  m.def("ep_ipc_wait(Tensor like, int[] bases, int rank) -> ()");
  m.def("ep_ipc_return(Tensor y, int k, int capmax, int[] bases, int rank) -> ()");
  m.def("health_init() -> bool", &health_init);
  m.def("hip_clear_error() -> int", &hip_clear_error);
  m.def("health_words() -> int[]", &health_words);
  m.def("health_clear(int word=-1) -> ()", &health_clear);
  m.def("ep_ipc_combine(Tensor slot, int k, int capmax, int[] bases, int rank, Tensor(a!) out) -> ()");
  m.def("ep_ipc_stats(int ptr) -> int[]", &ep_ipc_stats);
  m.def("ep_ipc_error(int ptr) -> int", [](int64_t p) -> int64_t { return bfly::ep_ipc_error(reinterpret_cast<const void*>(p)); });
  m.def("attn_prefill_paged(Tensor q, Tensor k_cache, Tensor v_cache, Tensor tables, Tensor cu_q, "
        "Tensor positions, int max_q, float scale, Tensor(a!) out) -> ()");
  m.def("attn_prefill(Tensor q, Tensor k, Tensor v, Tensor cu_seqlens, int max_seqlen, float scale, "
        "bool causal, Tensor(a!) out, Tensor? cu_seqlens_k=None, Tensor(b!)? lse=None) -> ()");
  m.def("attn_lse_merge(Tensor(a!) acc_o, Tensor(b!) acc_lse, Tensor o, Tensor lse) -> ()");
}

TORCH_LIBRARY_IMPL(bfly, CUDA, m) {
  m.impl("rms_norm", &rms_norm);
  m.impl("layer_norm", &layer_norm);
  m.impl("rope_kv", &rope_kv);
  m.impl("kv_append", &kv_append);
  m.impl("silu_mul", &silu_mul);
  m.impl("gelu", &gelu);
  m.impl("add", &add);
  m.impl("embed", &embed);
  m.impl("gather_rows", &gather_rows);
  m.impl("zero_", &zero_);
  m.impl("fill32_", &fill32_);
  m.impl("sample_pack", &sample_pack);
  m.impl("sample_merge", &sample_merge);
  m.impl("init_hash", &init_hash);
  m.impl("sample", &sample);
  m.impl("tkp_begin", &tkp_begin);
  m.impl("tkp_pass", &tkp_pass);
  m.impl("tkp_select", &tkp_select);
  m.impl("tkp_final", &tkp_final);
  m.impl("gemm", &gemm);
  m.impl("gemm_silu_gate", &gemm_silu_gate);
  m.impl("gemm_packed", &gemm_packed);
  m.impl("gemm_with_plan", &gemm_with_plan);
  m.impl("gemm_deferred", &gemm_deferred);
  m.impl("splitk_reduce", &splitk_reduce);
  m.impl("rms_norm_partial", &rms_norm_partial);
  m.impl("rms_norm_partial_route", &rms_norm_partial_route);
  m.impl("gemm_rs", &gemm_rs);
  m.impl("gemm_deferred_rs", &gemm_deferred_rs);
  m.impl("rms_norm_rows", &rms_norm_rows);
  m.impl("attn_decode", &attn_decode);
  m.impl("attn_prefill", &attn_prefill);
  m.impl("attn_prefill_paged", &attn_prefill_paged);
  m.impl("attn_lse_merge", &attn_lse_merge);
  m.impl("probe", &probe);
  m.impl("custom_all_reduce", &custom_all_reduce);
  m.impl("moe_route", &moe_route);
  m.impl("moe_gate_scale", &moe_gate_scale);
  m.impl("moe_align", &moe_align);
  m.impl("moe_grouped_gemm", &moe_grouped_gemm);
  m.impl("moe_combine", &moe_combine);
  m.impl("moe_combine_slabs", &moe_combine_slabs);
  m.impl("ep_ipc_dispatch_prefill", &ep_ipc_dispatch_prefill);
  m.impl("ep_pack", &ep_pack);
  m.impl("ep_combine", &ep_combine);
  m.impl("ep_ipc_dispatch", &ep_ipc_dispatch);
  m.impl("ep_ipc_wait", &ep_ipc_wait);
  m.impl("ep_ipc_return", &ep_ipc_return);
  m.impl("ep_ipc_combine", &ep_ipc_combine);
}
