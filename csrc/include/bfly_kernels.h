// Host-side launch API of the butterfly_amd HIP kernels. Every launcher is stream-ordered,
// allocation-free and synchronisation-free, so it can be captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace bfly {

typedef __bf16 bf16;

// EPI_SILU_GATE: the SwiGLU epilogue followed by the MoE dense decode path's routing weight
// (what moe_gate_scale did as a separate pass): see RowScale::gate.
enum GemmEpilogue { EPI_NONE = 0, EPI_BIAS = 1, EPI_SILU = 2, EPI_SILU_GATE = 3 };

// Per-row output scales of the tile / decode-ring / mid-M epilogues.
// RMSNorm: the X rows are un-normalised RMSNorm inputs (x * g); row m is multiplied by
// rsqrt(sum_c ss[m * chunks + c] * inv_dim + eps) before the epilogue.
// MoE gate (EPI_SILU_GATE, tile kernel only): SwiGLU output column f of row m is rounded to
// bf16, multiplied by gate[m * gld + ge0 + f / gF] and rounded again, bit-identical to the
// SiLU epilogue followed by moe_gate_scale.
struct RowScale {
  const float* ss;   // nullptr: no scaling
  int chunks;
  float inv_dim, eps;
  const float* gate = nullptr;
  int gld = 0, ge0 = 0, gF = 0;
};

struct GemmPlan {
  int kind;  // 0 = skinny (decode), 1 = LDS-tiled, 3 = decode ring, 5 = mid-M 8-wave,
             // 4 = 256x256 8-phase big tile (BK 64, prefill; kind 2 was the removed ring kernel)
  int mt, nt;
  int wk;    // skinny: waves splitting K inside a workgroup (1, 2, 4)
  int bm, bn;
  int sk;    // split-K factor
};

// norm.hip
// `part` (optional): x is instead the sum of `sk` f32 split-K slabs [sk][rows][dim] of the
// producing GEMM (its deferred reduce fused here)
void launch_rmsnorm(const bf16* x, long x_stride, bf16* residual, const bf16* w, bf16* y,
                    long y_stride, int rows, int dim, float eps, bool add_residual,
                    hipStream_t stream, const float* part = nullptr, int sk = 0);
// launch_rmsnorm over split-K slabs that also routes every normalised row for a MoE layer
// (router_w [E][dim], E = 4 or 8): writes gates [rows][E], topk_ids / topk_w [rows][topk] as
// launch_moe_route would from y. < 0: unsupported.
int launch_rmsnorm_route(const float* part, int sk, bf16* residual, const bf16* w, bf16* y, int rows,
                         int dim, float eps, bool add_residual, const bf16* router_w, int E, int topk,
                         float* gates, int* topk_ids, float* topk_w, hipStream_t stream);
// Row-split add + RMSNorm whose consumer GEMM applies the row scale: writes y = x * w and the
// partial sums of squares ssp[rows][rmsnorm_rows_chunks(dim)]; pass RowScale{ssp, chunks, 1/dim,
// eps} to the GEMM that consumes y.
int rmsnorm_rows_chunks(int dim);
int launch_rmsnorm_rows(const bf16* x, long x_stride, bf16* residual, const bf16* w, bf16* y, float* ssp,
                        int rows, int dim, bool add_residual, hipStream_t stream,
                        const float* part = nullptr, int sk = 0);
void launch_layernorm(const bf16* x, bf16* residual, const bf16* w, const bf16* b, bf16* y,
                      int rows, int dim, float eps, bool add_residual, hipStream_t stream);

// rope.hip
// `part` (optional): the QKV row is the sum of `sk` f32 split-K slabs [sk][T][row] of the
// GEMM (deferred reduce fused here); the bf16 row is written to `qkv` as well
// Caches hold bf16, or FP8 e4m3 when `kv_fp8` (bfly_kv.h).
void launch_rope_kv(bf16* qkv, int T, int Hq, int Hkv, int D, const int* positions,
                    const float* cos_t, const float* sin_t, const int* slots, void* k_cache,
                    void* v_cache, int block_size, hipStream_t stream,
                    const float* part = nullptr, int sk = 0, int kv_fp8 = 0);
void launch_kv_append(const bf16* k, long k_stride, const bf16* v, long v_stride,
                      const int* slots, void* k_cache, void* v_cache, int T, int Hkv, int D,
                      int block_size, hipStream_t stream, int kv_fp8 = 0);

// elementwise.hip
void launch_silu_mul(const bf16* gu, bf16* out, long rows, int ffn, int interleave,
                     hipStream_t stream);
void launch_gelu(const bf16* x, bf16* out, long n, hipStream_t stream);
void launch_add(const bf16* a, const bf16* b, bf16* out, long n, hipStream_t stream);
void launch_init_hash(bf16* out, long rows, int cols, long ld, long grow0, long gcol0, long gcols,
                      uint32_t seed, float amp, hipStream_t stream);
void launch_embed(const int* ids, const bf16* table, bf16* out, int T, int dim, int vstart,
                  int vlocal, hipStream_t stream);
// out[i, :] = src[idx[i], :] over rows of `words` 4-byte words (strides in words); idx < 0 or
// out of range leaves row i untouched
void launch_gather_rows(const void* src, long src_ld, const void* idx, bool idx64, void* out, long out_ld,
                        int words, long rows, long nsrc, hipStream_t stream);

// sample.hip
constexpr int kSampleMaxChunks = 64;
void launch_sample(const bf16* logits, long row_stride, int rows, int V, int vstart,
                   const float* temps, const long* seeds, uint64_t* workspace, int* out_ids,
                   float* out_scores, hipStream_t stream, const float* thresh = nullptr,
                   int check_finite = 0);
// TP merge of per-shard winners: pair [rows][2] f32 (score, id); allp [tp][rows][2] -> ids
void launch_sample_pack(const float* scores, const int* ids, float* pair, int rows, hipStream_t stream);
void launch_sample_merge(const float* allp, int tp, int rows, int* out, hipStream_t stream);
// exact top-k / top-p thresholds by radix select (sample.hip): state [rows, 8] f32 bits,
// smax [rows] int32 (zeroed), hist [rows, 512] f32 (zeroed); see the kernel comment
void launch_tkp_begin(const bf16* logits, long row_stride, int rows, int V, const float* temps,
                      const int* top_k, const float* top_p, float* state, int* smax, hipStream_t stream);
void launch_tkp_pass(const bf16* logits, long row_stride, int rows, int V, const float* temps,
                     float* state, const int* smax, float* hist, int pass, int phase, hipStream_t stream);
void launch_tkp_select(const float* top_p, float* state, float* hist, int rows, int pass, int phase,
                       hipStream_t stream);
void launch_tkp_final(const float* state, int rows, float* thresh, hipStream_t stream);

// gemm.hip
GemmPlan plan_gemm(int M, int N, int K);
size_t gemm_workspace_bytes(int M, int N, int K);
int launch_gemm_plan(const GemmPlan& p, const bf16* X, long ldx, const bf16* W, long ldw, int M,
                     int N, int K, int epi, const bf16* bias, bf16* out, long ldo, float* ws,
                     size_t ws_bytes, hipStream_t stream);
int gemm_check(int M, int N, int K, int epi);
// 0 if the auto plan for this shape takes a RowScale (tile and decode-ring kernels)
int gemm_rowscale_check(int M, int N, int K, int epi);
// Y = X W^T without epilogue; when the plan splits K, the f32 slabs are left in the workspace
// (at gemm_slab_offset_floats(), layout [sk][M][N]) for the consumer kernel to reduce, and the
// split count is returned; otherwise `out` is written and 1 is returned. < 0: error.
int launch_gemm_deferred(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                         bf16* out, long ldo, float* ws, size_t ws_bytes, hipStream_t stream,
                         const RowScale* rs = nullptr);
size_t gemm_slab_offset_floats();
void launch_splitk_reduce(const float* part, int sk, int M, int N, bf16* out, long ldo,
                          hipStream_t stream);
int launch_gemm(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K, int epi,
                const bf16* bias, bf16* out, long ldo, float* ws, size_t ws_bytes,
                hipStream_t stream, const RowScale* rs = nullptr);
// out[M, N/2] = gate-scaled SwiGLU (EPI_SILU_GATE) on the tile kernel without split-K: the
// gate/up GEMM of the dense MoE decode path with moe_gate_scale folded into its epilogue.
// gates [M][gld] f32; output column f belongs to expert ge0 + f / gF.
// Decode GEMM over the K-tile-blocked copy Wp ([N/256][K/64][256][64]) of a weight, with the plan
// the row-major weight would run: < 0 (nothing launched) when that plan is not a 64-row tile plan.
// `rs`: row scale and / or MoE gate (EPI_SILU_GATE). Split-K plans need `ws`; with `defer` their
// slabs stay in it for the consumer (returns the split count), else they are reduced (returns 1).
// `dry`: only report whether it applies (0).
int launch_gemm_packed(const bf16* X, long ldx, const bf16* Wp, int M, int N, int K, int epi, bf16* out,
                       long ldo, hipStream_t stream, const RowScale* rs = nullptr, bool dry = false,
                       float* ws = nullptr, size_t ws_bytes = 0, bool defer = false);
int launch_gemm_silu_gate(const bf16* X, long ldx, const bf16* W, long ldw, int M, int N, int K,
                          bf16* out, long ldo, const float* gates, int gld, int ge0, int gF,
                          hipStream_t stream);

// attention.hip
int attn_decode_splits(int max_ctx, int part_tokens);
int attn_decode_part_tokens(int B, int Hkv, int max_ctx);
int launch_attn_decode(const bf16* q, long q_stride, const void* k_cache, const void* v_cache,
                       const int* block_tables, int bt_stride, const int* ctx_lens, int B, int Hq,
                       int Hkv, int D, int block_size, float scale, int max_ctx, int part_tokens,
                       bf16* out, float* part_o, float* part_ml, hipStream_t stream,
                       int kv_fp8 = 0);            // caches hold FP8 e4m3 (bfly_kv.h)
int launch_attn_prefill(const bf16* q, long q_stride, const bf16* k, long k_stride, const bf16* v,
                        long v_stride, const int* cu_seqlens, int nseq, int max_seqlen, int Hq,
                        int Hkv, int D, float scale, bool causal, bf16* out, long o_stride,
                        hipStream_t stream, const int* cu_k = nullptr,
                        float* lse = nullptr);
// attention_paged.hip — chunked prefill over the paged cache: query rows [cu_q[s], cu_q[s+1])
// of sequence s at positions[row] attend causally to keys [0, positions[row]] read through
// tables[s] (the chunk's own K/V already appended). G = Hq / Hkv <= 8.
int launch_attn_prefill_paged(const bf16* q, long q_stride, const void* k_cache, const void* v_cache,
                              const int* tables, int bt_stride, const int* cu_q, const int* positions,
                              int nseq, int max_q, int Hq, int Hkv, int D, int block_size, float scale,
                              bf16* out, long o_stride, hipStream_t stream, int kv_fp8 = 0);
// K16 (context parallel): acc_o [T, H, 128] f32 / acc_lse [T, H] f32 absorb (o, lse).
int launch_attn_lse_merge(float* acc_o, float* acc_lse, const bf16* o, long o_stride,
                          const float* lse, int T, int H, int D, hipStream_t stream);

// allreduce.hip — one-shot IPC all-reduce (+ fused residual add / RMSNorm)
constexpr int kArBlocks = 128;
constexpr int kArMaxWorld = 8;
constexpr long kArDataOff = 65536;
// herr: this process's host-mapped health words (health_words_device()); a flag wait that
// times out also stores 1 into herr[kHealthCar] / herr[kHealthEp], which the host error
// poller reads without any HIP call (so it sees a stuck peer while the stream is still busy)
struct ArPeers { char* base[kArMaxWorld]; uint32_t* herr; };
constexpr int kHealthCar = 0, kHealthEp = 1, kHealthWords = 16;
uint32_t* health_words_device();        // lazily allocated pinned, mapped, coherent host memory
uint32_t health_word(int i);            // host read (no HIP call once allocated)
void health_clear(int word = -1);   // one word (kHealthCar / kHealthEp) or, -1, all of them
// flags/counters, two input buffers and two reduced-chunk buffers (two-shot), all double-buffered
inline long car_buffer_bytes(long cap) { return kArDataOff + 4 * cap; }
// `slabs` (optional): the input is split-K partials [sk][rows][dim] f32, reduced in the publish.
// `blocks`: the grid (<= kArBlocks), the same on every rank and for every call of a communicator:
// kArBlocks on a node (one rank per GPU); kArBlocks / world for ranks that share one GPU (tests),
// so the waves of ranks that arrived first and spin on their peers' flags can never occupy every
// CU — a late rank's one-workgroup-per-CU GEMM must still find CUs to run on.
int launch_custom_allreduce(const bf16* in, bf16* out, bf16* residual, const bf16* w, float eps,
                            int rows, int dim, const ArPeers& peers, int world, int rank,
                            long cap, hipStream_t stream, const float* slabs = nullptr, int sk = 0,
                            bool two_shot = false, int blocks = kArBlocks);
void* car_alloc(size_t bytes);
void car_free(void* p);
int car_ipc_handle(void* p, unsigned char* out64);
void* car_ipc_open(const unsigned char* h64);
void car_ipc_close(void* p);
int car_clear_error(void* base);
int car_error(const void* base);

// ep_ipc.hip — byte-minimal EP dispatch / return over peer IPC buffers (decode MoE)
constexpr long kEpHeaderBytes = 65536;
struct EpLayout { long x, ids, w, back, total; };   // byte offsets in a rank's buffer
EpLayout ep_ipc_layout(int ep, int capmax, int H, int K);
int launch_ep_ipc_dispatch(const bf16* x, const int* ids, const float* w, const int* slots, int T, int K,
                           int H, int El, int ep, int capmax, const ArPeers& peers, int rank, int* slot_out,
                           hipStream_t stream);
int launch_ep_ipc_wait(const ArPeers& peers, int ep, int rank, hipStream_t stream);
int launch_ep_ipc_return(const bf16* y, int H, int K, int ep, int capmax, const ArPeers& peers, int rank,
                         hipStream_t stream);
int launch_ep_ipc_combine(const int* slot, int T, int H, int K, int ep, int capmax, const ArPeers& peers,
                          int rank, bf16* out, hipStream_t stream);
// Prefill-sized dispatch (any T <= capmax): a one-workgroup scan routes the tokens (slot_out,
// per-destination totals), then one workgroup per token stores its row once into each owning
// rank's block; the last arriver publishes the row counts and raises the dispatch flags. The
// receive blocks are not marked row by row: consumers bound each block by its count
// (ep_ipc_counts_offset / launch_moe_align bcnt).
int launch_ep_ipc_dispatch_prefill(const bf16* x, const int* ids, const float* w, int T, int K, int H, int El,
                                   int ep, int capmax, const ArPeers& peers, int rank, int* slot_out,
                                   hipStream_t stream);
long ep_ipc_counts_offset();
int ep_ipc_stats(const void* base, long long* out2);
int ep_ipc_error(const void* base);

// moe.hip
int launch_moe_route(const bf16* x, long x_stride, const bf16* wr, int T, int H, int E, int K,
                     float* gates, int* topk_ids, float* topk_w, hipStream_t stream);
void launch_moe_gate_scale(bf16* h, const float* gates, long T, int E, int e0, int El, int F,
                           hipStream_t stream);

// sparse MoE (moe.hip + gemm.hip grouped tiles)
int moe_max_tiles(int TK, int El, int BM);
// bcnt / bcap (optional): rows are blocks of bcap rows, of which the first bcnt[block] are
// valid (EP IPC receive buffer): other rows get no slot and no combined output
int launch_moe_align(const int* topk_ids, int T, int K, int e0, int El, int BM, int* rows,
                     int* slot_of, int4* tiles, int* count, hipStream_t stream,
                     const int* bcnt = nullptr, int bcap = 0);
int launch_moe_combine(const bf16* y, const int* slot_of, const float* w, int T, int K, int H,
                       bf16* out, hipStream_t stream, const int* bcnt = nullptr, int bcap = 0);
constexpr int kMoeGroupBM = 64;
int launch_gemm_grouped(const bf16* X, long ldx, const bf16* W, long ldw, long w_estride, int N,
                        int K, int epi, const int* rows, const int4* tiles, const int* count,
                        int max_tiles, bf16* out, long ldo, hipStream_t stream, int bm = 64,
                        int slots = 0, int sk = 1, float* part = nullptr);
int launch_ep_pack(const bf16* x, const int* ids, const float* w, const int* slots, int T, int K, int H,
                   int El, int ep, int cap, bf16* send, float* meta, int* slot, hipStream_t stream);
int launch_ep_combine(const bf16* back, const int* slot, int T, int H, int ep, bf16* out, hipStream_t stream);
int launch_moe_combine_slabs(const float* part, int sk, long slab, const int* slot_of, const float* w,
                             int T, int K, int H, bf16* out, hipStream_t stream,
                             const int* bcnt = nullptr, int bcap = 0);

// probe.hip
void launch_probe(int which, float* out, hipStream_t stream);

}  // namespace bfly
