// Host-side launch API of the gfx950 kernels. Every launcher is capture-safe (no
// allocation, no synchronisation) so decode steps can be recorded into hipGraphs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nga {

// Kernel-form selection for A/B runs and tests. Each form starts from its NGA_* environment
// variable, read ONCE (first use); launchers read the table, never the environment, and
// tests / benchmarks switch forms explicitly through ops.kernel_forms (no per-launch getenv).
enum KernelForm {
  KF_DECODE_DMA = 0,   // NGA_DECODE_DMA: 2 ring form of the LDS-DMA decode kernel (default), 1 its whole-page form, 0 register kernel
  KF_DECODE_NT,        // NGA_DECODE_NT: register decode kernel's KV loads nt: 1 always, 2 bf16 pages only (default), 0 never
  KF_SEARCH_DMA,       // NGA_SEARCH_DMA: 0 forces the register form of the fused search kernel
  KF_PREFILL_V1,       // NGA_PREFILL_V1: 1 disables the 32x32 prefill kernel
  KF_PREFILL_KS,       // NGA_PREFILL_KS: 1 / 2 forces the 32x32 prefill kernel's wave-group count
  KF_ROPE_VNT,         // NGA_ROPE_VNT: non-temporal 2-byte V^T page stores in the RoPE / KV-write kernels: 1 all, 2 tokens with no same-page neighbour
  KF_DECODE_DMA_AUX,   // NGA_DECODE_DMA_AUX: cache policy of the LDS-DMA decode kernel's KV loads: 2 nt (default), 0 default policy
  KF_COUNT
};
int kernel_form(KernelForm f);
void set_kernel_form(KernelForm f, int value);
const char* kernel_form_name(KernelForm f);


// norm.hip
void launch_rmsnorm(uint16_t* out, uint16_t* resid, const uint16_t* delta, const uint16_t* w,
                    float eps, int64_t rows, int H, int64_t in_stride, int64_t out_stride,
                    hipStream_t stream);
void launch_layernorm(uint16_t* out, const uint16_t* x, const uint16_t* resid, const uint16_t* g,
                      const uint16_t* b, float eps, int64_t rows, int H, hipStream_t stream);
// resid += delta (stored); out = LN(resid) * g + b
void launch_add_layernorm(uint16_t* out, uint16_t* resid, const uint16_t* delta, const uint16_t* g,
                          const uint16_t* b, float eps, int64_t rows, int H, hipStream_t stream);

// activation.hip
void launch_silu_mul(uint16_t* out, const uint16_t* in, int64_t T, int F, hipStream_t stream);
void launch_gelu_tanh_mul(uint16_t* out, const uint16_t* in, int64_t T, int F, hipStream_t stream);
// mode 0: erf GELU, 1: tanh GELU, 2: quick_gelu (x * sigmoid(1.702 x))
void launch_bias_gelu(uint16_t* x, const uint16_t* bias, int64_t T, int F, int mode,
                      hipStream_t stream);

// rope.hip
// kc / vc: bf16 caches, or fp8 e4m3fn ones (kv_fp8) storing k * inv_ks and v * inv_vs.
// part: optional fp32 K-split partial slabs [S, T, row] of the qkv projection; their bf16 sum is
// rotated / copied into qkv (which is then output only)
void launch_rope_cache(uint16_t* qkv, const int32_t* pos, const float* cos_sin,
                       const int32_t* slots, void* kc, void* vc, int64_t T, int Hq,
                       int Hkv, int D, int BS, bool kv_fp8, float inv_ks, float inv_vs,
                       hipStream_t stream, const float* part = nullptr, int S = 0);

// attention_decode.hip
int decode_attn_pages_per_part(int num_seqs, int Hkv, int max_ctx);
// kc / vc: bf16, or fp8 e4m3fn holding k / k_scale and v / v_scale (kv_fp8)
void launch_decode_attention(uint16_t* out, int64_t out_stride, const uint16_t* q,
                             int64_t q_stride, const void* kc, const void* vc,
                             const int32_t* block_tables, int max_blocks, const int32_t* ctx_lens,
                             int num_seqs, int Hq, int Hkv, int D, int max_ctx, float scale,
                             int pages_per_part, float* part_ml, float* part_o, int window,
                             bool kv_fp8, float k_scale, float v_scale, hipStream_t stream,
                             bool skip_empty = false);

// attention_prefill.hip
struct PrefillParams {
  uint16_t* out;
  int64_t out_stride;
  const uint16_t* q;
  int64_t q_stride;
  const uint16_t* k;  // non-paged K rows (packed like q)
  const uint16_t* v;
  int64_t kv_stride;
  const uint16_t* kc;  // paged caches
  const uint16_t* vc;
  const int32_t* block_tables;
  int max_blocks;
  const int32_t* cu_q;      // [B+1] offsets of each sequence's query rows
  const int32_t* ctx_lens;  // [B] total keys (paged)
  int Hq;
  int Hkv;
  float scale;
  int ntiles;  // query tiles per (sequence, head) — set by the launcher
  int per_xcd; // workgroups per XCD slice of the 1-D grid — set by the launcher
  int total;   // ntiles * Hq * num_seqs — set by the launcher
  int window;  // > 0: sliding-window causal attention (query i sees keys (i - window, i])
  int impl;    // 0: pick by size, 1: the 16x16 kernel, 2: the 32x32 kernel where it applies
  int kv_fp8;      // paged caches hold fp8 e4m3fn (k / k_scale, v / v_scale); 16x16 kernel only
  float v_scale;   // output multiplier (fp8 caches; `scale` already includes k_scale)
  // work-list mode of the 32x32 kernel (nullptr: enumerated grid): [n, 2] (sequence, row
  // block) pairs, and the device count n
  const int32_t* items;
  const int32_t* n_items;
};
void launch_prefill_attention(const PrefillParams& p, int num_seqs, int max_q_len, int D,
                              bool paged, bool causal, hipStream_t stream);
// 32x32-MFMA prefill (paged, head_dim 128); returns false when it does not take the call
bool launch_prefill_attention_v2(const PrefillParams& p, int num_seqs, int max_q_len, int D,
                                 bool paged, bool causal, hipStream_t stream);
// work-list launch (p.items / p.n_items set): a fixed grid of `grid` workgroups; ks = wave
// groups (1 or 2). Rows per row block: 32 * 4 / hpw with hpw = 4, 2, 1 for Hq/Hkv % 4, % 2, else.
void launch_prefill_attention_v2_worklist(const PrefillParams& p, int grid, int ks, bool causal,
                                          hipStream_t stream);
// work-list launch of the 16x16 kernel (paged, head_dim 64 / 128 / 256, bf16 or fp8 pages):
// items are (sequence, 64-row tile) pairs, q head = item index % Hq
void launch_prefill_attention_v1_worklist(const PrefillParams& p, int grid, int D, bool causal,
                                          hipStream_t stream);

// sampling.hip
void launch_sample(float* logits, int B, int V, const float* temperature, const int32_t* top_k,
                   const float* top_p, const float* rep_penalty, const int32_t* history,
                   int hist_len, const int64_t* seeds, const int64_t* steps, int32_t* out_tok,
                   float* out_logprob, hipStream_t stream);

// vector_search.hip
void launch_score(const uint16_t* Q, int nq, const uint16_t* X, int64_t N, int D,
                  const float* row_bias, float* S, float dot_scale, hipStream_t stream);
// fused score + per-block top-k over work items (row range + <= 64 query slots); candidates
// out [n_items * 64, nblk, k]; k <= score_topk_kmax(max_q_per_item)
int score_topk_kmax(int nq_per_item);
// 1 if launch_score_topk takes the LDS-DMA form (one workgroup per CU: size nblk to the CUs)
int score_topk_dma_ok(int D, int max_q_per_item);
void launch_score_topk(const uint16_t* Q, int nq, const uint16_t* X, int64_t N, int D,
                       const float* row_bias, float dot_scale, const int64_t* row_beg,
                       const int64_t* row_end, const int32_t* qtab, const int32_t* slot_rows, int n_items,
                       int max_q_per_item, int nblk, int k, float* out_v, int64_t* out_r, hipStream_t stream);
constexpr int IVF_PLAN_MAX_LISTS = 16384;
void launch_ivf_plan(const int64_t* probes, int nq, int nprobe, int nlist, int32_t* qtab,
                     int32_t* slot_rows, hipStream_t stream);
void launch_topk(const float* in, const int64_t* in_idx, int64_t rows, int64_t row_len,
                 int64_t seg_len, int k, float* out_v, int64_t* out_i, hipStream_t stream);

// embedding.hip: rows of this rank's vocabulary shard [vocab_lo, vocab_lo + rows), zeros
// for ids outside it; H % 8 == 0
void launch_embedding(uint16_t* out, const uint16_t* table, const int32_t* ids, int T, int H, int64_t vocab_lo,
                      int64_t rows, float scale, hipStream_t stream);

// pool.hip
void launch_pool_l2norm(const uint16_t* hidden, const int32_t* cu, int B, int H, int mode,
                        int normalize, float* out, hipStream_t stream);
void launch_row_sqnorm(const uint16_t* X, int64_t N, int D, float* out, hipStream_t stream);

// dsp.hip (complex64 passed as interleaved float pairs)
constexpr int kFirMaxTaps = 1024;
void launch_fir_c64(const float* x, int n, const float* taps, int ntaps, const float* hist, float* y,
                    hipStream_t stream);
void launch_fm_demod(const float* x, int n, float prev_re, float prev_im, int has_prev, float* y,
                     hipStream_t stream);
void launch_resample_pcm(const float* x, int n, const float* h, int nh, int down, int pre, int nout,
                         float gain, float* yf, int16_t* yi, hipStream_t stream);
void launch_quant_fp8_rows(const uint16_t* x, int64_t ldx, int64_t rows, int H, int mode, uint8_t* y,
                           float* scale, hipStream_t stream);

// moe.hip (sparse MoE MLP)
struct MoeGemmParams {
  const uint16_t* A;         // MODE 0: token rows x [T, K] (gathered); MODE 1: [M, K] sorted rows
  int64_t lda;
  const uint16_t* W;         // [E, w_rows, K] expert weights
  int64_t w_rows;            // rows per expert (2F for gate|up, N for down)
  int K;
  int F;                     // MODE 0: features (up rows start at F)
  int mt;                    // M tiles (table entries)
  int nt;                    // N blocks: F / 128 (MODE 0) or N / 256 (MODE 1)
  const int32_t* sorted_tok;
  const float* sorted_w;
  const int32_t* tiles;      // [mt, 3]: expert, first row, end row (expert -1: unused)
  uint16_t* out;
  int64_t ldo;
  int act;                   // MODE 0: 0 silu, 1 gelu_tanh
};
void launch_moe_route(const uint16_t* logits, int64_t ld, int T, int E, int k, int32_t* ids,
                      float* w, hipStream_t stream);
void launch_moe_align(const int32_t* ids, const float* w, int M, int k, int e0, int E, int bm,
                      int32_t* sorted_tok, float* sorted_w, int32_t* inv, int32_t* tiles,
                      int mt_cap, hipStream_t stream);
void launch_moe_gemm(const MoeGemmParams& p, int bm, int mode, hipStream_t stream);
void launch_moe_combine(const uint16_t* y, const int32_t* inv, int T, int k, int H, uint16_t* out,
                        hipStream_t stream);

// gemm_skinny.hip (decode-shape projection GEMM, out = x . W^T)
struct GemvParams {
  const uint16_t* x;   // [M, K] rows, stride ldx (16-B aligned)
  int64_t ldx;
  const uint16_t* w;   // [N, K] (epi 2: [2N, K] = [gate | up])
  int M, N, K;         // M <= 4; K % 8 == 0, M * K * 2 <= 160 KiB
  void* out;           // epi 0 / 2: bf16 [M, ldo]; epi 1: fp32 [M, ldo]
  int64_t ldo;
};
// out = x . W^T for M <= 4 rows (gemv.hip); false if the shape is out of range
bool launch_gemv(const GemvParams& p, int epi, hipStream_t stream);

struct SkinnyGemmParams {
  const uint16_t* x;   // [M, K] rows, stride ldx (16-B aligned)
  int64_t ldx;
  const uint16_t* w;   // [rows, K] contiguous (epi 2: [2N, K] = [gate | up])
  int M, N, K;         // N: output features; K % 64 == 0
  int split;           // K slices (epi 1 only may exceed 1)
  void* out;           // epi 0 / 2: bf16 [M, ldo]; epi 1: fp32 [split, M, N]
  int64_t ldo;
  int nN, nM;          // weight-row blocks, token-row tiles (set by the caller from the cfg)
  int krot;            // 1: each block starts its K walk at a block-dependent step
  int wpack;           // 1: w is tile-packed [nN][K/64][BN][64] for this cfg's BN (pack_weight)
  int xpack;           // 1: x is tile-packed [nM][K/64][BM][64] for this cfg's BM (pack_rows)
};
// scatter of packed step inputs (staging.hip): segment s = bytes [off, off + bytes) of the
// device staging buffer -> dst (16-B aligned offsets / destinations, bytes % 4 == 0)
constexpr int kMaxSegments = 32;
struct SegmentTable {
  int n;
  int64_t dst[kMaxSegments];
  int64_t off[kMaxSegments];
  int64_t bytes[kMaxSegments];
};
void launch_scatter_segments(const uint8_t* src, const SegmentTable& t, hipStream_t stream);

int skinny_gemm_cfg_count();
void launch_region_marker(int end, int* sink, hipStream_t stream);
void skinny_gemm_cfg_info(int cfg, int* info);   // {BN, BM, WN, WM, NSTAGE, BK}
void launch_skinny_gemm(const SkinnyGemmParams& p, int cfg, int epi, hipStream_t stream);
void launch_splitk_swiglu(const float* P, int S, int M, int F, uint16_t* out, int64_t ldo,
                          hipStream_t stream);
void launch_splitk_reduce(const float* P, int S, int M, int N, uint16_t* out, int64_t ldo,
                          hipStream_t stream);
void launch_splitk_add_rmsnorm(const float* P, int S, int M, uint16_t* resid, const uint16_t* w,
                               float eps, int H, uint16_t* out, hipStream_t stream);

}  // namespace nga
