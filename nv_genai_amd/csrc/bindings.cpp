// PyTorch bindings for the gfx950 kernels (nv_genai_amd._C).
// Every entry point validates dtype / device / shape / contiguity against what its kernel
// and launch grid assume before launching (a malformed launch on the GPU box can fault the
// device), and launches on PyTorch's current HIP stream so calls are hipGraph-capturable.
#include <atomic>
#include <torch/extension.h>

#include <cstdlib>
#include <functional>
#include <c10/hip/HIPStream.h>

#include "kernels/custom_ar.h"
#include "kernels/kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

#define CHECK_DEV(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, dt) TORCH_CHECK((x).scalar_type() == (dt), #x " must be " #dt)
#define CHECK_BF16(x) \
  CHECK_DEV(x);       \
  CHECK_DT(x, at::kBFloat16)

uint16_t* bfp(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

// paged KV caches: bf16, or fp8 e4m3fn (returns true); both caches must agree
bool kv_is_fp8(const Tensor& kc, const Tensor& vc) {
  TORCH_CHECK(kc.scalar_type() == vc.scalar_type(), "k and v caches must have the same dtype");
  TORCH_CHECK(kc.scalar_type() == at::kBFloat16 || kc.scalar_type() == at::kFloat8_e4m3fn,
              "KV caches must be bfloat16 or float8_e4m3fn");
  TORCH_CHECK(kc.is_cuda() && vc.is_cuda(), "KV caches must be on the GPU");
  return kc.scalar_type() == at::kFloat8_e4m3fn;
}
const uint16_t* cbfp(const c10::optional<Tensor>& t) {
  return t.has_value() ? reinterpret_cast<const uint16_t*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------------ norms / activations
void rmsnorm(Tensor out, Tensor x, Tensor w, double eps) {
  CHECK_BF16(out); CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "rmsnorm expects 2-D [rows, H]");
  const int H = (int)x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "rmsnorm: H must be a multiple of 8 and <= 8192");
  TORCH_CHECK(x.stride(1) == 1 && out.stride(1) == 1 && w.numel() == H && w.is_contiguous());
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == H);
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "rmsnorm: row strides must be 16-B aligned");
  nga::launch_rmsnorm(bfp(out), bfp(x), nullptr, bfp(w), (float)eps, x.size(0), H, x.stride(0),
                      out.stride(0), cur_stream(x));
}

// resid += delta; out = rmsnorm(resid) * w
void add_rmsnorm(Tensor out, Tensor resid, Tensor delta, Tensor w, double eps) {
  CHECK_BF16(out); CHECK_BF16(resid); CHECK_BF16(delta); CHECK_BF16(w);
  CHECK_CONTIG(resid); CHECK_CONTIG(delta); CHECK_CONTIG(out);
  TORCH_CHECK(resid.dim() == 2 && resid.sizes() == delta.sizes() && resid.sizes() == out.sizes());
  const int H = (int)resid.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192 && w.numel() == H);
  nga::launch_rmsnorm(bfp(out), bfp(resid), bfp(delta), bfp(w), (float)eps, resid.size(0), H, H, H,
                      cur_stream(resid));
}

void layernorm(Tensor out, Tensor x, c10::optional<Tensor> resid, Tensor g, Tensor b, double eps) {
  CHECK_BF16(out); CHECK_BF16(x); CHECK_BF16(g); CHECK_BF16(b);
  CHECK_CONTIG(out); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && out.sizes() == x.sizes());
  const int H = (int)x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192 && g.numel() == H && b.numel() == H);
  if (resid.has_value()) {
    CHECK_BF16(*resid); CHECK_CONTIG(*resid);
    TORCH_CHECK(resid->sizes() == x.sizes());
  }
  nga::launch_layernorm(bfp(out), bfp(x), cbfp(resid), bfp(g), bfp(b), (float)eps, x.size(0), H,
                        cur_stream(x));
}

// resid += delta; out = LayerNorm(resid) * g + b
void add_layernorm(Tensor out, Tensor resid, Tensor delta, Tensor g, Tensor b, double eps) {
  CHECK_BF16(out); CHECK_BF16(resid); CHECK_BF16(delta); CHECK_BF16(g); CHECK_BF16(b);
  CHECK_CONTIG(out); CHECK_CONTIG(resid); CHECK_CONTIG(delta);
  TORCH_CHECK(resid.dim() == 2 && resid.sizes() == delta.sizes() && resid.sizes() == out.sizes());
  const int H = (int)resid.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192 && g.numel() == H && b.numel() == H);
  nga::launch_add_layernorm(bfp(out), bfp(resid), bfp(delta), bfp(g), bfp(b), (float)eps,
                            resid.size(0), H, cur_stream(resid));
}

void gelu_tanh_mul(Tensor out, Tensor x) {
  CHECK_BF16(out); CHECK_BF16(x); CHECK_CONTIG(out); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(1) == 2 * out.size(1) && x.size(0) == out.size(0));
  TORCH_CHECK(out.size(1) % 8 == 0);
  nga::launch_gelu_tanh_mul(bfp(out), bfp(x), x.size(0), (int)out.size(1), cur_stream(x));
}

void silu_mul(Tensor out, Tensor x) {
  CHECK_BF16(out); CHECK_BF16(x); CHECK_CONTIG(out); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(1) == 2 * out.size(1) && x.size(0) == out.size(0));
  TORCH_CHECK(out.size(1) % 8 == 0);
  nga::launch_silu_mul(bfp(out), bfp(x), x.size(0), (int)out.size(1), cur_stream(x));
}

void bias_gelu(Tensor x, c10::optional<Tensor> bias, int64_t mode) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "bias_gelu: mode 0 (erf), 1 (tanh) or 2 (quick)");
  CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 8 == 0);
  if (bias.has_value()) {
    CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == x.size(1));
  }
  nga::launch_bias_gelu(bfp(x), cbfp(bias), x.size(0), (int)x.size(1), (int)mode, cur_stream(x));
}

// ------------------------------------------------------------------ rope + kv cache
void rope_cache(Tensor qkv, Tensor pos, Tensor cos_sin, c10::optional<Tensor> slots,
                c10::optional<Tensor> kc, c10::optional<Tensor> vc, int64_t Hq, int64_t Hkv,
                int64_t D, double k_scale, double v_scale, c10::optional<Tensor> part) {
  CHECK_BF16(qkv); CHECK_CONTIG(qkv);
  CHECK_DEV(pos); CHECK_DT(pos, at::kInt);
  CHECK_DEV(cos_sin); CHECK_DT(cos_sin, at::kFloat); CHECK_CONTIG(cos_sin);
  TORCH_CHECK(D == 128 || D == 64 || D == 256, "rope_cache: head_dim must be 64, 128 or 256");
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) == (Hq + 2 * Hkv) * D, "rope_cache: qkv must be [T, (Hq+2Hkv)*D]");
  TORCH_CHECK(pos.numel() == qkv.size(0));
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D);
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "rope_cache: KV scales must be positive");
  int BS = 64;
  const int32_t* sp = nullptr;
  void *kp = nullptr, *vp = nullptr;
  bool fp8 = false;
  if (slots.has_value()) {
    TORCH_CHECK(kc.has_value() && vc.has_value());
    CHECK_DEV(*slots); CHECK_DT(*slots, at::kInt);
    TORCH_CHECK(slots->numel() == qkv.size(0));
    fp8 = kv_is_fp8(*kc, *vc);
    CHECK_CONTIG(*kc); CHECK_CONTIG(*vc);
    TORCH_CHECK(kc->dim() == 4 && kc->size(1) == Hkv && kc->size(3) == D, "k cache must be [nb, Hkv, BS, D]");
    TORCH_CHECK(vc->dim() == 4 && vc->size(1) == Hkv && vc->size(2) == D, "v cache must be [nb, Hkv, D, BS]");
    BS = (int)kc->size(2);
    TORCH_CHECK(vc->size(3) == BS && kc->size(0) == vc->size(0));
    sp = slots->data_ptr<int32_t>();
    kp = kc->data_ptr();
    vp = vc->data_ptr();
  }
  const float* pp = nullptr;
  int S = 0;
  if (part.has_value()) {
    CHECK_DEV(*part); CHECK_DT(*part, at::kFloat); CHECK_CONTIG(*part);
    TORCH_CHECK(part->dim() == 3 && part->size(1) == qkv.size(0) && part->size(2) == qkv.size(1),
                "rope_cache: partial slabs must be [S, T, (Hq+2Hkv)*D]");
    pp = part->data_ptr<float>();
    S = (int)part->size(0);
  }
  nga::launch_rope_cache(bfp(qkv), pos.data_ptr<int32_t>(), cos_sin.data_ptr<float>(), sp, kp, vp,
                         qkv.size(0), (int)Hq, (int)Hkv, (int)D, BS, fp8, (float)(1.0 / k_scale),
                         (float)(1.0 / v_scale), cur_stream(qkv), pp, S);
}

// ------------------------------------------------------------------ MoE
void moe_route(Tensor logits, int64_t k, Tensor ids, Tensor w) {
  CHECK_BF16(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "moe_route: logits must be [T, E]");
  const int64_t T = logits.size(0), E = logits.size(1);
  TORCH_CHECK(E >= 1 && E <= 64 && k >= 1 && k <= 8 && k <= E, "moe_route: 1 <= k <= min(8, E), E <= 64");
  CHECK_DEV(ids); CHECK_DT(ids, at::kInt); CHECK_DEV(w); CHECK_DT(w, at::kFloat);
  TORCH_CHECK(ids.numel() >= T * k && w.numel() >= T * k);
  nga::launch_moe_route(bfp(logits), logits.stride(0), (int)T, (int)E, (int)k,
                        ids.data_ptr<int32_t>(), w.data_ptr<float>(), cur_stream(logits));
}

void moe_align(Tensor ids, Tensor w, int64_t T, int64_t k, int64_t e0, int64_t E, int64_t bm,
               Tensor sorted_tok, Tensor sorted_w, Tensor inv, Tensor tiles, int64_t mt_cap) {
  const int64_t M = T * k;
  CHECK_DEV(ids); CHECK_DT(ids, at::kInt);
  CHECK_DEV(w); CHECK_DT(w, at::kFloat);
  CHECK_DEV(sorted_tok); CHECK_DT(sorted_tok, at::kInt);
  CHECK_DEV(sorted_w); CHECK_DT(sorted_w, at::kFloat);
  CHECK_DEV(inv); CHECK_DT(inv, at::kInt);
  CHECK_DEV(tiles); CHECK_DT(tiles, at::kInt);
  TORCH_CHECK(E >= 1 && E <= 64 && (bm == 64 || bm == 128) && e0 >= 0);
  TORCH_CHECK(ids.numel() >= M && w.numel() >= M && sorted_tok.numel() >= M &&
              sorted_w.numel() >= M && inv.numel() >= M && tiles.numel() >= 3 * mt_cap);
  // every expert's rows fit the table: sum_e ceil(cnt_e / bm) <= M / bm + E
  TORCH_CHECK(mt_cap >= (M + bm - 1) / bm + E, "moe_align: M-tile table too small");
  TORCH_CHECK(k >= 1 && k <= 8);
  nga::launch_moe_align(ids.data_ptr<int32_t>(), w.data_ptr<float>(), (int)M, (int)k, (int)e0, (int)E,
                        (int)bm, sorted_tok.data_ptr<int32_t>(), sorted_w.data_ptr<float>(),
                        inv.data_ptr<int32_t>(), tiles.data_ptr<int32_t>(), (int)mt_cap,
                        cur_stream(ids));
}

// mode 0: out [M, F] = act(A[sorted_tok] @ W_e[:F]^T) * (A[sorted_tok] @ W_e[F:]^T)
// mode 1: out [M, N] = (A @ W_e^T) * sorted_w
void moe_gemm(Tensor A, Tensor W, Tensor sorted_tok, Tensor sorted_w, Tensor tiles, int64_t mt,
              int64_t bm, Tensor out, int64_t mode, int64_t act) {
  CHECK_BF16(A); CHECK_BF16(W); CHECK_BF16(out);
  CHECK_CONTIG(W); CHECK_CONTIG(out);
  CHECK_DEV(sorted_tok); CHECK_DT(sorted_tok, at::kInt);
  CHECK_DEV(sorted_w); CHECK_DT(sorted_w, at::kFloat);
  CHECK_DEV(tiles); CHECK_DT(tiles, at::kInt);
  TORCH_CHECK(mode == 0 || mode == 1);
  TORCH_CHECK(bm == 64 || bm == 128);
  TORCH_CHECK(W.dim() == 3 && A.dim() == 2 && out.dim() == 2 && A.stride(1) == 1);
  const int64_t K = W.size(2);
  TORCH_CHECK(A.size(1) == K && K % 64 == 0 && A.stride(0) % 8 == 0, "moe_gemm: K must match and be a multiple of 64");
  TORCH_CHECK(tiles.numel() >= 3 * mt);
  nga::MoeGemmParams p{};
  p.A = bfp(A);
  p.lda = A.stride(0);
  p.W = bfp(W);
  p.w_rows = W.size(1);
  p.K = (int)K;
  p.mt = (int)mt;
  if (mode == 0) {
    TORCH_CHECK(W.size(1) % 256 == 0, "moe_gemm: 2F must be a multiple of 256");
    p.F = (int)(W.size(1) / 2);
    TORCH_CHECK(out.size(1) == p.F, "moe_gemm: out must be [M, F]");
    p.nt = p.F / 128;
  } else {
    TORCH_CHECK(W.size(1) % 256 == 0 && out.size(1) == W.size(1), "moe_gemm: out must be [M, N], N % 256 == 0");
    p.F = 0;
    p.nt = (int)(W.size(1) / 256);
  }
  TORCH_CHECK(sorted_tok.numel() >= out.size(0) && sorted_w.numel() >= out.size(0));
  TORCH_CHECK(mode == 1 || A.size(0) >= 1);
  // rows addressed by the table are < out.size(0) (moe_align writes positions < M = out rows)
  p.sorted_tok = sorted_tok.data_ptr<int32_t>();
  p.sorted_w = sorted_w.data_ptr<float>();
  p.tiles = tiles.data_ptr<int32_t>();
  p.out = bfp(out);
  p.ldo = out.stride(0);
  p.act = (int)act;
  nga::launch_moe_gemm(p, (int)bm, (int)mode, cur_stream(out));
}

void moe_combine(Tensor y, Tensor inv, int64_t T, int64_t k, Tensor out) {
  CHECK_BF16(y); CHECK_BF16(out); CHECK_CONTIG(y); CHECK_CONTIG(out);
  CHECK_DEV(inv); CHECK_DT(inv, at::kInt);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == T && y.dim() == 2 && y.size(1) == out.size(1));
  TORCH_CHECK(out.size(1) % 8 == 0 && inv.numel() >= T * k && y.size(0) >= T * k);
  nga::launch_moe_combine(bfp(y), inv.data_ptr<int32_t>(), (int)T, (int)k, (int)out.size(1),
                          bfp(out), cur_stream(y));
}

// ------------------------------------------------------------------ decode-shape GEMM
std::vector<int64_t> skinny_cfg(int64_t cfg) {   // {BN, BM, WN, WM, NSTAGE, BK}
  int info[6];
  nga::skinny_gemm_cfg_info((int)cfg, info);
  return {info[0], info[1], info[2], info[3], info[4], info[5]};
}

// epi 0: out [M, N] bf16 = x @ w^T; 1: out fp32 [split, M, N] partial slabs; 2: out [M, F] bf16 =
// silu(x @ w[:F]^T) * (x @ w[F:]^T)
// wpack: w is the pack_weight() image for this cfg ([nN * K/64 * BN, 64] rows); n_out: the
// output features then (the packed tensor no longer carries them)
// xpack > 0: x is the pack_rows() image for this cfg and xpack the real token rows M
void skinny_gemm(Tensor out, Tensor x, Tensor w, int64_t epi, int64_t split, int64_t cfg, int64_t krot,
                 int64_t wpack, int64_t n_out, int64_t xpack, int64_t k_in) {
  CHECK_BF16(x); CHECK_BF16(w); CHECK_DEV(out);
  CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() >= 2, "skinny_gemm: 2-D x / w");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0, "skinny_gemm: x rows must be contiguous and 16-B aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "skinny_gemm: x / w must be 16-B aligned");
  const int64_t M = xpack ? xpack : x.size(0), K = xpack ? k_in : x.size(1);
  TORCH_CHECK(K % 64 == 0 && K >= 64, "skinny_gemm: K must be a multiple of 64");
  TORCH_CHECK(wpack || w.size(1) == K, "skinny_gemm: K must match");
  TORCH_CHECK(M >= 1 && M <= 65536, "skinny_gemm: 1 <= M <= 65536");
  int info[6];
  nga::skinny_gemm_cfg_info((int)cfg, info);
  TORCH_CHECK(info[0] > 0, "skinny_gemm: unknown tile configuration ", cfg);
  TORCH_CHECK(info[5] == 64 || (!wpack && !xpack), "skinny_gemm: packed operands are 64-deep tiles (BK 64 configurations only)");
  const int BN = info[0], BM = info[1];
  TORCH_CHECK(epi >= 0 && epi <= 2, "skinny_gemm: epi 0, 1 or 2");
  TORCH_CHECK(split >= 1 && split <= K / 64 && (epi == 1 || split == 1), "skinny_gemm: 1 <= split <= K / 64 (> 1 only for epi 1)");
  nga::SkinnyGemmParams p{};
  p.x = bfp(x);
  p.ldx = x.stride(0);
  p.w = bfp(w);
  p.M = (int)M;
  p.K = (int)K;
  p.split = (int)split;
  p.krot = krot ? 1 : 0;
  p.wpack = wpack ? 1 : 0;
  p.xpack = xpack ? 1 : 0;
  if (xpack) {
    const int64_t nm = (M + info[1] - 1) / info[1];
    TORCH_CHECK(x.size(1) == 64 && x.size(0) == nm * (K / 64) * info[1],
                "skinny_gemm: packed x must be [nM * K/64 * BM, 64] for this cfg");
  }
  const int64_t wrows = wpack ? (epi == 2 ? 2 * n_out : n_out) : w.size(0);
  if (epi == 2) {
    TORCH_CHECK(wrows % 2 == 0, "skinny_gemm: SwiGLU weights are [gate | up] rows");
    p.N = (int)(wrows / 2);
    TORCH_CHECK(p.N % (BN / 2) == 0, "skinny_gemm: F must be a multiple of BN / 2 = ", BN / 2);
    p.nN = p.N / (BN / 2);
  } else {
    p.N = (int)wrows;
    p.nN = (p.N + BN - 1) / BN;
  }
  if (wpack)   // the packed image holds nN whole tiles of every K step
    TORCH_CHECK(w.dim() == 2 && w.size(1) == 64 && w.size(0) == (int64_t)p.nN * (K / 64) * BN,
                "skinny_gemm: packed weights must be [nN * K/64 * BN, 64] for this cfg");
  TORCH_CHECK(p.N % 8 == 0, "skinny_gemm: N must be a multiple of 8");
  p.nM = (int)((M + BM - 1) / BM);
  TORCH_CHECK((int64_t)p.nN * p.nM * split < (1ll << 31));
  if (epi == 1) {
    CHECK_DT(out, at::kFloat); CHECK_CONTIG(out);
    TORCH_CHECK(out.numel() >= split * M * p.N, "skinny_gemm: partial buffer needs split * M * N floats");
    p.ldo = p.N;
  } else {
    CHECK_DT(out, at::kBFloat16);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == p.N && out.stride(1) == 1 &&
                out.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0,
                "skinny_gemm: out must be [M, N] with 8-B aligned rows");
    p.ldo = out.stride(0);
  }
  p.out = out.data_ptr();
  nga::launch_skinny_gemm(p, (int)cfg, (int)epi, cur_stream(x));
}

void gemv(Tensor out, Tensor x, Tensor w, int64_t epi) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "gemv: 2-D x / w / out");
  TORCH_CHECK(x.device() == w.device() && x.device() == out.device(), "gemv: one device");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && w.is_contiguous(), "gemv: x rows / w contiguous, 16-B aligned");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) | reinterpret_cast<uintptr_t>(w.data_ptr())) % 16 == 0,
              "gemv: x / w must be 16-B aligned");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 4 && K % 8 == 0 && w.size(1) == K && M * K * 2 <= 160 * 1024,
              "gemv: 1 <= M <= 4, K % 8 == 0, M x K bf16 within 160 KiB");
  TORCH_CHECK(epi >= 0 && epi <= 2, "gemv: epi 0 (bf16), 1 (fp32), 2 (SwiGLU)");
  const int64_t N = epi == 2 ? w.size(0) / 2 : w.size(0);
  TORCH_CHECK(epi != 2 || w.size(0) % 2 == 0, "gemv: SwiGLU weight has 2F rows");
  TORCH_CHECK(out.size(0) == M && out.size(1) >= N && out.stride(1) == 1, "gemv: out [M, >= N]");
  TORCH_CHECK(epi == 1 ? out.scalar_type() == at::kFloat : out.scalar_type() == at::kBFloat16, "gemv: out dtype");
  nga::GemvParams p{};
  p.x = bfp(x);
  p.ldx = x.stride(0);
  p.w = bfp(w);
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.out = out.data_ptr();
  p.ldo = out.stride(0);
  TORCH_CHECK(nga::launch_gemv(p, (int)epi, cur_stream(x)), "gemv: shape out of range");
}

void splitk_swiglu(Tensor out, Tensor P, int64_t S) {
  CHECK_DEV(P); CHECK_BF16(out);
  TORCH_CHECK(out.device() == P.device(), "splitk_swiglu: out and P on one device");
  const int64_t M = out.size(0), F = out.size(1);
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.stride(0) % 8 == 0, "splitk_swiglu: out [M, F] rows 16-B aligned");
  TORCH_CHECK(P.is_contiguous() && P.scalar_type() == at::kFloat, "splitk_swiglu: P fp32 contiguous");
  TORCH_CHECK(S >= 1 && F % 8 == 0 && P.numel() >= S * M * 2 * F, "splitk_swiglu: P must hold S x M x 2F floats");
  nga::launch_splitk_swiglu(P.data_ptr<float>(), (int)S, (int)M, (int)F, bfp(out), out.stride(0), cur_stream(P));
}

void splitk_reduce(Tensor out, Tensor P, int64_t S) {
  CHECK_DEV(P); CHECK_DT(P, at::kFloat); CHECK_CONTIG(P); CHECK_BF16(out);
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.stride(0) % 8 == 0, "splitk_reduce: out [M, N] rows 16-B aligned");
  const int64_t M = out.size(0), N = out.size(1);
  TORCH_CHECK(S >= 1 && N % 8 == 0 && P.numel() >= S * M * N, "splitk_reduce: P must hold S x M x N floats");
  nga::launch_splitk_reduce(P.data_ptr<float>(), (int)S, (int)M, (int)N, bfp(out), out.stride(0), cur_stream(P));
}

// resid += sum of the S partial slabs; out = rmsnorm(resid) * w
void splitk_add_rmsnorm(Tensor out, Tensor resid, Tensor P, int64_t S, Tensor w, double eps) {
  CHECK_BF16(out); CHECK_BF16(resid); CHECK_BF16(w); CHECK_CONTIG(out); CHECK_CONTIG(resid);
  CHECK_DEV(P); CHECK_DT(P, at::kFloat); CHECK_CONTIG(P);
  TORCH_CHECK(resid.dim() == 2 && out.sizes() == resid.sizes());
  const int64_t M = resid.size(0), H = resid.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192 && w.numel() == H && w.is_contiguous());
  TORCH_CHECK(S >= 1 && P.numel() >= S * M * H, "splitk_add_rmsnorm: P must hold S x M x H floats");
  nga::launch_splitk_add_rmsnorm(P.data_ptr<float>(), (int)S, (int)M, bfp(resid), bfp(w), (float)eps, (int)H,
                                 bfp(out), cur_stream(resid));
}

// ------------------------------------------------------------------ attention
int64_t decode_pages_per_part(int64_t num_seqs, int64_t Hkv, int64_t max_ctx) {
  return nga::decode_attn_pages_per_part((int)num_seqs, (int)Hkv, (int)max_ctx);
}

void decode_attention(Tensor out, Tensor q, Tensor kc, Tensor vc, Tensor block_tables,
                      Tensor ctx_lens, int64_t Hq, int64_t Hkv, int64_t max_ctx, double scale,
                      int64_t pages_per_part, Tensor part_ml, Tensor part_o, int64_t window,
                      double k_scale, double v_scale, bool skip_empty) {
  CHECK_BF16(out); CHECK_BF16(q);
  const bool fp8 = kv_is_fp8(kc, vc);
  CHECK_CONTIG(kc); CHECK_CONTIG(vc);
  CHECK_DEV(block_tables); CHECK_DT(block_tables, at::kInt); CHECK_CONTIG(block_tables);
  CHECK_DEV(ctx_lens); CHECK_DT(ctx_lens, at::kInt);
  const int64_t B = ctx_lens.numel();
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(2) == 64 &&
              (kc.size(3) == 128 || kc.size(3) == 256),
              "decode_attention: k cache must be [nb, Hkv, 64, 128|256]");
  const int64_t D = kc.size(3);
  TORCH_CHECK(q.dim() == 2 && q.size(0) >= B && q.stride(1) == 1 && q.size(1) >= Hq * D,
              "decode_attention: q must be [B, >=Hq*D] with unit inner stride");
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= B && out.stride(1) == 1 && out.size(1) >= Hq * D);
  TORCH_CHECK(vc.sizes() == at::IntArrayRef({kc.size(0), Hkv, D, 64}), "v cache must be [nb, Hkv, D, 64]");
  TORCH_CHECK(window >= 0);
  TORCH_CHECK(Hq % Hkv == 0 && Hq / Hkv <= 16, "decode_attention: G = Hq/Hkv must be <= 16");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B);
  TORCH_CHECK(block_tables.size(1) * 64 >= max_ctx, "block table too narrow for max_ctx");
  TORCH_CHECK(pages_per_part >= 1);
  const int64_t pages = (max_ctx + 63) / 64;
  const int64_t nparts = (pages + pages_per_part - 1) / pages_per_part;
  if (nparts > 1) {
    TORCH_CHECK(nparts <= 256, "decode_attention: at most 256 key partitions");
    CHECK_DEV(part_ml); CHECK_DEV(part_o);
    TORCH_CHECK(part_ml.numel() >= B * Hq * nparts * 2 && part_o.numel() >= B * Hq * nparts * D,
                "decode_attention: partition workspace too small");
  }
  nga::launch_decode_attention(bfp(out), out.stride(0), bfp(q), q.stride(0), kc.data_ptr(),
                               vc.data_ptr(), block_tables.data_ptr<int32_t>(),
                               (int)block_tables.size(1), ctx_lens.data_ptr<int32_t>(), (int)B,
                               (int)Hq, (int)Hkv, (int)D, (int)max_ctx, (float)scale,
                               (int)pages_per_part,
                               nparts > 1 ? part_ml.data_ptr<float>() : nullptr,
                               nparts > 1 ? part_o.data_ptr<float>() : nullptr, (int)window, fp8,
                               (float)k_scale, (float)v_scale, cur_stream(q), skip_empty);
}

// Work-list prefill (32x32 kernel): q / out rows are absolute token rows of the step (the
// cu_q offsets of ALL its sequences); items [n, 2] int32 (sequence, row block) pairs, n_items
// a 1-element device int32 (read by the kernel, so a captured graph replays any step's list)
void prefill_attention_worklist(Tensor out, Tensor q, Tensor kc, Tensor vc, Tensor block_tables,
                                Tensor cu_q, Tensor ctx_lens, int64_t Hq, int64_t Hkv, double scale,
                                bool causal, int64_t window, Tensor items, Tensor n_items, int64_t grid,
                                int64_t ks, int64_t impl, double k_scale, double v_scale) {
  CHECK_BF16(out); CHECK_BF16(q);
  CHECK_CONTIG(kc); CHECK_CONTIG(vc);
  TORCH_CHECK(impl == 1 || impl == 2, "prefill_attention_worklist: impl 1 (16x16) or 2 (32x32)");
  TORCH_CHECK(Hq % Hkv == 0, "prefill_attention_worklist: Hq % Hkv");
  const bool fp8 = kv_is_fp8(kc, vc);
  TORCH_CHECK(kc.dim() == 4 && kc.size(1) == Hkv && kc.size(2) == 64, "k cache must be [nb, Hkv, 64, D]");
  const int64_t D = kc.size(3);
  TORCH_CHECK(impl == 2 ? (D == 128 && !fp8) : (D == 64 || D == 128 || D == 256),
              "prefill_attention_worklist: the 32x32 kernel takes bf16 head_dim 128 pages, the 16x16 one "
              "head_dim 64 / 128 / 256");
  TORCH_CHECK(vc.sizes() == at::IntArrayRef({kc.size(0), Hkv, D, 64}), "v cache must be [nb, Hkv, D, 64]");
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1 && q.size(1) >= Hq * D && q.stride(0) % 8 == 0);
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) >= Hq * D && out.size(0) == q.size(0));
  CHECK_DEV(block_tables); CHECK_DT(block_tables, at::kInt); CHECK_CONTIG(block_tables);
  TORCH_CHECK(block_tables.dim() == 2 && (impl == 1 || block_tables.size(1) <= 1024),
              "prefill_attention_worklist: at most 1024 pages per sequence (32x32 kernel)");
  CHECK_DEV(cu_q); CHECK_DT(cu_q, at::kInt); CHECK_CONTIG(cu_q);
  CHECK_DEV(ctx_lens); CHECK_DT(ctx_lens, at::kInt); CHECK_CONTIG(ctx_lens);
  TORCH_CHECK(cu_q.numel() == ctx_lens.numel() + 1 && block_tables.size(0) >= ctx_lens.numel(),
              "prefill_attention_worklist: cu_q [B+1], ctx_lens [B], block_tables [>=B, pages]");
  CHECK_DEV(items); CHECK_DT(items, at::kInt); CHECK_CONTIG(items);
  CHECK_DEV(n_items); CHECK_DT(n_items, at::kInt);
  TORCH_CHECK(items.dim() == 2 && items.size(1) == 2 && n_items.numel() == 1,
              "prefill_attention_worklist: items [n, 2], n_items [1]");
  TORCH_CHECK(window >= 0 && (window == 0 || causal));
  TORCH_CHECK(grid >= 1 && grid <= 65535 && (ks == 1 || ks == 2), "prefill_attention_worklist: grid / ks");
  nga::PrefillParams p{};
  p.out = bfp(out);
  p.out_stride = out.stride(0);
  p.q = bfp(q);
  p.q_stride = q.stride(0);
  p.cu_q = cu_q.data_ptr<int32_t>();
  p.Hq = (int)Hq;
  p.Hkv = (int)Hkv;
  p.scale = (float)scale;
  p.window = (int)window;
  p.kc = static_cast<const uint16_t*>(kc.data_ptr());
  p.vc = static_cast<const uint16_t*>(vc.data_ptr());
  p.block_tables = block_tables.data_ptr<int32_t>();
  p.max_blocks = (int)block_tables.size(1);
  p.ctx_lens = ctx_lens.data_ptr<int32_t>();
  p.v_scale = 1.f;
  p.kv_fp8 = fp8 ? 1 : 0;
  if (fp8) {
    p.scale = (float)(scale * k_scale);
    p.v_scale = (float)v_scale;
  }
  p.items = items.data_ptr<int32_t>();
  p.n_items = n_items.data_ptr<int32_t>();
  if (impl == 2) nga::launch_prefill_attention_v2_worklist(p, (int)grid, (int)ks, causal, cur_stream(q));
  else nga::launch_prefill_attention_v1_worklist(p, (int)grid, (int)D, causal, cur_stream(q));
}

void prefill_attention(Tensor out, Tensor q, c10::optional<Tensor> k, c10::optional<Tensor> v,
                       c10::optional<Tensor> kc, c10::optional<Tensor> vc,
                       c10::optional<Tensor> block_tables, Tensor cu_q,
                       c10::optional<Tensor> ctx_lens, int64_t Hq, int64_t Hkv, int64_t D,
                       int64_t max_q_len, double scale, bool causal, int64_t window,
                       int64_t impl, double k_scale, double v_scale) {
  CHECK_BF16(out); CHECK_BF16(q);
  TORCH_CHECK(impl >= 0 && impl <= 6,
              "prefill_attention: impl is 0 (auto), 1, 2, 3, 4 (auto, alone), 5 (32x32, 8 waves per tile) "
              "or 6 (32x32, register-staged tiles)");
  CHECK_DEV(cu_q); CHECK_DT(cu_q, at::kInt); CHECK_CONTIG(cu_q);
  TORCH_CHECK(D == 64 || D == 128 || (D == 32 && !kc.has_value()) || (D == 256 && kc.has_value()),
              "prefill_attention: head_dim must be 64 or 128 (32: packed only, 256: paged only)");
  TORCH_CHECK(window >= 0 && (window == 0 || causal), "prefill_attention: a window needs causal attention");
  TORCH_CHECK(Hq % Hkv == 0);
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1 && q.size(1) >= Hq * D && q.stride(0) % 8 == 0);
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) >= Hq * D && out.size(0) == q.size(0));
  const int64_t B = cu_q.numel() - 1;
  nga::PrefillParams p{};
  p.out = bfp(out);
  p.out_stride = out.stride(0);
  p.q = bfp(q);
  p.q_stride = q.stride(0);
  p.cu_q = cu_q.data_ptr<int32_t>();
  p.Hq = (int)Hq;
  p.Hkv = (int)Hkv;
  p.scale = (float)scale;
  p.window = (int)window;
  const bool paged = kc.has_value();
  if (paged) {
    TORCH_CHECK(vc.has_value() && block_tables.has_value() && ctx_lens.has_value());
    p.kv_fp8 = kv_is_fp8(*kc, *vc) ? 1 : 0;
    CHECK_CONTIG(*kc); CHECK_CONTIG(*vc);
    if (p.kv_fp8) {
      p.scale = (float)(scale * k_scale);
      p.v_scale = (float)v_scale;
    }
    TORCH_CHECK(kc->dim() == 4 && kc->size(1) == Hkv && kc->size(2) == 64 && kc->size(3) == D);
    TORCH_CHECK(vc->sizes() == at::IntArrayRef({kc->size(0), Hkv, D, 64}));
    CHECK_DEV(*block_tables); CHECK_DT(*block_tables, at::kInt); CHECK_CONTIG(*block_tables);
    CHECK_DEV(*ctx_lens); CHECK_DT(*ctx_lens, at::kInt);
    TORCH_CHECK(block_tables->dim() == 2 && block_tables->size(0) >= B && ctx_lens->numel() >= B);
    p.kc = bfp(*kc);
    p.vc = bfp(*vc);
    p.block_tables = block_tables->data_ptr<int32_t>();
    p.max_blocks = (int)block_tables->size(1);
    p.ctx_lens = ctx_lens->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(k.has_value() && v.has_value());
    CHECK_BF16(*k); CHECK_BF16(*v);
    TORCH_CHECK(k->dim() == 2 && k->stride(1) == 1 && k->stride(0) == v->stride(0) && k->size(0) == q.size(0));
    TORCH_CHECK(k->stride(0) % 8 == 0 && k->size(1) >= Hkv * D && v->size(1) >= Hkv * D);
    p.k = bfp(*k);
    p.v = bfp(*v);
    p.kv_stride = k->stride(0);
  }
  p.impl = (int)impl;
  nga::launch_prefill_attention(p, (int)B, (int)max_q_len, (int)D, paged, causal, cur_stream(q));
}

// ------------------------------------------------------------------ sampling
void sample(Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p,
            c10::optional<Tensor> rep_penalty, c10::optional<Tensor> history, Tensor seeds,
            Tensor steps, Tensor out_tok, Tensor out_logprob) {
  CHECK_DEV(logits); CHECK_DT(logits, at::kFloat); CHECK_CONTIG(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.size(1) <= 262144, "sample: vocab must be <= 262144");
  const int64_t B = logits.size(0);
  CHECK_DT(temperature, at::kFloat); CHECK_DT(top_k, at::kInt); CHECK_DT(top_p, at::kFloat);
  CHECK_DT(seeds, at::kLong); CHECK_DT(steps, at::kLong);
  CHECK_DT(out_tok, at::kInt); CHECK_DT(out_logprob, at::kFloat);
  TORCH_CHECK(temperature.numel() >= B && top_k.numel() >= B && top_p.numel() >= B &&
              seeds.numel() >= B && steps.numel() >= B && out_tok.numel() >= B && out_logprob.numel() >= B);
  const float* rp = nullptr;
  const int32_t* hp = nullptr;
  int hl = 0;
  if (rep_penalty.has_value() && history.has_value()) {
    CHECK_DT(*rep_penalty, at::kFloat); CHECK_DT(*history, at::kInt); CHECK_CONTIG(*history);
    TORCH_CHECK(history->dim() == 2 && history->size(0) >= B && rep_penalty->numel() >= B);
    rp = rep_penalty->data_ptr<float>();
    hp = history->data_ptr<int32_t>();
    hl = (int)history->size(1);
  }
  nga::launch_sample(logits.data_ptr<float>(), (int)B, (int)logits.size(1), temperature.data_ptr<float>(),
                     top_k.data_ptr<int32_t>(), top_p.data_ptr<float>(), rp, hp, hl,
                     seeds.data_ptr<int64_t>(), steps.data_ptr<int64_t>(), out_tok.data_ptr<int32_t>(),
                     out_logprob.data_ptr<float>(), cur_stream(logits));
}

// ------------------------------------------------------------------ embedding gather
void embedding(Tensor out, Tensor table, Tensor ids, int64_t vocab_lo, double scale) {
  CHECK_BF16(out); CHECK_BF16(table); CHECK_CONTIG(out); CHECK_CONTIG(table);
  CHECK_DEV(ids); CHECK_DT(ids, at::kInt); CHECK_CONTIG(ids);
  TORCH_CHECK(table.dim() == 2 && table.size(1) % 8 == 0, "embedding: table [rows, H], H % 8 == 0");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == ids.numel() && out.size(1) == table.size(1),
              "embedding: out [T, H] for T ids");
  nga::launch_embedding(bfp(out), bfp(table), ids.data_ptr<int32_t>(), (int)ids.numel(), (int)table.size(1),
                        vocab_lo, table.size(0), (float)scale, cur_stream(ids));
}

// ------------------------------------------------------------------ vector search
void score(Tensor Q, Tensor X, c10::optional<Tensor> row_bias, Tensor S, double dot_scale) {
  CHECK_BF16(Q); CHECK_BF16(X); CHECK_CONTIG(Q); CHECK_CONTIG(X);
  CHECK_DEV(S); CHECK_DT(S, at::kFloat); CHECK_CONTIG(S);
  TORCH_CHECK(Q.dim() == 2 && X.dim() == 2 && Q.size(1) == X.size(1));
  const int64_t D = X.size(1);
  TORCH_CHECK(D % 32 == 0 && D <= 1216, "score: D must be a multiple of 32 and <= 1216");
  TORCH_CHECK(S.size(0) == Q.size(0) && S.size(1) == X.size(0));
  const float* bp = nullptr;
  if (row_bias.has_value()) {
    CHECK_DEV(*row_bias); CHECK_DT(*row_bias, at::kFloat);
    TORCH_CHECK(row_bias->numel() == X.size(0));
    bp = row_bias->data_ptr<float>();
  }
  nga::launch_score(bfp(Q), (int)Q.size(0), bfp(X), X.size(0), (int)D, bp, S.data_ptr<float>(),
                    (float)dot_scale, cur_stream(X));
}

// fused score + per-block top-k (flat: row_beg/row_end/qtab absent, n_items = ceil(nq / 64))
void score_topk(Tensor Q, Tensor X, c10::optional<Tensor> row_bias, double dot_scale,
                c10::optional<Tensor> row_beg, c10::optional<Tensor> row_end, c10::optional<Tensor> qtab,
                c10::optional<Tensor> slot_rows, int64_t n_items, int64_t max_q_per_item, int64_t nblk,
                int64_t k, Tensor out_v, Tensor out_r) {
  CHECK_BF16(Q); CHECK_BF16(X); CHECK_CONTIG(Q); CHECK_CONTIG(X);
  TORCH_CHECK(Q.dim() == 2 && X.dim() == 2 && Q.size(1) == X.size(1));
  const int64_t D = X.size(1);
  TORCH_CHECK(D % 32 == 0 && (D <= 1216 || nga::score_topk_dma_ok((int)D, (int)max_q_per_item)),
              "score_topk: D must be a multiple of 32 and <= 1216 (<= 2048 for <= 16 queries per item)");
  TORCH_CHECK(max_q_per_item >= 1 && max_q_per_item <= 64, "score_topk: 1..64 queries per item");
  TORCH_CHECK(k >= 1 && k <= nga::score_topk_kmax((int)max_q_per_item), "score_topk: k too large");
  TORCH_CHECK(n_items >= 1 && nblk >= 1 && nblk <= 65535 && n_items <= 65535, "score_topk: bad grid");
  TORCH_CHECK(X.size(0) < (int64_t(1) << 31), "score_topk: rows must fit int32");
  const bool items = row_beg.has_value();
  TORCH_CHECK(items == row_end.has_value() && items == qtab.has_value(),
              "score_topk: row_beg, row_end and qtab go together");
  if (!items) TORCH_CHECK(n_items == (Q.size(0) + 63) / 64, "score_topk: flat search has ceil(nq/64) items");
  const float* bp = nullptr;
  if (row_bias.has_value()) {
    CHECK_DEV(*row_bias); CHECK_DT(*row_bias, at::kFloat);
    TORCH_CHECK(row_bias->numel() == X.size(0));
    bp = row_bias->data_ptr<float>();
  }
  const int64_t *rb = nullptr, *re = nullptr;
  const int32_t* qt = nullptr;
  const int32_t* sr = nullptr;
  int64_t out_rows = n_items * 64;
  if (slot_rows.has_value()) {
    TORCH_CHECK(items, "score_topk: slot_rows needs item tables");
    CHECK_DEV(*slot_rows); CHECK_DT(*slot_rows, at::kInt); CHECK_CONTIG(*slot_rows);
    TORCH_CHECK(slot_rows->numel() == n_items * 64, "score_topk: slot_rows must be [n_items, 64]");
    sr = slot_rows->data_ptr<int32_t>();
    // rows of the pair-ordered output: the caller sizes it to its pair count (every slot_rows
    // entry must be < that; the plan kernel writes pair indices < nq * nprobe)
    out_rows = out_v.size(0);
  }
  if (items) {
    CHECK_DEV(*row_beg); CHECK_DEV(*row_end); CHECK_DEV(*qtab);
    CHECK_DT(*row_beg, at::kLong); CHECK_DT(*row_end, at::kLong); CHECK_DT(*qtab, at::kInt);
    CHECK_CONTIG(*row_beg); CHECK_CONTIG(*row_end); CHECK_CONTIG(*qtab);
    TORCH_CHECK(row_beg->numel() == n_items && row_end->numel() == n_items && qtab->numel() == n_items * 64,
                "score_topk: item tables must be [n_items], [n_items], [n_items, 64]");
    rb = row_beg->data_ptr<int64_t>();
    re = row_end->data_ptr<int64_t>();
    qt = qtab->data_ptr<int32_t>();
  }
  CHECK_DEV(out_v); CHECK_DEV(out_r); CHECK_DT(out_v, at::kFloat); CHECK_DT(out_r, at::kLong);
  CHECK_CONTIG(out_v); CHECK_CONTIG(out_r);
  TORCH_CHECK(out_v.dim() == 3 && out_v.size(1) == nblk && out_v.size(2) == k && out_v.size(0) == out_rows &&
                  out_r.sizes() == out_v.sizes(),
              "score_topk: outputs must be [n_items * 64 (or the pair count with slot_rows), nblk, k]");
  nga::launch_score_topk(bfp(Q), (int)Q.size(0), bfp(X), X.size(0), (int)D, bp, (float)dot_scale, rb, re, qt,
                         sr, (int)n_items, (int)max_q_per_item, (int)nblk, (int)k, out_v.data_ptr<float>(),
                         out_r.data_ptr<int64_t>(), cur_stream(X));
}

// (query, probe) pairs -> per-list work-item slots (qtab, slot_rows: [nlist * ceil(nq/64) * 64])
void ivf_plan(Tensor probes, int64_t nlist, Tensor qtab, Tensor slot_rows) {
  CHECK_DEV(probes); CHECK_DT(probes, at::kLong); CHECK_CONTIG(probes);
  TORCH_CHECK(probes.dim() == 2, "ivf_plan: probes [nq, nprobe]");
  TORCH_CHECK(nlist >= 1 && nlist <= nga::IVF_PLAN_MAX_LISTS, "ivf_plan: nlist out of range");
  const int64_t nq = probes.size(0), nprobe = probes.size(1);
  const int64_t slots = nlist * ((nq + 63) / 64) * 64;
  CHECK_DEV(qtab); CHECK_DEV(slot_rows); CHECK_DT(qtab, at::kInt); CHECK_DT(slot_rows, at::kInt);
  CHECK_CONTIG(qtab); CHECK_CONTIG(slot_rows);
  TORCH_CHECK(qtab.numel() == slots && slot_rows.numel() == slots, "ivf_plan: tables must hold nlist*ceil(nq/64)*64");
  if (nq == 0) return;
  nga::launch_ivf_plan(probes.data_ptr<int64_t>(), (int)nq, (int)nprobe, (int)nlist, qtab.data_ptr<int32_t>(),
                       slot_rows.data_ptr<int32_t>(), cur_stream(probes));
}

void topk(Tensor in, c10::optional<Tensor> in_idx, int64_t seg_len, int64_t k, Tensor out_v,
          Tensor out_i) {
  CHECK_DEV(in); CHECK_DT(in, at::kFloat); CHECK_CONTIG(in);
  TORCH_CHECK(in.dim() == 2);
  TORCH_CHECK(k >= 1 && k <= 1024, "topk: k must be in [1, 1024]");
  const int64_t rows = in.size(0), len = in.size(1);
  const int64_t nseg = (len + seg_len - 1) / seg_len;
  CHECK_DT(out_v, at::kFloat); CHECK_DT(out_i, at::kLong); CHECK_CONTIG(out_v); CHECK_CONTIG(out_i);
  TORCH_CHECK(out_v.numel() == rows * nseg * k && out_i.numel() == rows * nseg * k, "topk: bad output size");
  const int64_t* ip = nullptr;
  if (in_idx.has_value()) {
    CHECK_DT(*in_idx, at::kLong); CHECK_CONTIG(*in_idx);
    TORCH_CHECK(in_idx->sizes() == in.sizes());
    ip = in_idx->data_ptr<int64_t>();
  }
  nga::launch_topk(in.data_ptr<float>(), ip, rows, len, seg_len, (int)k, out_v.data_ptr<float>(),
                   out_i.data_ptr<int64_t>(), cur_stream(in));
}

// packed step-input upload: scatter segments of the device staging buffer `src` (uint8) to
// raw device addresses (the engine's fixed step buffers), one kernel for every segment
void scatter_segments(Tensor src, const std::vector<int64_t>& dst, const std::vector<int64_t>& off,
                      const std::vector<int64_t>& bytes) {
  CHECK_DEV(src); CHECK_CONTIG(src); CHECK_DT(src, at::kByte);
  TORCH_CHECK(dst.size() == off.size() && off.size() == bytes.size() && dst.size() <= (size_t)nga::kMaxSegments,
              "scatter_segments: matching dst / off / bytes lists of at most 32 segments");
  nga::SegmentTable t{};
  t.n = (int)dst.size();
  for (size_t i = 0; i < dst.size(); ++i) {
    TORCH_CHECK(off[i] % 16 == 0 && dst[i] % 16 == 0 && bytes[i] % 4 == 0 && bytes[i] >= 0 &&
                    off[i] + bytes[i] <= src.numel(),
                "scatter_segments: 16-B aligned segments of whole 4-B words inside the staging buffer");
    t.dst[i] = dst[i];
    t.off[i] = off[i];
    t.bytes[i] = bytes[i];
  }
  nga::launch_scatter_segments(reinterpret_cast<const uint8_t*>(src.data_ptr()), t, cur_stream(src));
}

// Host staging the GPU reads in place: pinned, mapped, portable and coherent (fine-grained) host
// memory, so a kernel can take a step's packed inputs straight from it, with no copy dispatch
// before it
Tensor host_staging(int64_t nbytes) {
  TORCH_CHECK(nbytes > 0, "host_staging: size");
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, (size_t)nbytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable);
  TORCH_CHECK(e == hipSuccess && p, "host_staging: hipHostMalloc: ", hipGetErrorString(e));
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipHostFree(q); },
                          torch::TensorOptions().dtype(torch::kUInt8));
}

// the scatter kernel reading a host_staging buffer through its device mapping, on `device`'s
// current stream
void scatter_host(Tensor host, int64_t device, const std::vector<int64_t>& dst, const std::vector<int64_t>& off,
                  const std::vector<int64_t>& bytes) {
  TORCH_CHECK(!host.is_cuda() && host.is_contiguous() && host.scalar_type() == at::kByte,
              "scatter_host: host staging must be a uint8 CPU tensor from host_staging()");
  TORCH_CHECK(dst.size() == off.size() && off.size() == bytes.size() && dst.size() <= (size_t)nga::kMaxSegments,
              "scatter_host: matching dst / off / bytes lists of at most 32 segments");
  void* dp = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dp, host.data_ptr(), 0);
  TORCH_CHECK(e == hipSuccess && dp, "scatter_host: not a mapped host buffer: ", hipGetErrorString(e));
  nga::SegmentTable t{};
  t.n = (int)dst.size();
  for (size_t i = 0; i < dst.size(); ++i) {
    TORCH_CHECK(off[i] % 16 == 0 && dst[i] % 16 == 0 && bytes[i] % 4 == 0 && bytes[i] >= 0 &&
                    off[i] + bytes[i] <= host.numel(),
                "scatter_host: 16-B aligned segments of whole 4-B words inside the staging buffer");
    t.dst[i] = dst[i];
    t.off[i] = off[i];
    t.bytes[i] = bytes[i];
  }
  nga::launch_scatter_segments(reinterpret_cast<const uint8_t*>(dp), t,
                               c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream());
}

// a begin / end marker kernel on the current stream (kernel-trace window delimiters)
void region_marker(Tensor sink, int64_t end) {
  CHECK_DEV(sink); CHECK_DT(sink, at::kInt);
  nga::launch_region_marker((int)end, sink.data_ptr<int32_t>(), cur_stream(sink));
}

void pool_l2norm(Tensor hidden, Tensor cu, int64_t mode, bool normalize, Tensor out) {
  CHECK_BF16(hidden); CHECK_CONTIG(hidden);
  CHECK_DEV(cu); CHECK_DT(cu, at::kInt);
  CHECK_DEV(out); CHECK_DT(out, at::kFloat); CHECK_CONTIG(out);
  const int64_t H = hidden.size(1), B = cu.numel() - 1;
  TORCH_CHECK(H % 8 == 0 && H <= 8192 && out.size(0) == B && out.size(1) == H);
  nga::launch_pool_l2norm(bfp(hidden), cu.data_ptr<int32_t>(), (int)B, (int)H, (int)mode,
                          normalize ? 1 : 0, out.data_ptr<float>(), cur_stream(hidden));
}

void row_sqnorm(Tensor X, Tensor out) {
  CHECK_BF16(X); CHECK_CONTIG(X);
  CHECK_DEV(out); CHECK_DT(out, at::kFloat);
  TORCH_CHECK(X.dim() == 2 && X.size(1) % 8 == 0 && out.numel() == X.size(0));
  nga::launch_row_sqnorm(bfp(X), X.size(0), (int)X.size(1), out.data_ptr<float>(), cur_stream(X));
}

// ---- DSP (FM-ASR front end)
void fir_c64(Tensor x, Tensor taps, c10::optional<Tensor> hist, Tensor y) {
  CHECK_DEV(x); CHECK_DT(x, at::kComplexFloat); CHECK_CONTIG(x);
  CHECK_DEV(taps); CHECK_DT(taps, at::kFloat); CHECK_CONTIG(taps);
  CHECK_DEV(y); CHECK_DT(y, at::kComplexFloat); CHECK_CONTIG(y);
  const int64_t n = x.numel(), nt = taps.numel();
  TORCH_CHECK(nt >= 1 && nt <= nga::kFirMaxTaps, "fir_c64: 1..1024 taps");
  TORCH_CHECK(y.numel() == n, "fir_c64: output size");
  const float* hp = nullptr;
  if (hist.has_value()) {
    CHECK_DEV(*hist); CHECK_DT(*hist, at::kComplexFloat); CHECK_CONTIG(*hist);
    TORCH_CHECK(hist->numel() == nt - 1, "fir_c64: history must hold ntaps-1 samples");
    hp = reinterpret_cast<const float*>(hist->data_ptr());
  }
  nga::launch_fir_c64(reinterpret_cast<const float*>(x.data_ptr()), (int)n, taps.data_ptr<float>(), (int)nt, hp,
                      reinterpret_cast<float*>(y.data_ptr()), cur_stream(x));
}

void fm_demod(Tensor x, double prev_re, double prev_im, bool has_prev, Tensor y) {
  CHECK_DEV(x); CHECK_DT(x, at::kComplexFloat); CHECK_CONTIG(x);
  CHECK_DEV(y); CHECK_DT(y, at::kFloat); CHECK_CONTIG(y);
  const int64_t n = x.numel();
  TORCH_CHECK(y.numel() == (has_prev ? n : std::max<int64_t>(0, n - 1)), "fm_demod: output size");
  nga::launch_fm_demod(reinterpret_cast<const float*>(x.data_ptr()), (int)n, (float)prev_re, (float)prev_im,
                       has_prev ? 1 : 0, y.data_ptr<float>(), cur_stream(x));
}

void resample_pcm(Tensor x, Tensor h, int64_t down, int64_t pre, double gain, c10::optional<Tensor> yf,
                  c10::optional<Tensor> yi) {
  CHECK_DEV(x); CHECK_DT(x, at::kFloat); CHECK_CONTIG(x);
  CHECK_DEV(h); CHECK_DT(h, at::kFloat); CHECK_CONTIG(h);
  TORCH_CHECK(down >= 1 && pre >= 0, "resample_pcm: bad down/pre");
  int64_t nout = -1;
  float* fp = nullptr;
  int16_t* ip = nullptr;
  if (yf.has_value()) {
    CHECK_DEV(*yf); CHECK_DT(*yf, at::kFloat); CHECK_CONTIG(*yf);
    nout = yf->numel();
    fp = yf->data_ptr<float>();
  }
  if (yi.has_value()) {
    CHECK_DEV(*yi); CHECK_DT(*yi, at::kShort); CHECK_CONTIG(*yi);
    TORCH_CHECK(nout < 0 || yi->numel() == nout, "resample_pcm: outputs differ in size");
    nout = yi->numel();
    ip = yi->data_ptr<int16_t>();
  }
  TORCH_CHECK(nout >= 0, "resample_pcm: need an output");
  nga::launch_resample_pcm(x.data_ptr<float>(), (int)x.numel(), h.data_ptr<float>(), (int)h.numel(), (int)down,
                           (int)pre, (int)nout, (float)gain, fp, ip, cur_stream(x));
}

// ---- FP8 W8A8: row-wise activation quantisation (mode 0: x; mode 1: silu(gate) * up)
void quant_fp8_rows(Tensor x, int64_t mode, Tensor y, Tensor scale) {
  CHECK_BF16(x);
  CHECK_DEV(y); CHECK_CONTIG(y); CHECK_DEV(scale); CHECK_CONTIG(scale);
  TORCH_CHECK(y.scalar_type() == at::kFloat8_e4m3fn, "quant_fp8_rows: y must be float8_e4m3fn");
  CHECK_DT(scale, at::kFloat);
  TORCH_CHECK(mode == 0 || mode == 1, "quant_fp8_rows: mode 0 (x) or 1 (silu(gate) * up)");
  TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && x.stride(1) == 1, "quant_fp8_rows: 2-D, unit column stride");
  const int64_t rows = x.size(0);
  const int64_t H = mode == 0 ? x.size(1) : x.size(1) / 2;
  TORCH_CHECK(mode == 0 || x.size(1) % 2 == 0, "quant_fp8_rows: SwiGLU input must be [rows, 2F]");
  TORCH_CHECK(H % 8 == 0 && x.stride(0) % 8 == 0, "quant_fp8_rows: H and the row stride must be multiples of 8");
  TORCH_CHECK(y.size(0) >= rows && y.size(1) == H, "quant_fp8_rows: y must be [>= rows, H]");
  TORCH_CHECK(scale.numel() >= rows, "quant_fp8_rows: scale must hold one value per row");
  nga::launch_quant_fp8_rows(bfp(x), x.stride(0), rows, (int)H, (int)mode,
                             reinterpret_cast<uint8_t*>(y.data_ptr()), scale.data_ptr<float>(), cur_stream(x));
}

// ---- custom all-reduce over IPC peer buffers (TP decode)
struct CustomAR {
  std::unique_ptr<nga::CustomAllReduce> impl;
  CustomAR(int64_t rank, int64_t world, int64_t cap_bytes, double timeout_s)
      : impl(new nga::CustomAllReduce((int)rank, (int)world, cap_bytes, timeout_s)) {}
  py::bytes handle() const { return py::bytes(impl->handle()); }
  void open(const std::vector<std::string>& handles) { impl->open(handles); }
  // out may alias inp (in-place all-reduce)
  void all_reduce(Tensor inp, Tensor out, int64_t algo) {
    CHECK_DEV(inp); CHECK_DEV(out); CHECK_CONTIG(inp); CHECK_CONTIG(out);
    TORCH_CHECK(inp.scalar_type() == out.scalar_type() && inp.numel() == out.numel(),
                "custom all-reduce: in/out must match");
    TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat,
                "custom all-reduce: bf16 or fp32");
    TORCH_CHECK(algo >= 0 && algo <= 2, "custom all-reduce: algo 0 (auto), 1 (one-shot), 2 (two-shot)");
    const int64_t bytes = inp.numel() * inp.element_size();
    impl->run(inp.data_ptr(), out.data_ptr(), bytes, inp.scalar_type() == at::kBFloat16, (int)algo,
              cur_stream(inp));
  }
  // resid += all_reduce(inp); out = rmsnorm(resid) * w   (bf16 [rows, H])
  void all_reduce_add_rmsnorm(Tensor inp, Tensor resid, Tensor w, Tensor out, double eps) {
    CHECK_BF16(inp); CHECK_BF16(resid); CHECK_BF16(w); CHECK_BF16(out);
    CHECK_CONTIG(inp); CHECK_CONTIG(resid); CHECK_CONTIG(w); CHECK_CONTIG(out);
    TORCH_CHECK(inp.dim() == 2 && resid.sizes() == inp.sizes() && out.sizes() == inp.sizes(),
                "all_reduce_add_rmsnorm: inp/resid/out must be the same [rows, H]");
    TORCH_CHECK(w.numel() == inp.size(1), "all_reduce_add_rmsnorm: weight must have H entries");
    impl->run_add_rmsnorm(inp.data_ptr(), bfp(resid), bfp(w), bfp(out), (int)inp.size(0), (int)inp.size(1),
                          (float)eps, cur_stream(inp));
  }
  // out [rows, world * cols] = every rank's inp [rows, cols] side by side (rank order)
  void all_gather(Tensor inp, Tensor out) {
    CHECK_DEV(inp); CHECK_DEV(out); CHECK_CONTIG(inp); CHECK_CONTIG(out);
    TORCH_CHECK(inp.scalar_type() == out.scalar_type() && inp.dim() == 2 && out.dim() == 2 &&
                out.size(0) == inp.size(0) && out.size(1) == inp.size(1) * impl->world(),
                "custom all-gather: out must be [rows, world * cols] of inp's dtype");
    const int64_t row_bytes = inp.size(1) * inp.element_size();
    TORCH_CHECK(row_bytes % 16 == 0, "custom all-gather: row bytes must be a multiple of 16");
    impl->run_gather(inp.data_ptr(), out.data_ptr(), inp.size(0), row_bytes, cur_stream(inp));
  }
  int64_t error() const { return impl->error(); }
  int64_t capacity() const { return impl->capacity(); }
  void set_two_shot_threshold(int64_t b) { impl->set_two_shot_threshold(b); }
  void set_max_blocks(int64_t b) { impl->set_max_blocks((int)b); }
  int64_t max_blocks() const { return impl->max_blocks(); }
};

// ---- debug launch checking (SURVEY.md §5.2 "stream-ordering asserts in debug builds"):
// NGA_DEBUG_SYNC=1 checks every kernel launch and synchronises its stream right after it, so
// an asynchronous fault is reported by the op that caused it (the HIP_LAUNCH_BLOCKING-style
// localisation the box's no-debugger policy calls for). Streams under hipGraph capture are
// only launch-checked. Off by default: no cost on the serving path.
bool debug_sync() {
  static const bool on = [] {
    const char* e = std::getenv("NGA_DEBUG_SYNC");
    return e != nullptr && e[0] != '\0' && e[0] != '0';
  }();
  return on;
}

void post_launch(const char* name) {
  if (!debug_sync()) return;
  hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, name, ": kernel launch failed: ", hipGetErrorString(e));
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
    e = hipStreamSynchronize(st);
    TORCH_CHECK(e == hipSuccess, name, ": kernel failed on the GPU: ", hipGetErrorString(e));
  }
}

template <typename... A>
std::function<void(A...)> checked(const char* name, void (*f)(A...)) {
  return [name, f](A... a) {
    f(std::forward<A>(a)...);
    post_launch(name);
  };
}

}  // namespace


// ---- kernel-form registry (kernels.h): environment read once, then set explicitly
namespace nga {
namespace {
struct FormSpec {
  const char* name;
  const char* env;
  int dflt;
};
const FormSpec kForms[KF_COUNT] = {
    {"decode_dma", "NGA_DECODE_DMA", 2}, {"decode_nt", "NGA_DECODE_NT", 2},
    {"search_dma", "NGA_SEARCH_DMA", 1}, {"prefill_v1", "NGA_PREFILL_V1", 0},
    {"prefill_ks", "NGA_PREFILL_KS", 0}, {"rope_vnt", "NGA_ROPE_VNT", 2},
    {"decode_dma_aux", "NGA_DECODE_DMA_AUX", 2}};
std::atomic<int>* forms() {
  static std::atomic<int> v[KF_COUNT];
  static const bool init = [] {
    for (int i = 0; i < KF_COUNT; ++i) {
      const char* e = std::getenv(kForms[i].env);
      v[i].store(e && e[0] ? std::atoi(e) : kForms[i].dflt);
    }
    return true;
  }();
  (void)init;
  return v;
}
}  // namespace
int kernel_form(KernelForm f) { return forms()[f].load(std::memory_order_relaxed); }
void set_kernel_form(KernelForm f, int value) { forms()[f].store(value); }
const char* kernel_form_name(KernelForm f) { return kForms[f].name; }
}  // namespace nga

namespace {
int form_id(const std::string& name) {
  for (int i = 0; i < nga::KF_COUNT; ++i)
    if (name == nga::kernel_form_name((nga::KernelForm)i)) return i;
  TORCH_CHECK(false, "unknown kernel form ", name);
  return -1;
}
}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "nv_genai_amd gfx950 HIP kernels";
  m.def("debug_sync", &debug_sync);
  m.def("kernel_form", [](const std::string& n) { return (int64_t)nga::kernel_form((nga::KernelForm)form_id(n)); });
  m.def("set_kernel_form", [](const std::string& n, int64_t v) { nga::set_kernel_form((nga::KernelForm)form_id(n), (int)v); });
  m.def("rmsnorm", checked("rmsnorm", &rmsnorm));
  m.def("add_rmsnorm", checked("add_rmsnorm", &add_rmsnorm));
  m.def("layernorm", checked("layernorm", &layernorm));
  m.def("add_layernorm", checked("add_layernorm", &add_layernorm));
  m.def("gelu_tanh_mul", checked("gelu_tanh_mul", &gelu_tanh_mul));
  m.def("silu_mul", checked("silu_mul", &silu_mul));
  m.def("bias_gelu", checked("bias_gelu", &bias_gelu));
  m.def("rope_cache", checked("rope_cache", &rope_cache));
  m.def("decode_pages_per_part", &decode_pages_per_part);
  m.def("decode_attention", checked("decode_attention", &decode_attention));
  m.def("prefill_attention", checked("prefill_attention", &prefill_attention));
  m.def("prefill_attention_worklist", checked("prefill_attention_worklist", &prefill_attention_worklist));
  m.def("moe_route", checked("moe_route", &moe_route));
  m.def("moe_align", checked("moe_align", &moe_align));
  m.def("moe_gemm", checked("moe_gemm", &moe_gemm));
  m.def("moe_combine", checked("moe_combine", &moe_combine));
  m.def("skinny_cfg", &skinny_cfg);
  m.def("skinny_cfg_count", [] { return (int64_t)nga::skinny_gemm_cfg_count(); });
  m.def("skinny_gemm", checked("skinny_gemm", &skinny_gemm));
  m.def("splitk_reduce", checked("splitk_reduce", &splitk_reduce));
  m.def("splitk_swiglu", checked("splitk_swiglu", &splitk_swiglu));
  m.def("gemv", checked("gemv", &gemv));
  m.def("splitk_add_rmsnorm", checked("splitk_add_rmsnorm", &splitk_add_rmsnorm));
  m.def("sample", checked("sample", &sample));
  m.def("embedding", checked("embedding", &embedding));
  m.def("score", checked("score", &score));
  m.def("topk", checked("topk", &topk));
  m.def("score_topk", checked("score_topk", &score_topk));
  m.def("ivf_plan", checked("ivf_plan", &ivf_plan));
  m.def("score_topk_kmax", [](int64_t q) { return (int64_t)nga::score_topk_kmax((int)q); });
  m.def("score_topk_dma_ok", [](int64_t d, int64_t q) { return (bool)nga::score_topk_dma_ok((int)d, (int)q); });
  m.def("pool_l2norm", checked("pool_l2norm", &pool_l2norm));
  m.def("region_marker", checked("region_marker", &region_marker));
  m.def("scatter_segments", checked("scatter_segments", &scatter_segments));
  m.def("host_staging", &host_staging);
  m.def("scatter_host", checked("scatter_host", &scatter_host));
  m.def("row_sqnorm", checked("row_sqnorm", &row_sqnorm));
  m.def("fir_c64", checked("fir_c64", &fir_c64));
  m.def("fm_demod", checked("fm_demod", &fm_demod));
  m.def("resample_pcm", checked("resample_pcm", &resample_pcm));
  m.def("quant_fp8_rows", checked("quant_fp8_rows", &quant_fp8_rows));
  py::class_<CustomAR>(m, "CustomAllReduce")
      .def(py::init<int64_t, int64_t, int64_t, double>(), py::arg("rank"), py::arg("world"),
           py::arg("capacity_bytes"), py::arg("timeout_s") = 5.0)
      .def("handle", &CustomAR::handle)
      .def("open", &CustomAR::open)
      .def("all_reduce", &CustomAR::all_reduce, py::arg("inp"), py::arg("out"), py::arg("algo") = 0)
      .def("all_reduce_add_rmsnorm", &CustomAR::all_reduce_add_rmsnorm)
      .def("all_gather", &CustomAR::all_gather)
      .def("error", &CustomAR::error)
      .def("capacity", &CustomAR::capacity)
      .def("set_two_shot_threshold", &CustomAR::set_two_shot_threshold)
      .def("set_max_blocks", &CustomAR::set_max_blocks)
      .def("max_blocks", &CustomAR::max_blocks);
}
