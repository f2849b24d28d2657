// Sparse mixture-of-experts MLP (Mixtral-8x7B, the reference's default chat model
// ``ai-mixtral-8x7b-instruct``, RetrievalAugmentedGeneration/common/configuration.py:75).
//
//   moe_route    router logits [T, E] -> top-k expert ids + renormalised softmax weights
//   moe_align    per-expert counts, a token order sorted by expert, the inverse map, and a
//                table of M-tiles (expert, first row, end row) for the grouped GEMMs
//   moe_gemm     grouped MFMA GEMM over that table. MODE 0 gathers the token rows of x
//                through the sorted order and multiplies by the expert's [gate | up] rows,
//                with the activation fused in the epilogue (act(gate) * up, never written
//                as [M, 2F]); MODE 1 multiplies the activation rows by the expert's down
//                rows and scales by the routing weight
//   moe_combine  sums each token's top-k rows (fp32) into [T, H]
//
// GEMM: see the block comment above moe_gemm_kernel. Weight rows are the MFMA A operand and
// token rows the B operand, so each lane
// ends with 4 consecutive output features of one token: 8-byte stores, and in MODE 0 the
// gate and up values of the same feature in the same lane — the tile's weight rows are
// ordered [gate f..f+15 | up f..f+15] per 32-row group, read straight from the standard
// [gate rows | up rows] layout by index (no repacked copy of the weights).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int BK = 64;   // K per stage (one 128-B row of bf16)
constexpr int MAX_E = 64;

__device__ __forceinline__ int swz(int row, int ch) {  // 16-B chunk position in a 128-B LDS row
  return row * BK + ((ch ^ ((row >> 1) & 7)) << 3);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x - x / (1.f + __expf(2.f * u));
}
}  // namespace

// ------------------------------------------------------------------ routing
// One thread per token. Softmax over all E experts, top-k, renormalised over the k: the full
// softmax denominator cancels, so the weights are a softmax over the k selected logits.
__global__ void moe_route_kernel(const uint16_t* __restrict__ logits, int64_t ld, int T, int E,
                                 int k, int32_t* __restrict__ ids, float* __restrict__ w) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const uint16_t* lp = logits + (int64_t)t * ld;
  uint64_t taken = 0;
  float top[8];
  int sel[8];
  for (int j = 0; j < k; ++j) {
    float best = -INFINITY;
    int bi = 0;
    for (int e = 0; e < E; ++e) {
      const float v = bf2f(lp[e]);
      if (!((taken >> e) & 1ull) && v > best) {
        best = v;
        bi = e;
      }
    }
    taken |= 1ull << bi;
    top[j] = best;
    sel[j] = bi;
  }
  float s = 0.f;
  for (int j = 0; j < k; ++j) s += __expf(top[j] - top[0]);
  const float inv = 1.f / s;
  for (int j = 0; j < k; ++j) {
    ids[(int64_t)t * k + j] = sel[j];
    w[(int64_t)t * k + j] = __expf(top[j] - top[0]) * inv;
  }
}

// ------------------------------------------------------------------ permutation + tile table
// One workgroup: LDS histogram of the local experts' assignments, an exclusive prefix into row
// offsets, the M-tile table, then every assignment's slot (LDS atomics: the order inside an
// expert is arbitrary, which changes no result — every output row is computed independently
// and combined in fixed top-k order).
__global__ void __launch_bounds__(1024) moe_align_kernel(
    const int32_t* __restrict__ ids, const float* __restrict__ w, int M, int k, int e0, int E,
    int bm, int32_t* __restrict__ sorted_tok, float* __restrict__ sorted_w,
    int32_t* __restrict__ inv, int32_t* __restrict__ tiles, int mt_cap) {
  __shared__ int cnt[MAX_E], off[MAX_E], cur[MAX_E];
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    cnt[e] = 0;
    cur[e] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const int e = ids[i] - e0;
    if (e >= 0 && e < E) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int o = 0, t = 0;
    for (int e = 0; e < E; ++e) {
      off[e] = o;
      for (int r0 = 0; r0 < cnt[e] && t < mt_cap; r0 += bm, ++t) {
        tiles[3 * t] = e;
        tiles[3 * t + 1] = o + r0;
        tiles[3 * t + 2] = o + min(cnt[e], r0 + bm);
      }
      o += cnt[e];
    }
    for (; t < mt_cap; ++t) {
      tiles[3 * t] = -1;
      tiles[3 * t + 1] = 0;
      tiles[3 * t + 2] = 0;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const int e = ids[i] - e0;
    if (e >= 0 && e < E) {
      const int pos = off[e] + atomicAdd(&cur[e], 1);
      sorted_tok[pos] = i / k;
      sorted_w[pos] = w[i];
      inv[i] = pos;
    } else {
      inv[i] = -1;
    }
  }
}

// ------------------------------------------------------------------ grouped GEMM
// Block tile: BN = 256 weight rows x BM token rows (BM = 128 prefill / 64 decode), K in steps
// of 64; 4 waves as 2 (weight rows) x 2 (token rows), each wave 128 x BM/2 (8 x BM/32 MFMA
// tiles: 43 FLOP per LDS byte read at BM = 128, against 32 for a 64 x 64 wave tile). Both
// operands are staged with LDS-DMA (global_load_lds, 16 B per lane) into two stage buffers of
// one __shared__ array: a wave's DMA instruction fills 1 KiB of LDS lane-linearly, so the XOR
// swizzle that keeps the ds_read_b128 fragment reads conflict-free is applied to each lane's
// global SOURCE chunk instead of the LDS address. NSTAGE stage buffers (3 at BM = 128:
// 144 KiB of the CU's 160; the DMA gets two K steps of MFMA time to land, one wave per SIMD
// hides nothing else). One barrier per K step: a counted vmcnt retires this stage's DMA while
// the next stage's stays in flight, a raw s_barrier (no __syncthreads: its fence would drain
// every DMA in flight) makes every wave's DMA visible and guarantees every wave is done with
// the buffer the DMA of stage k + NSTAGE - 1 then refills, and the stage is multiplied.
namespace {
constexpr int GEMM_BN = 256;
}  // namespace

// s_waitcnt vmcnt(N) with a compile-time N (the asm operand must be a literal)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N == 0 || N == 10 || N == 12, "add the count");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

// ABL (diagnostic builds with NGA_DIAG_BUILD=1, picked by NGA_MOE_ABLATE): 1 = no DMA inside
// the K loop (MFMA + LDS-read bound), 2 = no MFMAs (DMA + barrier bound), 3 = no DMA and no LDS
// fragment reads (MFMA + barrier), 4 = no DMA and no barrier; results are wrong in all of them
template <int BM, int MODE, int ABL = 0, int NSTAGE = 3>
__global__ void __launch_bounds__(256) moe_gemm_kernel(MoeGemmParams P) {
  constexpr int BN = GEMM_BN;
  constexpr int MTW = BM / 32;            // 16-row token tiles per wave
  constexpr int NTW = 8;                  // 16-row weight tiles per wave (128 rows)
  constexpr int STAGE = (BN + BM) * BK;   // uint16 elements per stage
  constexpr int W_GL = BN * 8 / 64 / 4;   // DMA instructions per wave per stage, weights (8)
  constexpr int X_GL = BM * 8 / 64 / 4;   // ... tokens (4 / 2)
  constexpr int NPS = W_GL + X_GL;         // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSTAGE * STAGE];

  // XCD-aware order (workgroups are dealt round-robin over the 8 XCDs): each XCD gets a
  // contiguous range of (n block, m tile) with m fastest, so the m tiles of one expert that
  // re-read the same weight tile share an L2.
  const int nblk = P.mt * P.nt;
  const int pblk = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, x8 = pblk % 8;
  const int L = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + pblk / 8;
  const int mti = L % P.mt, nb = L / P.mt;
  const int e = P.tiles[3 * mti];
  if (e < 0) return;
  const int row0 = P.tiles[3 * mti + 1], row1 = P.tiles[3 * mti + 2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = tid >> 6, wn = wv >> 1, wm = wv & 1;
  const int col = lane & 15, h = lane >> 4;
  const uint16_t* We = P.W + (int64_t)e * P.w_rows * P.K;

  // per-lane DMA sources (fixed over K): instruction i of wave wv fills LDS rows
  // [8 (wv * N + i), +8) lane-linearly; lane l lands in row + l/8, physical chunk l%8, which
  // holds logical chunk (l%8) ^ swizzle(row)
  const uint16_t* wsrc[W_GL];
#pragma unroll
  for (int i = 0; i < W_GL; ++i) {
    const int r = (wv * W_GL + i) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((r >> 1) & 7);
    int wrow;
    if (MODE == 0) {   // [gate f..f+15 | up f..f+15] per 32-row group
      const int f = nb * 128 + (r >> 7) * 64 + ((r >> 5) & 3) * 16 + (r & 15);
      wrow = (r & 16) ? P.F + f : f;
    } else {
      wrow = nb * BN + r;
    }
    wsrc[i] = We + (int64_t)wrow * P.K + ch * 8;
  }
  const uint16_t* xsrc[X_GL];
#pragma unroll
  for (int i = 0; i < X_GL; ++i) {
    const int r = (wv * X_GL + i) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((r >> 1) & 7);
    int pos = row0 + r;
    if (pos >= row1) pos = row0;   // padding rows of a partial tile: any valid row (not stored)
    const int64_t arow = MODE == 0 ? (int64_t)P.sorted_tok[pos] : (int64_t)pos;
    xsrc[i] = P.A + arow * P.lda + ch * 8;
  }
  auto issue = [&](int kt, int buf) {
    uint16_t* base = smem + buf * STAGE;
    const int k0 = kt * BK;   // stage index kt (callers clamp it to the last stage)
#pragma unroll
    for (int i = 0; i < W_GL; ++i) glds16(wsrc[i] + k0, base + (wv * W_GL + i) * 8 * BK);
#pragma unroll
    for (int i = 0; i < X_GL; ++i) glds16(xsrc[i] + k0, base + BN * BK + (wv * X_GL + i) * 8 * BK);
  };

  f32x4 acc[NTW][MTW];
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = (f32x4)(0.f);

  const int nk = P.K / BK;
  bf16x8 af[2][NTW], bfr[2][MTW];
  auto read_frags = [&](const uint16_t* ws, int s) {
    const uint16_t* xs = ws + BN * BK;
    const int ch = 4 * s + h;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
      bfr[s][mt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&xs[swz(wm * (BM / 2) + mt * 16 + col, ch)]));
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
      af[s][nt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&ws[swz(wn * 128 + nt * 16 + col, ch)]));
  };
  auto mfmas = [&](int s) {
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = mfma16(af[s][nt], bfr[s][mt], acc[nt][mt]);
  };
  constexpr int NR = NTW + MTW, NM = NTW * MTW;   // reads / MFMAs per k-step

  // (Measured and rejected: reading k-step 0's fragments of the next stage under this stage's
  // k-step-1 MFMAs, with the next stage's barrier moved between the two halves — 1015 ->
  // 1205 us on the Mixtral gate|up GEMM at 1536 tokens.)
#pragma unroll
  for (int st = 0; st < NSTAGE - 1; ++st)
    if (st < nk) issue(st, st);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (this wave's part); the DMA of the next NSTAGE - 2 stages stays in flight
    if (ABL == 1 || ABL >= 3 || NSTAGE == 2 || kt + 1 >= nk) wait_vmcnt<0>();
    else wait_vmcnt<NPS>();
    if (ABL != 4) __builtin_amdgcn_s_barrier();
    if (ABL != 1 && ABL < 3 && kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    if (ABL == 2) continue;
    const uint16_t* ws = smem + (kt % NSTAGE) * STAGE;
    // k-step 0's fragments first; then its MFMAs with k-step 1's reads interleaved (one wave
    // per SIMD: nothing else would hide the LDS latency). hipcc left alone sinks every read
    // next to its first use and waits lgkmcnt(0) every 8 MFMAs.
    if (ABL != 3 || kt == 0) {
      read_frags(ws, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_frags(ws, 1);
    }
    mfmas(0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / 4, 0);   // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, NR / 4, 0);   // DS read
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(1);
  }
  wait_vmcnt<0>();   // no DMA may still target this CU's LDS when the workgroup ends

  // epilogue: acc[nt][mt][r] = out[token col][weight row 4h + r] of the 16 x 16 tile
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
    const int pos = row0 + wm * (BM / 2) + mt * 16 + col;
    if (pos >= row1) continue;
    uint16_t* op = P.out + (int64_t)pos * P.ldo;
    if (MODE == 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int f = nb * 128 + wn * 64 + g * 16 + 4 * h;
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gt = acc[2 * g][mt][r], up = acc[2 * g + 1][mt][r];
          v[r] = f2bf((P.act == 0 ? silu(gt) : gelu_tanh(gt)) * up);
        }
        *reinterpret_cast<u16x4*>(op + f) = v;
      }
    } else {
      const float sc = P.sorted_w[pos];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n = nb * BN + wn * 128 + nt * 16 + 4 * h;
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(acc[nt][mt][r] * sc);
        *reinterpret_cast<u16x4*>(op + n) = v;
      }
    }
  }
}

// ------------------------------------------------------------------ combine
// out[t, :] = sum_j y[inv[t*k + j], :] (fp32), 8 features per thread
__global__ void moe_combine_kernel(const uint16_t* __restrict__ y, const int32_t* __restrict__ inv,
                                   int T, int k, int H, uint16_t* __restrict__ out) {
  const int64_t vec = H / 8;
  const int64_t total = (int64_t)T * vec;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / vec;
    const int c = (int)(i - t * vec) * 8;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int p = inv[t * k + j];
      if (p < 0) continue;
      const u16x8 v = load8(y + (int64_t)p * H + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] += bf2f(v[q]);
    }
    u16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(a[q]);
    store8(out + t * H + c, o);
  }
}

// ------------------------------------------------------------------ launchers
void launch_moe_route(const uint16_t* logits, int64_t ld, int T, int E, int k, int32_t* ids,
                      float* w, hipStream_t stream) {
  if (T == 0) return;
  moe_route_kernel<<<(T + 255) / 256, 256, 0, stream>>>(logits, ld, T, E, k, ids, w);
}

void launch_moe_align(const int32_t* ids, const float* w, int M, int k, int e0, int E, int bm,
                      int32_t* sorted_tok, float* sorted_w, int32_t* inv, int32_t* tiles,
                      int mt_cap, hipStream_t stream) {
  moe_align_kernel<<<1, 1024, 0, stream>>>(ids, w, M, k, e0, E, bm, sorted_tok, sorted_w, inv,
                                            tiles, mt_cap);
}

void launch_moe_gemm(const MoeGemmParams& p, int bm, int mode, hipStream_t stream) {
  const int nblk = p.mt * p.nt;
  if (nblk == 0) return;
  dim3 grid(nblk);
#ifdef NGA_DIAG_ABLATION  // diagnostic builds only (NGA_DIAG_BUILD=1): timings, not results
  static const int ablate = [] {
    const char* e = getenv("NGA_MOE_ABLATE");
    return e ? atoi(e) : 0;
  }();
  if (mode == 0 && bm == 128 && ablate >= 1 && ablate <= 5) {
    if (ablate == 5) moe_gemm_kernel<128, 0, 0, 2><<<grid, 256, 0, stream>>>(p);   // 2-stage
    else if (ablate == 1) moe_gemm_kernel<128, 0, 1><<<grid, 256, 0, stream>>>(p);
    else if (ablate == 2) moe_gemm_kernel<128, 0, 2><<<grid, 256, 0, stream>>>(p);
    else if (ablate == 3) moe_gemm_kernel<128, 0, 3><<<grid, 256, 0, stream>>>(p);
    else moe_gemm_kernel<128, 0, 4><<<grid, 256, 0, stream>>>(p);
    return;
  }
#endif
  if (mode == 0) {
    if (bm == 64) moe_gemm_kernel<64, 0><<<grid, 256, 0, stream>>>(p);
    else moe_gemm_kernel<128, 0><<<grid, 256, 0, stream>>>(p);
  } else {
    if (bm == 64) moe_gemm_kernel<64, 1><<<grid, 256, 0, stream>>>(p);
    else moe_gemm_kernel<128, 1><<<grid, 256, 0, stream>>>(p);
  }
}

void launch_moe_combine(const uint16_t* y, const int32_t* inv, int T, int k, int H, uint16_t* out,
                        hipStream_t stream) {
  if (T == 0) return;
  int64_t g = ((int64_t)T * H / 8 + 255) / 256;
  if (g > 4096) g = 4096;
  moe_combine_kernel<<<(unsigned)g, 256, 0, stream>>>(y, inv, T, k, H, out);
}

}  // namespace nga
