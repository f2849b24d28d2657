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
// GEMM tile: 256 threads = 4 waves as 2 (weight rows) x 2 (token rows); a block computes
// 128 weight rows x BM token rows, K in steps of 64 staged through XOR-swizzled LDS (the
// ds_read_b128 operand reads of a 16-row MFMA fragment hit 16 distinct 16-B bank slots), the
// next K tile held in registers while the current one is multiplied (issue-early /
// write-late). Weight rows are the MFMA A operand and token rows the B operand, so each lane
// ends with 4 consecutive output features of one token: 8-byte stores, and in MODE 0 the
// gate and up values of the same feature in the same lane — the tile's weight rows are
// ordered [gate f..f+15 | up f..f+15] per 32-row group, read straight from the standard
// [gate rows | up rows] layout by index (no repacked copy of the weights).
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int BN = 128;  // weight rows per block tile
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
template <int BM, int MODE>
__global__ void __launch_bounds__(256) moe_gemm_kernel(MoeGemmParams P) {
  constexpr int MTW = BM / 32;         // 16-row token tiles per wave (wave covers BM / 2 rows)
  constexpr int W_PER_T = BN * 8 / 256;  // 16-B weight chunks per thread per stage (4)
  constexpr int A_PER_T = BM * 8 / 256;  // token chunks per thread per stage (BM / 32)
  __shared__ __attribute__((aligned(16))) uint16_t ws[BN * BK];
  __shared__ __attribute__((aligned(16))) uint16_t as[BM * BK];

  // XCD-aware order (workgroups are dealt round-robin over the 8 XCDs): each XCD gets a
  // contiguous range of (n block, m tile) with m fastest, so the m tiles of one expert that
  // re-read the same weight tile share an L2.
  const int nblk = P.mt * P.nt;
  const int pblk = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, x = pblk % 8;
  const int L = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + pblk / 8;
  const int mti = L % P.mt, nb = L / P.mt;
  const int e = P.tiles[3 * mti];
  if (e < 0) return;
  const int row0 = P.tiles[3 * mti + 1], row1 = P.tiles[3 * mti + 2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = tid >> 6, wn = wv >> 1, wm = wv & 1;
  const int col = lane & 15, h = lane >> 4;
  const uint16_t* We = P.W + (int64_t)e * P.w_rows * P.K;

  // global source rows of this thread's staging chunks (fixed over K)
  const uint16_t* wsrc[W_PER_T];
#pragma unroll
  for (int i = 0; i < W_PER_T; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    int wrow;
    if (MODE == 0) {
      const int f = nb * 64 + (r >> 6) * 32 + ((r >> 5) & 1) * 16 + (r & 15);
      wrow = (r & 16) ? P.F + f : f;
    } else {
      wrow = nb * BN + r;
    }
    wsrc[i] = We + (int64_t)wrow * P.K + ch * 8;
  }
  const uint16_t* asrc[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    int pos = row0 + r;
    if (pos >= row1) pos = row0;   // padding rows of a partial tile: any valid row (not stored)
    const int64_t arow = MODE == 0 ? (int64_t)P.sorted_tok[pos] : (int64_t)pos;
    asrc[i] = P.A + arow * P.lda + ch * 8;
  }

  u16x8 wreg[W_PER_T], areg[A_PER_T];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < W_PER_T; ++i) wreg[i] = load8(wsrc[i] + k0);
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) areg[i] = load8(asrc[i] + k0);
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < W_PER_T; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<u16x8*>(&ws[swz(c >> 3, c & 7)]) = wreg[i];
    }
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<u16x8*>(&as[swz(c >> 3, c & 7)]) = areg[i];
    }
  };

  f32x4 acc[4][MTW];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = (f32x4)(0.f);

  const int nk = P.K / BK;
  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();  // the previous stage's fragment reads are done
    store();
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + h;
      bf16x8 af[4], bf[MTW];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        af[nt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&ws[swz(wn * 64 + nt * 16 + col, ch)]));
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
        bf[mt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&as[swz(wm * (BM / 2) + mt * 16 + col, ch)]));
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = mfma16(af[nt], bf[mt], acc[nt][mt]);
    }
  }

  // epilogue: acc[nt][mt][r] = out[token col][weight row 4h + r] of the 16 x 16 tile
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
    const int pos = row0 + wm * (BM / 2) + mt * 16 + col;
    if (pos >= row1) continue;
    uint16_t* op = P.out + (int64_t)pos * P.ldo;
    if (MODE == 0) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int f = nb * 64 + wn * 32 + g * 16 + 4 * h;
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
      for (int nt = 0; nt < 4; ++nt) {
        const int n = nb * BN + wn * 64 + nt * 16 + 4 * h;
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
