// In-HBM vector search kernels (K13 flat top-k, K14 IVF scan support, K15 k-merge).
//
// score_kernel: S[q, n] = <Q[q], X[n]> (+ per-row bias, e.g. -|x|^2 for L2) in fp32.
//   The batched-query scoring is a skinny GEMM bound by the X stream (2 GB for 1M x 1024
//   bf16): each wave owns 32 index rows (two 16-row MFMA A tiles loaded straight from HBM,
//   16 B per lane, 8 d-steps in flight), the block's <= 64 queries sit in LDS (XOR-swizzled
//   rows) and are the MFMA B operand, so every X byte is read once per 64 queries.
// topk_select_kernel: exact per-segment top-k by a 3-level radix descent on order-preserving
//   float keys (counts in LDS), then a bitonic sort of the <= k survivors. Used twice: per
//   4096-score segment, then once more over the per-segment candidates (the k-merge).
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int SC_QT = 64;    // queries per block
constexpr int SC_ROWS = 128; // index rows per block (32 per wave)
constexpr int SC_KB = 8;     // d-steps (x32) per prefetch batch

__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
}  // namespace

__global__ void __launch_bounds__(256) score_kernel(const uint16_t* __restrict__ Q, int nq,
                                                    const uint16_t* __restrict__ X, int64_t N,
                                                    int D, const float* __restrict__ row_bias,
                                                    float q_bias_scale, float* __restrict__ S,
                                                    float dot_scale) {
  // [16 * ngrp][D] query rows, swizzled 16-B chunks; sized by the launch to the queries
  // actually present (a 1024-d batch of 8 queries stages 32 KB, not 64 x 2 KB), so several
  // blocks share a CU and keep enough X loads in flight to stream HBM
  extern __shared__ __attribute__((aligned(16))) uint16_t q_s[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int q0 = blockIdx.y * SC_QT;
  const int nql = min(SC_QT, nq - q0);
  const int ngrp = (nql + 15) / 16;
  const int nch = D / 8;

  for (int c = tid; c < 16 * ngrp * nch; c += 256) {
    const int r = c / nch, ch = c % nch;
    u16x8 v = (u16x8)(0);
    if (r < nql) v = load8(Q + (int64_t)(q0 + r) * D + ch * 8);
    *reinterpret_cast<u16x8*>(&q_s[r * D + ((ch ^ (r & 15)) * 8)]) = v;
  }
  __syncthreads();

  // blocks stride over 128-row tiles of X, so the query staging above is paid once per
  // block rather than once per tile
  const int64_t ntiles = (N + SC_ROWS - 1) / SC_ROWS;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int64_t row_base = tile * SC_ROWS + w * 32;
  int64_t r0 = row_base + col, r1 = row_base + 16 + col;
  if (r0 >= N) r0 = N - 1;
  if (r1 >= N) r1 = N - 1;
  const uint16_t* x0 = X + r0 * D + 8 * h;
  const uint16_t* x1 = X + r1 * D + 8 * h;

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[i][g] = (f32x4)(0.f);

  const int nsteps = D / 32;
  u16x8 a0[SC_KB], a1[SC_KB];
#pragma unroll
  for (int j = 0; j < SC_KB; ++j) {
    if (j < nsteps) {
      a0[j] = load8(x0 + 32 * j);
      a1[j] = load8(x1 + 32 * j);
    }
  }
  for (int s0 = 0; s0 < nsteps; s0 += SC_KB) {
    u16x8 b0[SC_KB], b1[SC_KB];
    const bool more = s0 + SC_KB < nsteps;
#pragma unroll
    for (int j = 0; j < SC_KB; ++j) {
      if (more && s0 + SC_KB + j < nsteps) {
        b0[j] = load8(x0 + 32 * (s0 + SC_KB + j));
        b1[j] = load8(x1 + 32 * (s0 + SC_KB + j));
      }
    }
#pragma unroll
    for (int j = 0; j < SC_KB; ++j) {
      const int s = s0 + j;
      if (s < nsteps) {
        const int ch = 4 * s + h;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (g < ngrp) {
            const int qr = 16 * g + col;
            bf16x8 bq = as_bf16x8(*reinterpret_cast<const u16x8*>(&q_s[qr * D + ((ch ^ (qr & 15)) * 8)]));
            acc[0][g] = mfma16(as_bf16x8(a0[j]), bq, acc[0][g]);
            acc[1][g] = mfma16(as_bf16x8(a1[j]), bq, acc[1][g]);
          }
        }
      }
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < SC_KB; ++j) {
        a0[j] = b0[j];
        a1[j] = b1[j];
      }
    }
  }
  // acc[i][g]: S^T tile, row (index row) = 4h + r within the 16-row tile, col = query
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t rb = row_base + 16 * i + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int q = 16 * g + col;
      if (g < ngrp && q < nql) {
        float* dst = S + (int64_t)(q0 + q) * N + rb;
        f32x4 v = acc[i][g] * dot_scale;
        if (row_bias) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (rb + r < N) v[r] += row_bias[rb + r];
        }
        if (rb + 3 < N && (N & 3) == 0) {
          *reinterpret_cast<f32x4*>(dst) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (rb + r < N) dst[r] = v[r];
        }
      }
    }
  }
  }  // tile loop
}

// ---------------------------------------------------------------- top-k selection
namespace {
constexpr int TK_NT = 256;
constexpr int TK_BINS = 2048;
constexpr int TK_MAXK = 1024;
}  // namespace

__global__ void __launch_bounds__(TK_NT) topk_select_kernel(
    const float* __restrict__ in, const int64_t* __restrict__ in_idx, int64_t row_len,
    int64_t seg_len, int k, float* __restrict__ out_v, int64_t* __restrict__ out_i) {
  __shared__ uint32_t hist[TK_BINS];
  __shared__ uint32_t scan[TK_NT];
  __shared__ float sv[TK_MAXK];
  __shared__ int64_t si[TK_MAXK];
  __shared__ int sel_bin;
  __shared__ uint32_t sel_above;
  __shared__ uint32_t n_gt, n_eq;

  const int t = threadIdx.x;
  const int64_t row = blockIdx.y, seg = blockIdx.x, nseg = gridDim.x;
  const int64_t beg = seg * seg_len;
  const int64_t end = min(row_len, beg + seg_len);
  const float* x = in + row * row_len;
  const int64_t cnt = end > beg ? end - beg : 0;
  const int kk = (int)min<int64_t>(k, cnt);

  uint32_t prefix = 0, mask = 0;
  if (kk > 0 && kk < cnt) {
    uint32_t remaining = (uint32_t)kk;
    const int shifts[3] = {21, 10, 0};
    const int widths[3] = {11, 11, 10};
    for (int lvl = 0; lvl < 3; ++lvl) {
      for (int i = t; i < TK_BINS; i += TK_NT) hist[i] = 0;
      __syncthreads();
      const int sh = shifts[lvl];
      const uint32_t bm = (1u << widths[lvl]) - 1u;
      for (int64_t i = beg + t; i < end; i += TK_NT) {
        const uint32_t key = okey(x[i]);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> sh) & bm], 1u);
      }
      __syncthreads();
      // thread t owns 8 bins, descending: bins (2047 - 8t) .. (2040 - 8t)
      uint32_t loc[8], mine = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        loc[j] = hist[TK_BINS - 1 - 8 * t - j];
        mine += loc[j];
      }
      scan[t] = mine;
      __syncthreads();
      for (int off = 1; off < TK_NT; off <<= 1) {
        const uint32_t add = t >= off ? scan[t - off] : 0u;
        __syncthreads();
        scan[t] += add;
        __syncthreads();
      }
      const uint32_t incl = scan[t], excl = incl - mine;
      if (excl < remaining && incl >= remaining) {
        uint32_t run = excl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (run + loc[j] >= remaining && run < remaining) {
            sel_bin = TK_BINS - 1 - 8 * t - j;
            sel_above = run;
          }
          run += loc[j];
        }
      }
      __syncthreads();
      remaining -= sel_above;
      prefix |= ((uint32_t)sel_bin) << sh;
      mask |= bm << sh;
      __syncthreads();
    }
  }
  const uint32_t thr = prefix;  // keep key > thr, then fill with key == thr up to kk

  if (t == 0) {
    n_gt = 0;
    n_eq = 0;
  }
  __syncthreads();
  for (int64_t i = beg + t; i < end; i += TK_NT) {
    const float v = x[i];
    const uint32_t key = okey(v);
    if (key > thr || (kk == cnt)) {
      const uint32_t pos = atomicAdd(&n_gt, 1u);
      if (pos < (uint32_t)kk) {
        sv[pos] = v;
        si[pos] = in_idx ? in_idx[row * row_len + i] : i;
      }
    }
  }
  __syncthreads();
  const uint32_t ngt = min(n_gt, (uint32_t)kk);
  if (ngt < (uint32_t)kk) {
    for (int64_t i = beg + t; i < end; i += TK_NT) {
      const float v = x[i];
      if (okey(v) == thr) {
        const uint32_t pos = ngt + atomicAdd(&n_eq, 1u);
        if (pos < (uint32_t)kk) {
          sv[pos] = v;
          si[pos] = in_idx ? in_idx[row * row_len + i] : i;
        }
      }
    }
  }
  __syncthreads();
  // pad to power of two, bitonic sort descending
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = kk + t; i < P; i += TK_NT) {
    sv[i] = -INFINITY;
    si[i] = -1;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < P; i += TK_NT) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = ((i & size) == 0);
          const float a = sv[i], bb = sv[j];
          const bool swap = desc ? (a < bb) : (a > bb);
          if (swap) {
            sv[i] = bb;
            sv[j] = a;
            const int64_t ti = si[i];
            si[i] = si[j];
            si[j] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  float* ov = out_v + (row * nseg + seg) * k;
  int64_t* oi = out_i + (row * nseg + seg) * k;
  for (int i = t; i < k; i += TK_NT) {
    ov[i] = sv[i];
    oi[i] = si[i];
  }
}

void launch_score(const uint16_t* Q, int nq, const uint16_t* X, int64_t N, int D,
                  const float* row_bias, float* S, float dot_scale, hipStream_t stream) {
  if (nq == 0 || N == 0) return;
  const int64_t ntiles = (N + SC_ROWS - 1) / SC_ROWS;
  // ~4 resident blocks per CU on 256 CUs; each strides over ntiles / grid tiles
  const int64_t gx = ntiles < 1024 ? ntiles : 1024;
  dim3 grid((unsigned)gx, (nq + SC_QT - 1) / SC_QT);
  const int qrows = nq >= SC_QT ? SC_QT : ((nq + 15) / 16) * 16;
  const size_t lds = (size_t)qrows * D * sizeof(uint16_t);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)score_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  score_kernel<<<grid, 256, lds, stream>>>(Q, nq, X, N, D, row_bias, 0.f, S, dot_scale);
}

void launch_topk(const float* in, const int64_t* in_idx, int64_t rows, int64_t row_len,
                 int64_t seg_len, int k, float* out_v, int64_t* out_i, hipStream_t stream) {
  if (rows == 0) return;
  const int64_t nseg = (row_len + seg_len - 1) / seg_len;
  dim3 grid((unsigned)nseg, (unsigned)rows);
  topk_select_kernel<<<grid, TK_NT, 0, stream>>>(in, in_idx, row_len, seg_len, k, out_v, out_i);
}

}  // namespace nga
