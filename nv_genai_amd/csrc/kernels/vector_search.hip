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
#include <cstdlib>

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

// ---------------------------------------------------------------- fused score + top-k
// score_topk_kernel: the score kernel's MFMA stream with the top-k folded in, so no [nq, N]
// score matrix ever reaches HBM (only [queries, blocks, k] candidates).
//
// Work items (blockIdx.y): a row range of X plus up to 64 query slots. Flat search: one item
// per 64-query chunk over all rows. IVF: one item per (inverted list, 64-query chunk) over the
// list's contiguous rows, the slots holding the queries that probe that list (``qtab``), so a
// list is streamed once for every query that probes it. Blocks of an item (blockIdx.x) stride
// over its 32W-row tiles.
//
// Per lane and query group: a register top-K (descending, branch-free insertion) of the
// scores that lane produced (a 16x16 MFMA tile gives lane (col, h) rows 4h..4h+3 of query
// col). End of block: the 4 lanes of a query merge their lists through two xor-shuffle
// bitonic merges, the W waves' lists meet in LDS (the query tile's space, free by then) and
// one thread per query keeps the block's top k.
namespace {
template <int K>
__device__ __forceinline__ void tk_insert(float (&v)[K], int (&r)[K], float x, int row) {
  float cv = x;
  int cr = row;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const bool sw = cv > v[j];
    const float tv = v[j];
    const int tr = r[j];
    v[j] = sw ? cv : tv;
    r[j] = sw ? cr : tr;
    cv = sw ? tv : cv;
    cr = sw ? tr : cr;
  }
}

// (v, r) := top K of itself and the list held by lane ^ mask (both sorted descending)
template <int K>
__device__ __forceinline__ void tk_merge_xor(float (&v)[K], int (&r)[K], int mask) {
  float ov[K];
  int orr[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    ov[j] = __shfl_xor(v[j], mask, 64);
    orr[j] = __shfl_xor(r[j], mask, 64);
  }
  // max(a[j], b[K-1-j]) is bitonic and holds the top K of both; a half-cleaner cascade sorts it
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const bool tb = ov[K - 1 - j] > v[j];
    v[j] = tb ? ov[K - 1 - j] : v[j];
    r[j] = tb ? orr[K - 1 - j] : r[j];
  }
#pragma unroll
  for (int st = K / 2; st > 0; st >>= 1) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if ((j & st) == 0) {
        const bool sw = v[j + st] > v[j];
        const float a = v[j], b = v[j + st];
        const int ra = r[j], rb = r[j + st];
        v[j] = sw ? b : a;
        v[j + st] = sw ? a : b;
        r[j] = sw ? rb : ra;
        r[j + st] = sw ? ra : rb;
      }
    }
  }
}
}  // namespace

template <int NG, int W, int K>
__global__ void __launch_bounds__(64 * W) score_topk_kernel(
    const uint16_t* __restrict__ Q, int nq, const uint16_t* __restrict__ X, int64_t N, int D,
    const float* __restrict__ row_bias, float dot_scale, const int64_t* __restrict__ row_beg,
    const int64_t* __restrict__ row_end, const int32_t* __restrict__ qtab,
    const int32_t* __restrict__ slot_rows, int k, float* __restrict__ out_v, int64_t* __restrict__ out_r) {
  // X is streamed exactly once; non-temporal loads of it measured no faster than the default
  // policy (1M x 1024, 1 / 8 / 64 queries: 364.1 / 367.4 / 421.7 vs 364.8 / 366.7 / 420.9 us,
  // profiles/r3_search_dma/kb_search.json) and were removed
  auto xload = [](const uint16_t* p) -> u16x8 { return load8(p); };
  extern __shared__ __attribute__((aligned(16))) uint16_t q_s[];
  __shared__ int s_nql;
  constexpr int ROWS = 32 * W;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int item = blockIdx.y;
  const int nch = D / 8;
  const int64_t beg = row_beg ? row_beg[item] : 0;
  const int64_t end = row_end ? row_end[item] : N;
  const int nblk = gridDim.x;

  // query slot -> query index (-1: empty)
  auto slot_q = [&](int s) -> int {
    if (qtab) return qtab[item * 64 + s];
    const int q = item * 64 + s;
    return q < nq ? q : -1;
  };
  if (tid == 0) s_nql = 0;
  __syncthreads();
  if (tid < 64 && slot_q(tid) >= 0) atomicMax(&s_nql, tid + 1);
  __syncthreads();
  const int nql = s_nql;
  // candidate row of a slot: the slot itself (flat), or the (query, probe) pair it serves
  // (IVF: candidates land in [nq * nprobe, nblk, k] order, -1 = unused slot)
  auto slot_row = [&](int s) -> int64_t {
    return slot_rows ? (int64_t)slot_rows[item * 64 + s] : (int64_t)item * 64 + s;
  };
  if (nql == 0 || end <= beg) {
    // nothing to scan: every used slot still reports k empty candidates
    for (int i = tid; i < 64 * k; i += 64 * W) {
      const int s = i / k, j = i % k;
      const int64_t cr = slot_row(s);
      if (cr < 0) continue;
      const int64_t o = (cr * nblk + blockIdx.x) * k + j;
      out_v[o] = -INFINITY;
      out_r[o] = -1;
    }
    return;
  }
  const int ngrp = min(NG, (nql + 15) / 16);

  for (int c = tid; c < 16 * NG * nch; c += 64 * W) {
    const int r = c / nch, ch = c % nch;
    u16x8 v = (u16x8)(0);
    const int q = r < nql ? slot_q(r) : -1;
    if (q >= 0) v = load8(Q + (int64_t)q * D + ch * 8);
    *reinterpret_cast<u16x8*>(&q_s[r * D + ((ch ^ (r & 15)) * 8)]) = v;
  }
  __syncthreads();

  float tv[NG][K];
  int tr[NG][K];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int j = 0; j < K; ++j) {
      tv[g][j] = -INFINITY;
      tr[g][j] = -1;
    }

  const int64_t ntiles = (end - beg + ROWS - 1) / ROWS;
  const int nsteps = D / 32;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += nblk) {
    const int64_t row_base = beg + tile * ROWS + w * 32;
    int64_t r0 = row_base + col, r1 = row_base + 16 + col;
    if (r0 >= end) r0 = end - 1;
    if (r1 >= end) r1 = end - 1;
    const uint16_t* x0 = X + r0 * D + 8 * h;
    const uint16_t* x1 = X + r1 * D + 8 * h;

    f32x4 acc[2][NG];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[i][g] = (f32x4)(0.f);

    u16x8 a0[SC_KB], a1[SC_KB];
#pragma unroll
    for (int j = 0; j < SC_KB; ++j) {
      if (j < nsteps) {
        a0[j] = xload(x0 + 32 * j);
        a1[j] = xload(x1 + 32 * j);
      }
    }
    for (int s0 = 0; s0 < nsteps; s0 += SC_KB) {
      u16x8 b0[SC_KB], b1[SC_KB];
      const bool more = s0 + SC_KB < nsteps;
#pragma unroll
      for (int j = 0; j < SC_KB; ++j) {
        if (more && s0 + SC_KB + j < nsteps) {
          b0[j] = xload(x0 + 32 * (s0 + SC_KB + j));
          b1[j] = xload(x1 + 32 * (s0 + SC_KB + j));
        }
      }
#pragma unroll
      for (int j = 0; j < SC_KB; ++j) {
        const int s = s0 + j;
        if (s < nsteps) {
          const int ch = 4 * s + h;
#pragma unroll
          for (int g = 0; g < NG; ++g) {
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
    // acc[i][g][rr]: index row row_base + 16 i + 4 h + rr, query slot 16 g + col
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t rb = row_base + 16 * i + 4 * h;
      float bias[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        bias[rr] = (row_bias && rb + rr < end) ? row_bias[rb + rr] : 0.f;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (g < ngrp) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const float sc = acc[i][g][rr] * dot_scale + bias[rr];
            if (rb + rr < end && sc > tv[g][K - 1]) tk_insert<K>(tv[g], tr[g], sc, (int)(rb + rr));
          }
        }
      }
    }
  }

  // the 4 lanes (h = 0..3) of each query column merge their lists
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (g < ngrp) {
      tk_merge_xor<K>(tv[g], tr[g], 16);
      tk_merge_xor<K>(tv[g], tr[g], 32);
    }
  }
  __syncthreads();   // every wave is done with the query tile: its LDS holds the wave lists now
  float* mv = reinterpret_cast<float*>(q_s);                 // [64 slots][W][K]
  int* mr = reinterpret_cast<int*>(mv + 64 * W * K);
  if (h == 0) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g < ngrp) {
        const int sl = 16 * g + col;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          mv[(sl * W + w) * K + j] = tv[g][j];
          mr[(sl * W + w) * K + j] = tr[g][j];
        }
      }
    }
  }
  __syncthreads();
  if (tid < 64 && slot_row(tid) >= 0) {
    const int sl = tid;
    const int64_t o = (slot_row(sl) * nblk + blockIdx.x) * k;
    if (sl >= nql || slot_q(sl) < 0) {
      for (int j = 0; j < k; ++j) {
        out_v[o + j] = -INFINITY;
        out_r[o + j] = -1;
      }
    } else {
      int head[W];
#pragma unroll
      for (int u = 0; u < W; ++u) head[u] = 0;
      for (int j = 0; j < k; ++j) {
        float best = -INFINITY;
        int bu = -1;
#pragma unroll
        for (int u = 0; u < W; ++u) {
          const float x = head[u] < K ? mv[(sl * W + u) * K + head[u]] : -INFINITY;
          if (x > best) {
            best = x;
            bu = u;
          }
        }
        int row = -1;
        if (bu >= 0) {
#pragma unroll
          for (int u = 0; u < W; ++u)
            if (u == bu) {
              row = mr[(sl * W + u) * K + head[u]];
              ++head[u];
            }
        }
        out_v[o + j] = best;
        out_r[o + j] = row;
      }
    }
  }
}

// LDS-DMA form for items of <= 16 queries (one query group) and D a multiple of CH. The
// register form above loads its MFMA fragments straight from HBM: a wave instruction reads
// 16 rows x 64 B, half of each 128-B line, an order that tops out near 5.9 TB/s (and whose
// non-temporal variant re-fetches lines: 4.4 TB/s); lane-linear 1-KiB LDS-DMA reaches
// 6.5-6.8 TB/s non-temporal (scripts/dev/read_bw_probe.hip, profiles/r3_bw/read_bw.json).
// Here each wave owns a 32-row x CH-dim LDS slot. A unit of work is one CH-dim chunk of the
// wave's 32 rows: the wave waits for its unit's DMA, reads every fragment of it into
// registers, issues the next unit's DMA into the same slot, then runs the MFMAs against the
// query tile (LDS) and, after a row tile's last chunk, the register top-k insert. A wave only
// touches its own slot: no barrier in the loop. 4 x 32 KiB slots + the query tile fill the
// CU's LDS: one workgroup per CU, so the launcher sizes the grid to the CU count.
namespace {
__device__ __forceinline__ int stk_swz(int row) { return row & 15; }
}  // namespace

template <int K, int CH>
__global__ void __launch_bounds__(256, 1) score_topk_dma_kernel(
    const uint16_t* __restrict__ Q, int nq, const uint16_t* __restrict__ X, int64_t N, int D,
    const float* __restrict__ row_bias, float dot_scale, const int64_t* __restrict__ row_beg,
    const int64_t* __restrict__ row_end, const int32_t* __restrict__ qtab,
    const int32_t* __restrict__ slot_rows, int k, float* __restrict__ out_v, int64_t* __restrict__ out_r) {
  constexpr int W = 4, ROWS = 32 * W;
  constexpr int SLOT = 32 * CH;          // elements of one wave's slot
  constexpr int NC = CH / 8;             // 16-B positions per row chunk (64 or 32)
  constexpr int RPI = 64 / NC;           // rows per 1-KiB DMA instruction (1 or 2)
  constexpr int NI = 32 / RPI;           // DMA instructions per unit
  constexpr int NS = CH / 32;            // MFMA k-steps per unit
  // ONE LDS object: [W] slots, then the query tile [16][D]; the block merge reuses it
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* const q_s = smem + W * SLOT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int item = blockIdx.y;
  const int64_t beg = row_beg ? row_beg[item] : 0;
  const int64_t end = row_end ? row_end[item] : N;
  const int nblk = gridDim.x;
  const int nch = D / 8;
  auto slot_q = [&](int s) -> int {
    if (qtab) return qtab[item * 64 + s];
    const int q = item * 64 + s;
    return q < nq ? q : -1;
  };
  auto slot_row = [&](int s) -> int64_t {
    return slot_rows ? (int64_t)slot_rows[item * 64 + s] : (int64_t)item * 64 + s;
  };
  // used query slots: every wave computes it from a ballot (no LDS scalar: the slots and the
  // query tile take all 160 KiB)
  const unsigned long long used = __ballot(slot_q(lane) >= 0);
  const int nql = used ? 64 - __clzll((long long)used) : 0;
  if (nql == 0 || end <= beg) {
    for (int i = tid; i < 64 * k; i += 256) {
      const int s = i / k, j = i % k;
      const int64_t cr = slot_row(s);
      if (cr < 0) continue;
      const int64_t o = (cr * nblk + blockIdx.x) * k + j;
      out_v[o] = -INFINITY;
      out_r[o] = -1;
    }
    return;
  }

  uint16_t* const slot = smem + w * SLOT;
  const int64_t ntiles = (end - beg + ROWS - 1) / ROWS;
  const int nchx = D / CH;
  float bnext[2][4], bcur[2][4];
  // unit (tile, chunk) -> this wave's slot; DMA instruction i fills slot bytes [1 KiB i, +1 KiB):
  // rows RPI i .. (lane: row RPI i + lane / NC, position lane % NC holding logical 16-B chunk
  // (lane % NC) ^ swz(row)). With chunk 0 of a tile the tile's row biases are loaded too, so
  // they are in registers long before its top-k (a bias load after the DMA would be waited
  // for together with it).
  auto issue = [&](int64_t tile, int c) {
    const int64_t rbase = beg + tile * ROWS + w * 32;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int row = RPI * i + lane / NC;
      int64_t gr = rbase + row;
      if (gr >= end) gr = end - 1;
      const uint16_t* src = X + gr * D + c * CH + (((lane % NC) ^ stk_swz(row)) << 3);
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(slot + i * 512), 16, 0, 2);
    }
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int64_t r = rbase + 16 * i + 4 * h + rr;
          bnext[i][rr] = (row_bias && r < end) ? row_bias[r] : 0.f;
        }
    }
  };
  int64_t t = blockIdx.x;
  int c = 0;
  if (t < ntiles) issue(t, 0);
  // query tile after the first DMA (its wait is the first unit's anyway)
  for (int i = tid; i < 16 * nch; i += 256) {
    const int r = i / nch, ch = i % nch;
    u16x8 v = (u16x8)(0);
    const int q = r < nql ? slot_q(r) : -1;
    if (q >= 0) v = load8(Q + (int64_t)q * D + ch * 8);
    *reinterpret_cast<u16x8*>(&q_s[r * D + ((ch ^ (r & 15)) * 8)]) = v;
  }
  __syncthreads();

  float tv[K];
  int tr[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    tv[j] = -INFINITY;
    tr[j] = -1;
  }
  f32x4 acc[2] = {(f32x4)(0.f), (f32x4)(0.f)};
  while (t < ntiles) {
    int c2 = c + 1;
    int64_t t2 = t;
    if (c2 == nchx) {
      c2 = 0;
      t2 = t + nblk;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) bcur[i][rr] = bnext[i][rr];
    }
    u16x8 a[2][NS];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < NS; ++s)
        a[i][s] = *reinterpret_cast<const u16x8*>(slot + (16 * i + col) * CH + (((4 * s + h) ^ col) << 3));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot is free: next unit's DMA
    if (t2 < ntiles) issue(t2, c2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int ch = c * NC + 4 * s + h;
      const bf16x8 bq = as_bf16x8(*reinterpret_cast<const u16x8*>(&q_s[col * D + ((ch ^ col) << 3)]));
      acc[0] = mfma16(as_bf16x8(a[0][s]), bq, acc[0]);
      acc[1] = mfma16(as_bf16x8(a[1][s]), bq, acc[1]);
    }
    if (c == nchx - 1) {
      // acc[i][rr]: row tile_base + 16 i + 4 h + rr, query slot col
      const int64_t rbase = beg + t * ROWS + w * 32;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int64_t rb = rbase + 16 * i + 4 * h;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const float sc = acc[i][rr] * dot_scale + bcur[i][rr];
          if (rb + rr < end && sc > tv[K - 1]) tk_insert<K>(tv, tr, sc, (int)(rb + rr));
        }
        acc[i] = (f32x4)(0.f);
      }
    }
    t = t2;
    c = c2;
  }

  tk_merge_xor<K>(tv, tr, 16);
  tk_merge_xor<K>(tv, tr, 32);
  __syncthreads();   // every wave is past its last DMA wait and done with the query tile
  float* mv = reinterpret_cast<float*>(smem);                 // [16 slots][W][K]
  int* mr = reinterpret_cast<int*>(mv + 16 * W * K);
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      mv[(col * W + w) * K + j] = tv[j];
      mr[(col * W + w) * K + j] = tr[j];
    }
  }
  __syncthreads();
  if (tid < 64 && slot_row(tid) >= 0) {
    const int sl = tid;
    const int64_t o = (slot_row(sl) * nblk + blockIdx.x) * k;
    if (sl >= nql || sl >= 16 || slot_q(sl) < 0) {
      for (int j = 0; j < k; ++j) {
        out_v[o + j] = -INFINITY;
        out_r[o + j] = -1;
      }
    } else {
      int head[W];
#pragma unroll
      for (int u = 0; u < W; ++u) head[u] = 0;
      for (int j = 0; j < k; ++j) {
        float best = -INFINITY;
        int bu = -1;
#pragma unroll
        for (int u = 0; u < W; ++u) {
          const float x = head[u] < K ? mv[(sl * W + u) * K + head[u]] : -INFINITY;
          if (x > best) {
            best = x;
            bu = u;
          }
        }
        int row = -1;
        if (bu >= 0) {
#pragma unroll
          for (int u = 0; u < W; ++u)
            if (u == bu) {
              row = mr[(sl * W + u) * K + head[u]];
              ++head[u];
            }
        }
        out_v[o + j] = best;
        out_r[o + j] = row;
      }
    }
  }
}

int score_topk_kmax(int nq_per_item) { return nq_per_item <= 32 ? 16 : 8; }

int score_topk_dma_ok(int D, int max_q_per_item) {
  return kernel_form(KF_SEARCH_DMA) != 0 && max_q_per_item <= 16 && D % 256 == 0 && D >= 256 && D <= 2048;
}

void launch_score_topk(const uint16_t* Q, int nq, const uint16_t* X, int64_t N, int D,
                       const float* row_bias, float dot_scale, const int64_t* row_beg,
                       const int64_t* row_end, const int32_t* qtab, const int32_t* slot_rows, int n_items,
                       int max_q_per_item, int nblk, int k, float* out_v, int64_t* out_r, hipStream_t stream) {
  if (n_items == 0 || nblk == 0) return;
  if (score_topk_dma_ok(D, max_q_per_item)) {
    const int ch = (D % 512 == 0 && D <= 1024) ? 512 : 256;
    const size_t lds = (size_t)(4 * 32 * ch + 16 * D) * sizeof(uint16_t);
    const int KR = k <= 4 ? 4 : k <= 8 ? 8 : 16;
    dim3 grid((unsigned)nblk, (unsigned)n_items);
#define NGA_STKD(K_, CH_)                                                                       \
  do {                                                                                           \
    static bool attr_ = false;                                                                   \
    if (!attr_) {                                                                                \
      (void)hipFuncSetAttribute((const void*)score_topk_dma_kernel<K_, CH_>,                     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);         \
      (void)hipGetLastError();                                                                   \
      attr_ = true;                                                                              \
    }                                                                                            \
    score_topk_dma_kernel<K_, CH_><<<grid, 256, lds, stream>>>(Q, nq, X, N, D, row_bias,         \
                                                               dot_scale, row_beg, row_end,      \
                                                               qtab, slot_rows, k, out_v, out_r); \
  } while (0)
    if (ch == 512) {
      if (KR == 4) NGA_STKD(4, 512); else if (KR == 8) NGA_STKD(8, 512); else NGA_STKD(16, 512);
    } else {
      if (KR == 4) NGA_STKD(4, 256); else if (KR == 8) NGA_STKD(8, 256); else NGA_STKD(16, 256);
    }
#undef NGA_STKD
    return;
  }
  const int ng = max_q_per_item <= 16 ? 1 : max_q_per_item <= 32 ? 2 : 4;
  const int W = ng == 4 ? 8 : 4;
  const int KR = k <= 4 ? 4 : k <= 8 ? 8 : 16;
  const size_t qs = (size_t)16 * ng * D * sizeof(uint16_t);
  const size_t mg = (size_t)64 * W * KR * 8;
  const size_t lds = qs > mg ? qs : mg;
  dim3 grid((unsigned)nblk, (unsigned)n_items);
#define NGA_STK(NG_, W_, K_)                                                                    \
  do {                                                                                           \
    static bool attr_ = false;                                                                   \
    if (!attr_) {                                                                                \
      /* 160 KiB of LDS minus the kernel's static s_nql */                                     \
      (void)hipFuncSetAttribute((const void*)score_topk_kernel<NG_, W_, K_>,                     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 64);    \
      (void)hipGetLastError();                                                                   \
      attr_ = true;                                                                              \
    }                                                                                            \
    score_topk_kernel<NG_, W_, K_><<<grid, 64 * W_, lds, stream>>>(Q, nq, X, N, D, row_bias,     \
                                                                   dot_scale, row_beg, row_end,  \
                                                                   qtab, slot_rows, k, out_v,    \
                                                                   out_r);                       \
  } while (0)
  if (ng == 1) {
    if (KR == 4) NGA_STK(1, 4, 4); else if (KR == 8) NGA_STK(1, 4, 8); else NGA_STK(1, 4, 16);
  } else if (ng == 2) {
    if (KR == 4) NGA_STK(2, 4, 4); else if (KR == 8) NGA_STK(2, 4, 8); else NGA_STK(2, 4, 16);
  } else {
    if (KR == 4) NGA_STK(4, 8, 4); else NGA_STK(4, 8, 8);
  }
#undef NGA_STK
}

// ---------------------------------------------------------------- IVF scan plan
// One block groups the (query, probe) pairs by inverted list: pair i = (q = i / nprobe,
// list p) takes slot rank % 64 of work item p * chunks + rank / 64, rank = its arrival
// order among list p's pairs (LDS atomics). qtab[slot] = q, slot_rows[slot] = i; untouched
// slots stay -1. nlist <= IVF_PLAN_MAX_LISTS.
__global__ void __launch_bounds__(1024) ivf_plan_kernel(const int64_t* __restrict__ probes, int npairs,
                                                        int nprobe, int nlist, int chunks,
                                                        int32_t* __restrict__ qtab,
                                                        int32_t* __restrict__ slot_rows) {
  __shared__ int cnt[IVF_PLAN_MAX_LISTS];
  const int t = threadIdx.x;
  const int nslots = nlist * chunks * 64;
  for (int i = t; i < nlist; i += 1024) cnt[i] = 0;
  for (int i = t; i < nslots; i += 1024) {
    qtab[i] = -1;
    slot_rows[i] = -1;
  }
  __syncthreads();
  for (int i = t; i < npairs; i += 1024) {
    const int64_t p = probes[i];
    if (p < 0 || p >= nlist) continue;   // a short coarse top-k pads with -1
    const int rank = atomicAdd(&cnt[p], 1);
    if (rank >= chunks * 64) continue;   // cannot happen: a list has <= nq probing queries
    const int slot = ((int)p * chunks + rank / 64) * 64 + rank % 64;
    qtab[slot] = i / nprobe;
    slot_rows[slot] = i;
  }
}

void launch_ivf_plan(const int64_t* probes, int nq, int nprobe, int nlist, int32_t* qtab,
                     int32_t* slot_rows, hipStream_t stream) {
  const int chunks = (nq + 63) / 64;
  ivf_plan_kernel<<<1, 1024, 0, stream>>>(probes, nq * nprobe, nprobe, nlist, chunks, qtab, slot_rows);
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
