// Prefill attention, 32x32 MFMA form (K1 causal-GQA over the paged KV cache, head_dim 128).
//
// Why a second kernel: attention_prefill.hip gives every wave 16 query rows (16x16x32 MFMA),
// so each K / V^T fragment it reads from LDS feeds one MFMA — per key tile a 4-wave workgroup
// reads 128 KiB of LDS for 2 MFLOP, which is as many LDS cycles (256 B/clk/CU) as MFMA cycles,
// and the softmax VALU comes on top (≈535 TF). Here a wave owns 32 query rows and uses
// mfma_f32_32x32x16_bf16: the same fragment bytes feed twice the FLOPs.
//
// Layout per wave and 64-key tile (lane l, r = l & 31, h = l >> 5):
//   S^T[key][q] = K . Q^T   — 2 key sub-tiles x 8 d-steps. A = K rows read from LDS, B = Q^T
//                             held in registers for the whole kernel (qf[8]). The K row a
//                             lane supplies for MFMA row i is perm(i) (bits 2 and 3 swapped),
//                             which makes accumulator register j of a lane hold key
//                             (j & 7) + 8h + 16 (j >> 3) of the sub-tile: 8 contiguous keys
//                             per register half, exactly the P^T operand order below.
//   online softmax per query column (exp2 domain, lazy rescale as in the 16x16 kernel); the
//   row max is 31 fmax in-lane + one exchange with lane l ^ 32.
//   O^T[d][q] += V^T . P^T  — 4 d-tiles x 4 key-steps. A = V^T rows (keys contiguous in the
//                             paged Vt cache), B = the bf16 P accumulator registers, no lane
//                             movement.
// Workgroup = 4 waves sharing each K / V^T tile: with G = Hq / Hkv a multiple of 4 the waves
// are the 4 query heads of one GQA group over the same 32 positions (identical causal range,
// no wave runs ahead of another's diagonal), otherwise 4 row blocks (or 2 x 2) of one head.
// Tiles arrive by LDS-DMA (global_load_lds, 8 x 16 B per lane per tile), XOR-swizzled through
// the source address so the fragment reads are bank-conflict-free, double-buffered: the DMA of
// tile t + 1 is issued right after the barrier that opens tile t and has the whole tile's MFMA
// time to land. 64 KiB of LDS per workgroup -> 2 workgroups (2 waves per SIMD) per CU.
//
// Paged layout as attention_prefill.hip: K [blocks, Hkv, 64, 128], V^T [blocks, Hkv, 128, 64];
// queries are the last q_len positions of a ctx_len context. Sliding window via P.window.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr float V2_LOG2E = 1.4426950408889634f;
constexpr float V2_RESCALE_LOG2 = 8.f;
constexpr int V2_MAX_TILES = 1024;   // block-table entries staged in LDS (64K-token contexts)

// 16-B chunk swizzle of a 128-element K row: 4 bits of the row, distinct over the 16 rows of
// every ds_read_b128 lane group of the perm()-ed row order
__device__ __forceinline__ int kswz(int row) { return (row & 3) | (((row >> 3) & 3) << 2); }
// 16-B chunk swizzle of a 64-key V^T row
__device__ __forceinline__ int vswz(int row) { return (row >> 1) & 7; }
}  // namespace

// ABL (diagnostic, NGA_PV2_ABLATE; results are wrong): 1 = no DMA inside the loop, 2 = no
// compute, 3 = no softmax (P = S), 4 = no DMA and no barrier inside the loop
template <bool CAUSAL, int HPW, int ABL = 0>
__global__ void __launch_bounds__(256, 2) prefill_attn_v2_kernel(PrefillParams P) {
  constexpr int D = 128, KT = 64;
  constexpr int TILE = KT * D;          // elements of one K (or V^T) tile: 16 KiB
  constexpr int RB = 4 / HPW;           // 32-row query blocks per workgroup
  constexpr int RW = 32 * RB;           // query rows per workgroup
  // ONE LDS object: [buffer 0: K | V^T][buffer 1: K | V^T][block ids of the sequence].
  // (With several LDS variables the compiler gives their accesses alias scopes and then waits
  // vmcnt(0) before fragment reads of a buffer whose earlier DMA it cannot see retired —
  // serialising the prefetch; a VMEM block-table load inside the loop did the same.)
  __shared__ __attribute__((aligned(16))) uint16_t smem[4 * TILE + 2 * V2_MAX_TILES];
  int32_t* sbt = reinterpret_cast<int32_t*>(smem + 4 * TILE);

  // XCD-aware order (as the 16x16 kernel): each XCD gets a contiguous range of
  // (sequence, kv head, head group, query block), longest causal blocks first.
  const int pblk = blockIdx.x;
  const int L = (pblk & 7) * P.per_xcd + (pblk >> 3);
  if (L >= P.total) return;
  const int G = P.Hq / P.Hkv;
  const int ngrp = G / HPW;
  const int qb = P.ntiles - 1 - L % P.ntiles;
  const int hg = (L / P.ntiles) % (P.Hkv * ngrp);
  const int b = L / (P.ntiles * P.Hkv * ngrp);
  const int q0 = P.cu_q[b], qlen = P.cu_q[b + 1] - q0;
  if (qb * RW >= qlen) return;
  const int ctx = P.ctx_lens[b];
  const int kvh = hg / ngrp;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hq = kvh * G + (hg % ngrp) * HPW + w % HPW;
  const int rb = w / HPW;
  const int r32 = lane & 31, h = lane >> 5;

  // this lane's query row (a column of the S^T / O^T tiles)
  const int row_first = qb * RW + rb * 32;       // wave-uniform
  const bool wave_active = row_first < qlen;
  int qr = row_first + r32;
  const bool row_ok = qr < qlen;
  if (!row_ok) qr = qlen - 1;
  const int qpos = ctx - qlen + qr;
  const int qmin_w = ctx - qlen + row_first;                       // wave's first query position
  const int qmax_w = ctx - qlen + min(qlen - 1, row_first + 31);   // and its last
  const int W = CAUSAL ? P.window : 0;

  bf16x8 qf[8];
  {
    const uint16_t* qp = P.q + (int64_t)(q0 + qr) * P.q_stride + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = as_bf16x8(load8(qp + 16 * s));
  }

  // tile range of the workgroup
  const int last_key = CAUSAL ? ctx - qlen + min(qlen - 1, qb * RW + RW - 1) : ctx - 1;
  const int n_tiles = last_key / KT + 1;
  const int t_first = W > 0 ? max(0, ctx - qlen + qb * RW - W + 1) / KT : 0;

  // per-lane DMA source offsets (fixed over tiles): wave instruction i fills LDS chunk
  // positions [64 (4w + i), +64) of the K tile (16 chunks per row) and of the V^T tile
  // (8 per row); position p holds logical chunk (p % n) ^ swizzle(row)
  int koff[4], voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = (4 * w + i) * 64 + lane;
    const int kr = p >> 4, vr = p >> 3;
    koff[i] = kr * D + (((p & 15) ^ kswz(kr)) << 3);
    voff[i] = vr * KT + (((p & 7) ^ vswz(vr)) << 3);
  }
  {
    const int32_t* btab = P.block_tables + (int64_t)b * P.max_blocks;
    for (int i = t_first + tid; i < n_tiles; i += 256) sbt[i] = btab[i];
    __syncthreads();
  }
  auto issue = [&](int t, uint16_t* ks) {
    const int64_t blk = sbt[t];
    const uint16_t* kp = P.kc + (blk * P.Hkv + kvh) * (int64_t)TILE;
    const uint16_t* vp = P.vc + (blk * P.Hkv + kvh) * (int64_t)TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(kp + koff[i], ks + (4 * w + i) * 512);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(vp + voff[i], ks + TILE + (4 * w + i) * 512);
  };

  // fragment read addresses (elements, within a buffer)
  const int prow = (r32 & ~12) | ((r32 & 4) << 1) | ((r32 & 8) >> 1);   // perm(r32)
  const int ksw = kswz(prow);                                           // same for prow + 32
  const int vsw = vswz(r32);                                            // same for r32 + 32 dt

  const float sl2 = P.scale * V2_LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x16)(0.f);

  auto compute = [&](int t, const uint16_t* ks) {
    const uint16_t* vs = ks + TILE;
    f32x16 sacc[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      sacc[kk] = (f32x16)(0.f);
      const uint16_t* kr = ks + (32 * kk + prow) * D;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8 a = as_bf16x8(*reinterpret_cast<const u16x8*>(kr + (((2 * s + h) ^ ksw) << 3)));
        sacc[kk] = mfma32(a, qf[s], sacc[kk]);
      }
    }
    const int kbase = t * KT;
    const bool need_mask = CAUSAL ? (kbase + KT - 1 > qmin_w || (W > 0 && kbase <= qmax_w - W))
                                  : (kbase + KT > ctx);
    if (need_mask) {   // raw scores; the scale is folded into the exp
      const int k0 = kbase + 8 * h;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = k0 + 32 * kk + 16 * (j >> 3) + (j & 7);
          const bool ok = CAUSAL ? (key <= qpos && (W == 0 || key > qpos - W)) : (key < ctx);
          sacc[kk][j] = ok ? sacc[kk][j] : -INFINITY;
        }
    }
    bf16x8 pf[4];
    if constexpr (ABL == 3) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 16; ++j) pf[2 * kk + (j >> 3)][j & 7] = (__bf16)sacc[kk][j];
    } else {
    float mloc = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 16; ++j) mloc = fmaxf(mloc, sacc[kk][j]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    mloc *= sl2;
    const bool grow = mloc > m + V2_RESCALE_LOG2;
    if (__ballot(grow)) {
      const float m_new = grow ? mloc : m;
      const float alpha = grow ? __builtin_amdgcn_exp2f(m - m_new) : 1.f;
      m = m_new;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    }
    const float mo = m == -INFINITY ? 0.f : -m;
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        const float e0 = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kk][j], sl2, mo));
        const float e1 = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kk][j + 1], sl2, mo));
        ls0 += e0;
        ls1 += e1;
        pf[2 * kk + (j >> 3)][j & 7] = (__bf16)e0;
        pf[2 * kk + (j >> 3)][(j & 7) + 1] = (__bf16)e1;
      }
    l += ls0 + ls1;
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const uint16_t* vr = vs + (32 * dt + r32) * KT;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 a = as_bf16x8(*reinterpret_cast<const u16x8*>(vr + (((2 * s + h) ^ vsw) << 3)));
        o[dt] = mfma32(a, pf[s], o[dt]);
      }
    }
  };

  auto step = [&](int t, const uint16_t* cur, uint16_t* nxt) {
    // this wave's DMA of tile t has landed; the barrier makes every wave's visible and
    // guarantees every wave is done reading the buffer the next DMA refills. (Raw s_barrier:
    // __syncthreads' fence would also wait for the DMA issued below.)
    if constexpr (ABL != 1 && ABL != 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (ABL != 4) __builtin_amdgcn_s_barrier();
    if (ABL != 1 && ABL != 4 && t + 1 < n_tiles) issue(t + 1, nxt);
    if constexpr (ABL == 2) return;
    const int kbase = t * KT;
    const bool wave_needs = wave_active && (!CAUSAL || kbase <= qmax_w) &&
                            (W == 0 || kbase + KT - 1 > qmin_w - W);
    if (wave_needs) compute(t, cur);
  };
  issue(t_first, smem);
  for (int t = t_first; t < n_tiles; ++t) {
    const int bb = (t - t_first) & 1;
    step(t, smem + bb * 2 * TILE, smem + (bb ^ 1) * 2 * TILE);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may outlive the workgroup

  // epilogue: o[dt][j] = O^T[d = 32 dt + (j & 3) + 8 (j >> 2) + 4h][q = r32]
  l += __shfl_xor(l, 32, 64);
  if (row_ok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = P.out + (int64_t)(q0 + qr) * P.out_stride + (int64_t)hq * D + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = f2bf(o[dt][4 * g + j] * inv);
        *reinterpret_cast<u16x4*>(op + 32 * dt + 8 * g) = v;
      }
  }
}

bool launch_prefill_attention_v2(const PrefillParams& p, int num_seqs, int max_q_len, int D,
                                 bool paged, bool causal, hipStream_t stream) {
  static const bool disabled = [] {
    const char* e = getenv("NGA_PREFILL_V1");
    return e && atoi(e) != 0;
  }();
  if (disabled || D != 128 || !paged || p.max_blocks > V2_MAX_TILES) return false;
  if (num_seqs == 0 || max_q_len == 0) return true;
  const int G = p.Hq / p.Hkv;
  const int hpw = G % 4 == 0 ? 4 : G % 2 == 0 ? 2 : 1;
  const int rw = 32 * (4 / hpw);
  PrefillParams pp = p;
  pp.ntiles = (max_q_len + rw - 1) / rw;
  const int64_t total = (int64_t)pp.ntiles * (p.Hq / hpw) * num_seqs;
  pp.total = (int)total;
  pp.per_xcd = (int)((total + 7) / 8);
  dim3 grid(8 * pp.per_xcd);
#define NGA_PF2(CS, HP) prefill_attn_v2_kernel<CS, HP><<<grid, 256, 0, stream>>>(pp)
  static const int abl = [] {
    const char* e = getenv("NGA_PV2_ABLATE");
    return e ? atoi(e) : 0;
  }();
  if (abl && causal && hpw == 4) {
    if (abl == 1) prefill_attn_v2_kernel<true, 4, 1><<<grid, 256, 0, stream>>>(pp);
    else if (abl == 2) prefill_attn_v2_kernel<true, 4, 2><<<grid, 256, 0, stream>>>(pp);
    else if (abl == 3) prefill_attn_v2_kernel<true, 4, 3><<<grid, 256, 0, stream>>>(pp);
    else prefill_attn_v2_kernel<true, 4, 4><<<grid, 256, 0, stream>>>(pp);
    return true;
  }
  if (causal) {
    if (hpw == 4) NGA_PF2(true, 4); else if (hpw == 2) NGA_PF2(true, 2); else NGA_PF2(true, 1);
  } else {
    if (hpw == 4) NGA_PF2(false, 4); else if (hpw == 2) NGA_PF2(false, 2); else NGA_PF2(false, 1);
  }
#undef NGA_PF2
  return true;
}

}  // namespace nga
