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

// ABL (diagnostic builds with NGA_DIAG_BUILD=1, picked by NGA_PV2_ABLATE; results are wrong):
// 1 = no DMA inside the loop, 2 = no compute, 4 = no DMA and no barrier inside the loop,
// 8 = V(i+1)'s DMA issued at the top of iteration i with K(i+1) (a whole iteration to land),
// 16 = no vmcnt wait before the tile barrier
//
// KS = 2 (split-key, few prompts): 8 waves = two groups of the 4-wave layout above, group g
// walking key tiles t_first + 2i + g of the same row block with its own double buffers
// (128 KiB of LDS: one workgroup per CU, two waves per SIMD). A single ~1.2K-token prompt
// is only ~300 row-block workgroups — about one per CU — so the longest causal row block
// sets the time; two groups halve that critical path, and the second wave per SIMD
// overlaps one group's softmax with the other's MFMAs. Both groups run the same number of
// iterations (the odd last tile of group 1 is a fully masked ghost: no DMA) so the
// workgroup-wide barriers line up; at the end group 1 hands (m, l, O) to group 0 through
// LDS and group 0 writes the merged rows.
constexpr int V2_TILE = 64 * 128;       // elements of one K (or V^T) tile: 16 KiB

// One row block: query rows [RW qb, RW qb + RW) of sequence b, head group hg (its HPW heads
// share each K / V^T tile), over the row block's whole causal key range.
// Measured and removed (profiles/r4_prefill/): an 8-wave group sharing every tile (2 x 32 rows
// of each of 4 GQA heads: half the L2 -> CU tile re-reads) 603-625 us and register-staged
// tiles (ds_write_b128 of K / V^T around the mid-iteration barrier) 602.7 us, against 602-608 us
// for this 4-wave DMA form at 4 x 4,096; the diagnostic ablations show the DMA's landing time
// is not exposed (V issued a whole iteration early: 596 us; no vmcnt wait at all: 594 us).
template <bool CAUSAL, int HPW, int ABL, int KS, int RA = 8>
__device__ __forceinline__ void v2_row_block(const PrefillParams& P, uint16_t* smem, int b, int hg, int qb) {
  constexpr int D = 128, KT = 64;
  constexpr int TILE = V2_TILE;
  constexpr int NWV = 4;                // waves per wave group
  constexpr int RB = NWV / HPW;         // 32-row query blocks per workgroup
  constexpr int RW = 32 * RB;           // query rows per workgroup
  constexpr int NI = 16 / NWV;          // DMA instructions per wave per 16-KiB tile
  int32_t* sbt = reinterpret_cast<int32_t*>(smem + KS * 4 * TILE);
  const int grp = KS == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));
  uint16_t* const kbuf = smem + grp * 4 * TILE;
  uint16_t* const vbuf = kbuf + 2 * TILE;
  const int G = P.Hq / P.Hkv;
  const int ngrp = G / HPW;
  const int q0 = P.cu_q[b], qlen = P.cu_q[b + 1] - q0;
  if (qb * RW >= qlen) return;
  const int ctx = P.ctx_lens[b];
  const int kvh = hg / ngrp;

  const int tid = threadIdx.x & (64 * NWV - 1), lane = tid & 63;   // position within the wave group
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hq = kvh * G + (hg % ngrp) * HPW + w % HPW;
  const int rb = w / HPW;
  const int r32 = lane & 31, h = lane >> 5;

  // this lane's query row (a column of the S^T / O^T tiles). Every wave walks the
  // workgroup's whole tile range (uniform control flow for the software pipeline below); with
  // several row blocks per workgroup the earlier blocks' extra tiles are fully masked.
  int qr = qb * RW + rb * 32 + r32;
  const bool row_ok = qr < qlen;
  if (!row_ok) qr = qlen - 1;
  const int qpos = ctx - qlen + qr;
  const int W = CAUSAL ? P.window : 0;

  bf16x8 qf[8];
  {
    const uint16_t* qp = P.q + (int64_t)(q0 + qr) * P.q_stride + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = as_bf16x8(load8(qp + 16 * s));
  }

  // tile range of the workgroup; tiles needing a mask: at / past the first query's diagonal,
  // and (window) before the last query's window start
  const int wq_lo = ctx - qlen + qb * RW;
  const int wq_hi = ctx - qlen + min(qlen - 1, qb * RW + RW - 1);
  const int last_key = CAUSAL ? wq_hi : ctx - 1;
  const int n_tiles = last_key / KT + 1;
  const int t_first = W > 0 ? max(0, wq_lo - W + 1) / KT : 0;
  // iterations of each wave group: group g takes tiles t_first + KS i + g (a tile index past
  // n_tiles is a ghost: no DMA, fully masked)
  const int nt = (n_tiles - t_first + KS - 1) / KS;
  auto tile_of = [&](int i) { return t_first + KS * i + grp; };

  // per-lane DMA source offsets (fixed over tiles): wave instruction i fills LDS chunk
  // positions [64 (4w + i), +64) of the K tile (16 chunks per row) and of the V^T tile
  // (8 per row); position p holds logical chunk (p % n) ^ swizzle(row)
  // (byte offsets from a wave-uniform page base: the saddr + 32-bit voffset form, one VGPR
  // per DMA instead of a 64-bit lane address)
  uint32_t koff[NI], voff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int p = (NI * w + i) * 64 + lane;
    const int kr = p >> 4, vr = p >> 3;
    koff[i] = 2u * (kr * D + (((p & 15) ^ kswz(kr)) << 3));
    voff[i] = 2u * (vr * KT + (((p & 7) ^ vswz(vr)) << 3));
  }
  {
    const int32_t* btab = P.block_tables + (int64_t)b * P.max_blocks;
    for (int i = t_first + (int)threadIdx.x; i < n_tiles; i += 64 * NWV * KS) sbt[i] = btab[i];
    __syncthreads();
  }
  auto page = [&](int t) { return ((int64_t)sbt[t] * P.Hkv + kvh) * (int64_t)TILE; };
  auto issue_k = [&](int t, uint16_t* dst) {
    if (KS > 1 && t >= n_tiles) return;   // ghost tile
    const char* src = reinterpret_cast<const char*>(P.kc + page(t));
#pragma unroll
    for (int i = 0; i < NI; ++i)
      glds16(reinterpret_cast<const uint16_t*>(src + koff[i]), dst + (NI * w + i) * 512);
  };
  auto issue_v = [&](int t, uint16_t* dst) {
    if (KS > 1 && t >= n_tiles) return;   // ghost tile
    const char* src = reinterpret_cast<const char*>(P.vc + page(t));
#pragma unroll
    for (int i = 0; i < NI; ++i)
      glds16(reinterpret_cast<const uint16_t*>(src + voff[i]), dst + (NI * w + i) * 512);
  };
  auto sync_tiles = [&]() {
    // this wave's DMA has landed; the barrier makes every wave's visible and guarantees every
    // wave is done reading the buffers the next DMA refills. (Raw s_barrier: __syncthreads'
    // fence would also wait for the DMA issued after it.)
    if constexpr (ABL != 1 && ABL != 4 && ABL != 16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (ABL != 4) __builtin_amdgcn_s_barrier();
  };

  // fragment read addresses (elements, within a buffer)
  const int prow = (r32 & ~12) | ((r32 & 4) << 1) | ((r32 & 8) >> 1);   // perm(r32)
  const int koffr = prow * D, ksw = kswz(prow);      // same swizzle for prow + 32
  const int voffr = r32 * KT, vsw = vswz(r32);       // same swizzle for r32 + 32 dt

  const float sl2 = P.scale * V2_LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x16)(0.f);

  // The loop works in 32-key halves of the 64-key DMA tiles. Half h2 of tile t:
  //   S^T = K . Q^T  (8 MFMAs; K rows 32 h2 + perm(r) of the K tile)
  //   softmax        (16 scores per lane; keys (j & 7) + 8h + 16 (j >> 3) of the half)
  //   O^T += V^T . P^T (4 d-tiles x 2 key-steps; V^T chunks 4 h2 + 2 s + h)
  auto qk = [&](f32x16& S, const uint16_t* ks, int h2) {
    S = (f32x16)(0.f);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const bf16x8 a = as_bf16x8(*reinterpret_cast<const u16x8*>(
          ks + 32 * h2 * D + koffr + (((2 * s + h) ^ ksw) << 3)));
      S = mfma32(a, qf[s], S);
    }
  };
  auto mask = [&](f32x16& S, int t, int h2) {
    const int kbase = t * KT + 32 * h2;
    if (KS > 1 && t >= n_tiles) {   // ghost tile: stale LDS, nothing visible
#pragma unroll
      for (int j = 0; j < 16; ++j) S[j] = -INFINITY;
      return;
    }
    const bool need = CAUSAL ? (kbase + 31 > wq_lo || (W > 0 && kbase <= wq_hi - W))
                             : (kbase + 32 > ctx);
    if (need) {   // raw scores; the scale is folded into the exp
      const int k0 = kbase + 8 * h;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int key = k0 + 16 * (j >> 3) + (j & 7);
        const bool ok = CAUSAL ? (key <= qpos && (W == 0 || key > qpos - W)) : (key < ctx);
        S[j] = ok ? S[j] : -INFINITY;
      }
    }
  };
  // Softmax of one half, all VALU except the rare O rescale, which it returns as a factor:
  // lazy rescale — m only moves (and O / l are only rescaled) when a row's max over the half
  // exceeds it by more than 2^8; P <= 2^8 is harmless in fp32 sums and bf16 P.
  auto softmax = [&](const f32x16& S, bf16x8 (&pf)[2], float& alpha) -> bool {
    float mloc = S[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) mloc = fmaxf(mloc, S[j]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    mloc *= sl2;
    const bool grow = mloc > m + V2_RESCALE_LOG2;
    const float m_new = grow ? mloc : m;
    // non-growing lanes keep their scale (and a still -inf m must not meet -inf - -inf)
    alpha = grow ? __builtin_amdgcn_exp2f(m - m_new) : 1.f;
    m = m_new;
    // a half can be fully masked for a row (window, or a row block before the diagonal):
    // m may still be -inf then and the offset must not become +inf
    const float mo = m == -INFINITY ? 0.f : -m;
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const float e0 = __builtin_amdgcn_exp2f(__builtin_fmaf(S[j], sl2, mo));
      const float e1 = __builtin_amdgcn_exp2f(__builtin_fmaf(S[j + 1], sl2, mo));
      ls0 += e0;
      ls1 += e1;
      pf[j >> 3][j & 7] = (__bf16)e0;
      pf[j >> 3][(j & 7) + 1] = (__bf16)e1;
    }
    l = l * alpha + (ls0 + ls1);
    return grow;
  };
  auto rescale = [&](bool grow, float alpha) {
    if (__ballot(grow)) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    }
  };
  auto pv = [&](const bf16x8 (&pf)[2], const uint16_t* vs, int h2) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 a = as_bf16x8(*reinterpret_cast<const u16x8*>(
            vs + 32 * dt * KT + voffr + (((4 * h2 + 2 * s + h) ^ vsw) << 3)));
        o[dt] = mfma32(a, pf[s], o[dt]);
      }
  };
  // one pipeline stage: softmax + P.V of the previous half (S, V^T buffer vs, half vh2); the
  // softmax VALU is interleaved with the next half's S^T MFMAs (Sn, K buffer ks, half kh2)
  // skip_pv: S came from a ghost tile (KS = 2: its V^T buffer may hold whatever the LDS held
  // before this workgroup — a NaN pattern times P = 0 is still NaN)
  auto stage = [&](const f32x16& S, const uint16_t* vs, int vh2, f32x16& Sn, const uint16_t* ks,
                   int kh2, int t_next, bool skip_pv) {
    bf16x8 pf[2];
    float alpha;
    qk(Sn, ks, kh2);
    const bool grow = softmax(S, pf, alpha);
    // K fragment reads run RA ahead of their MFMAs: all 8 up front measured 1-3% faster than
    // 2 ahead (4 x 4,096: 616 -> 605 us; profiles/r3_ra)
    __builtin_amdgcn_sched_group_barrier(0x100, RA, 0);    // DS read
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
      if (g + RA < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);  // VALU
    }
    // keep P in this block: otherwise the exps sink past the rescale branch to their P.V use,
    // out of the region the MFMAs above cover
    asm volatile("" ::"v"(pf[0]), "v"(pf[1]), "v"(l));
    rescale(grow, alpha);
    if (!skip_pv) pv(pf, vs, vh2);
    mask(Sn, t_next, kh2);
  };

  // Software pipeline over tiles i = 0 .. nt-1 (t = t_first + i), in 32-key halves: each
  // stage runs the softmax + P.V of one half while the next half's S^T MFMAs overlap the
  // softmax VALU in the same wave (otherwise QK -> softmax -> PV is one serial chain per
  // wave). Iteration i: [stage A: PV(i-1, 1) || QK(i, 0)] [stage B: PV(i, 0) || QK(i, 1)].
  // It reads K(i), V(i-1), V(i); the DMA of K(i+1) goes out at its top (into the buffer of
  // K(i-1)) and that of V(i+1) after a mid-iteration barrier (into the buffer of V(i-1),
  // whose last reader was stage A).
  f32x16 Sa, Sb;
  auto iter = [&](int i, int par, bool first) {
    const int t = tile_of(i);
    const uint16_t* kc_ = kbuf + par * TILE;
    sync_tiles();   // K(i), V(i) landed; every wave is done with iteration i-1
    if constexpr (ABL != 1 && ABL != 4)
      if (i + 1 < nt) issue_k(t + KS, kbuf + (par ^ 1) * TILE);
    if constexpr (ABL == 8)
      if (i + 1 < nt) issue_v(t + KS, vbuf + (par ^ 1) * TILE);
    if constexpr (ABL != 2) {
      if (first) {
        qk(Sa, kc_, 0);
        mask(Sa, t, 0);
      } else {
        stage(Sb, vbuf + (par ^ 1) * TILE, 1, Sa, kc_, 0, t, false);
      }
    }
    if constexpr (ABL != 4) __builtin_amdgcn_s_barrier();   // V(i-1) is free
    if constexpr (ABL != 1 && ABL != 4 && ABL != 8)
      if (i + 1 < nt) issue_v(t + KS, vbuf + (par ^ 1) * TILE);
    if constexpr (ABL != 2) stage(Sa, vbuf + par * TILE, 0, Sb, kc_, 1, t, KS > 1 && t >= n_tiles);
  };

  issue_k(tile_of(0), kbuf);
  issue_v(tile_of(0), vbuf);
  iter(0, 0, true);
  for (int i = 1; i < nt; i += 2) {
    iter(i, 1, false);
    if (i + 1 < nt) iter(i + 1, 0, false);
  }
  if constexpr (ABL != 2) {   // the last half: V(nt-1) landed before iteration nt-1
    bf16x8 pf[2];
    float alpha;
    rescale(softmax(Sb, pf, alpha), alpha);
    if (!(KS > 1 && tile_of(nt - 1) >= n_tiles)) pv(pf, vbuf + ((nt - 1) & 1) * TILE, 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may outlive the workgroup

  // epilogue: o[dt][j] = O^T[d = 32 dt + (j & 3) + 8 (j >> 2) + 4h][q = r32]
  l += __shfl_xor(l, 32, 64);
  if constexpr (KS > 1) {
    // group 1 -> LDS (the tile buffers are free: every wave waited for its own DMA above and
    // the barrier below orders the hand-off); group 0 merges: O = 2^(m0-M) O0 + 2^(m1-M) O1
    __syncthreads();
    float* xo = reinterpret_cast<float*>(smem) + (w * 64 + lane) * 66;
    if (grp == 1) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int j = 0; j < 16; ++j) xo[16 * dt + j] = o[dt][j];
      xo[64] = m;
      xo[65] = l;
    }
    __syncthreads();
    if (grp == 1) return;
    const float m1 = xo[64], l1 = xo[65];
    const float M = fmaxf(m, m1);
    const float f0 = M == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m - M);
    const float f1 = M == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m1 - M);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int j = 0; j < 16; ++j) o[dt][j] = o[dt][j] * f0 + xo[16 * dt + j] * f1;
    l = l * f0 + l1 * f1;
  }
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

// ONE LDS object per workgroup: [K buffer 0 | K buffer 1 | V^T buffer 0 | V^T buffer 1] per
// wave group, then the block ids. (With several LDS variables the compiler gives their
// accesses alias scopes and then waits vmcnt(0) before fragment reads of a buffer whose
// earlier DMA it cannot see retired — serialising the prefetch; a VMEM block-table load
// inside the loop did the same.)
//
// Grid modes:
// * enumerated (P.items == nullptr): workgroup -> (sequence, head group, row block) in the
//   XCD-aware order below, longest causal blocks first;
// * work list (P.items: host-planned (sequence, row block) pairs, longest first, and
//   P.n_items on the device): a fixed grid walks items it = blockIdx.x + k gridDim.x with
//   head group it % NG. The grid does not depend on the step, so a hipGraph captures it once
//   and each replay reads that step's list (engine mixed-step graphs).
template <bool CAUSAL, int HPW, int ABL = 0, int KS = 1, int RA = 8>
__global__ void __launch_bounds__(256 * KS, KS == 1 ? 2 : 1) prefill_attn_v2_kernel(PrefillParams P) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[KS * 4 * V2_TILE + 2 * V2_MAX_TILES];
  const int G = P.Hq / P.Hkv;
  const int ngrp = G / HPW;
  const int NG = P.Hkv * ngrp;
  if (P.items) {
    const int total = *P.n_items * NG;
    for (int it = blockIdx.x; it < total; it += gridDim.x) {
      __syncthreads();   // the previous item's waves are done with the block-id table
      const int k = it / NG;
      v2_row_block<CAUSAL, HPW, ABL, KS, RA>(P, smem, P.items[2 * k], it % NG, P.items[2 * k + 1]);
    }
    return;
  }
  // XCD-aware order (as the 16x16 kernel): each XCD gets a contiguous range of
  // (sequence, kv head, head group, query block), longest causal blocks first.
  const int pblk = blockIdx.x;
  const int L = (pblk & 7) * P.per_xcd + (pblk >> 3);
  if (L >= P.total) return;
  const int qb = P.ntiles - 1 - L % P.ntiles;
  const int hg = (L / P.ntiles) % NG;
  const int b = L / (P.ntiles * NG);
  v2_row_block<CAUSAL, HPW, ABL, KS, RA>(P, smem, b, hg, qb);
}

bool launch_prefill_attention_v2(const PrefillParams& p, int num_seqs, int max_q_len, int D,
                                 bool paged, bool causal, hipStream_t stream) {
  const bool disabled = kernel_form(KF_PREFILL_V1) != 0;
  if (p.impl == 1 || ((p.impl == 0 || p.impl == 4) && disabled) || D != 128 || !paged || p.kv_fp8 ||
      p.max_blocks > V2_MAX_TILES)
    return false;
  const int ks_env = kernel_form(KF_PREFILL_KS);   // 1 | 2 forces the wave-group count (A/B)
  if (num_seqs == 0 || max_q_len == 0) return true;
  const int G = p.Hq / p.Hkv;
  const int hpw = G % 4 == 0 ? 4 : G % 2 == 0 ? 2 : 1;
  int rw = 32 * (4 / hpw);
  PrefillParams pp = p;
  pp.ntiles = (max_q_len + rw - 1) / rw;
  const int64_t total = (int64_t)pp.ntiles * (p.Hq / hpw) * num_seqs;
  // Size rule: this kernel needs about two of its workgroups per CU (two waves per SIMD) to
  // overlap one wave's softmax with the other's MFMAs. A single ~1K-token prompt is ~300
  // workgroups of 128 (row, head) pairs — one wave per SIMD, measured no faster than the
  // 16x16 kernel's ~500 half-size workgroups standalone and 1.6% slower end to end when it
  // shares the chip with the decode attention of a mixed step (benchmarks/kernel_bench.py
  // and scripts/archive/gpu_r2_attn_ab.sh). From ~6 such prompts (or long ones) up it is 15-25% faster.
  // Few row blocks (~one per CU, e.g. one ~1.2K-token prompt): the 8-wave split-key form.
  // impl 4 ("alone": a prefill with no decode attention beside it, e.g. a prefill-only step)
  // drops the sharing concern: standalone this kernel wins from one prompt up — 2 x 1,200
  // tokens 47.6 vs 75.9 us, 3 x 1,200 59.6 vs 97.6 us (profiles/r3_kernels/kb_prefill.json).
  int ks = p.impl == 3 ? 2 : p.impl == 2 ? 1 : (total <= 320 ? 2 : 1);
  if (ks_env == 1 || ks_env == 2) ks = ks_env;
  if (p.impl == 0 && ks == 1 && total < 2 * 256 * 2) return false;
  pp.total = (int)total;
  pp.per_xcd = (int)((total + 7) / 8);
  dim3 grid(8 * pp.per_xcd);
#define NGA_PF2(CS, HP)                                                                   \
  do {                                                                                      \
    if (ks == 2) prefill_attn_v2_kernel<CS, HP, 0, 2><<<grid, 512, 0, stream>>>(pp);        \
    else prefill_attn_v2_kernel<CS, HP><<<grid, 256, 0, stream>>>(pp);                      \
  } while (0)
#ifdef NGA_DIAG_ABLATION  // diagnostic builds only (NGA_DIAG_BUILD=1): results are wrong
  static const int abl = [] {
    const char* e = getenv("NGA_PV2_ABLATE");
    return e ? atoi(e) : 0;
  }();
  if (abl && causal && hpw == 4) {
    if (ks == 2) {
      if (abl == 1) prefill_attn_v2_kernel<true, 4, 1, 2><<<grid, 512, 0, stream>>>(pp);
      else if (abl == 2) prefill_attn_v2_kernel<true, 4, 2, 2><<<grid, 512, 0, stream>>>(pp);
      else prefill_attn_v2_kernel<true, 4, 4, 2><<<grid, 512, 0, stream>>>(pp);
      return true;
    }
    if (abl == 1) prefill_attn_v2_kernel<true, 4, 1><<<grid, 256, 0, stream>>>(pp);
    else if (abl == 2) prefill_attn_v2_kernel<true, 4, 2><<<grid, 256, 0, stream>>>(pp);
    else if (abl == 8) prefill_attn_v2_kernel<true, 4, 8><<<grid, 256, 0, stream>>>(pp);
    else if (abl == 16) prefill_attn_v2_kernel<true, 4, 16><<<grid, 256, 0, stream>>>(pp);
    else prefill_attn_v2_kernel<true, 4, 4><<<grid, 256, 0, stream>>>(pp);
    return true;
  }
#endif
  if (causal) {
    if (hpw == 4) NGA_PF2(true, 4); else if (hpw == 2) NGA_PF2(true, 2); else NGA_PF2(true, 1);
  } else {
    if (hpw == 4) NGA_PF2(false, 4); else if (hpw == 2) NGA_PF2(false, 2); else NGA_PF2(false, 1);
  }
#undef NGA_PF2
  return true;
}

void launch_prefill_attention_v2_worklist(const PrefillParams& p, int grid, int ks, bool causal,
                                          hipStream_t stream) {
  const int G = p.Hq / p.Hkv;
  const int hpw = G % 4 == 0 ? 4 : G % 2 == 0 ? 2 : 1;
  dim3 g(grid);
#define NGA_PFW(CS, HP)                                                                   \
  do {                                                                                    \
    if (ks == 2) prefill_attn_v2_kernel<CS, HP, 0, 2><<<g, 512, 0, stream>>>(p);          \
    else prefill_attn_v2_kernel<CS, HP><<<g, 256, 0, stream>>>(p);                        \
  } while (0)
  if (causal) {
    if (hpw == 4) NGA_PFW(true, 4); else if (hpw == 2) NGA_PFW(true, 2); else NGA_PFW(true, 1);
  } else {
    if (hpw == 4) NGA_PFW(false, 4); else if (hpw == 2) NGA_PFW(false, 2); else NGA_PFW(false, 1);
  }
#undef NGA_PFW
}

}  // namespace nga
