// Decode-shape projection GEMM (K6 for the decode and small mixed buckets, M <= 512):
//
//   out[M, N] = x[M, K] . W[N, K]^T          (nn.Linear layout: both operands K-contiguous)
//
// Why not the library GEMM: at M = 256 the Llama-3-8B q/k/v, o and down projections make only
// 24 / 16 / 16 output tiles of 256 x 256 for 256 CUs, and the tuned hipBLASLt solutions run
// them at 1.3-2.4 TB/s of weight traffic (profiles/r3_decode_step/gemm_small_m.log) while the
// weight stream alone bounds a layer at ~75 us. Every weight byte carries 256 FLOP at M = 256,
// so the kernel has to keep all 256 CUs streaming AND multiplying: the grid is sized to the CUs
// by an in-kernel K split (fp32 partial slabs, reduced by the consumer kernel), never by
// shrinking the tile below the MFMA-bound ratio.
//
// Block tile: BN weight rows x BM token rows x K slice, 4 or 8 waves as WN (weight) x WM (token);
// each wave owns (BN/WN) x (BM/WM) outputs as 16 x 16 MFMA tiles (mfma_f32_16x16x32_bf16).
// Weight rows are the MFMA A operand and token rows the B operand, so a lane ends with 4
// consecutive output features of one token (8-B bf16 / 16-B fp32 stores) and, for the fused
// SwiGLU epilogue, the gate and up values of the same features in the same lane: the tile's
// weight rows are ordered [gate f..f+15 | up f..f+15] per 32-row group, read from the standard
// [gate rows | up rows] layout by index (no repacked weight copy; moe.hip does the same).
//
// Staging: both operands by LDS-DMA (global_load_lds, 16 B per lane, 1 KiB = 8 rows x 128 B per
// wave instruction) into NSTAGE buffers of one __shared__ array; the XOR swizzle that keeps the
// ds_read_b128 fragment reads conflict-free goes on each lane's global SOURCE chunk (the DMA
// writes lane-linearly). One raw s_barrier per 64-deep K step after a counted vmcnt that
// retires only this step's DMA (a __syncthreads would drain every DMA in flight).
//
// Weights: the nn.Linear layout, or (wpack) pre-packed per block tile as [nN][K/64][BN][64], so
// each 64-deep K step of a block's weights is one contiguous BN x 128-B tile (the EPI 2 gate /
// up row interleave baked in): whole DRAM pages instead of 128-B pieces at K x 2-B strides.
//
// Grid: nN x nM x split blocks, remapped so each XCD gets a contiguous range with the token
// tile fastest: the blocks that read the same weight tile share an L2.
//
// Epilogues: 0 = bf16 out, 1 = fp32 partial slab [split, M, N] (summed by splitk_reduce /
// splitk_add_rmsnorm / the consumer), 2 = SwiGLU bf16 out [M, F] (N = F, gate rows [0, F),
// up rows [F, 2F)).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
// K per stage, SBK = 64 (one 128-B row of bf16 per operand row) or 32 (64-B rows: half the LDS
// per stage, so a 256 x 256 tile keeps 4 stages in 128 KiB instead of 2)

// 16-B chunk position in an LDS row of SBK bf16: the XOR key changes every 256 B of rows (2
// rows of 128 B, 4 rows of 64 B), so the 16 lanes of one ds_read_b128 pass (16 rows, one
// logical chunk) land in 16 distinct 16-B bank groups
template <int SBK>
__device__ __forceinline__ int sk_swz(int row, int ch) {
  constexpr int CPR = SBK / 8;             // 16-B chunks per row
  constexpr int RSH = SBK == 64 ? 1 : 2;   // log2(rows per 256 B)
  return row * SBK + ((ch ^ ((row >> RSH) & (CPR - 1))) << 3);
}

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[15:14];
// expcnt 7 / lgkmcnt 15 = no wait on those counters)
template <int N>
__device__ __forceinline__ void sk_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ float sk_silu(float x) { return x / (1.f + __expf(-x)); }

// a 16-B slab read. The slabs are read once, but non-temporal slab stores / loads measured no
// faster (the very next kernel reads them back; headline 40.08 / 39.82 QPS with nt stores vs
// 40.24 / 40.25 cached, profiles/r5_skinny_snt/) and were removed.
__device__ __forceinline__ f32x4 sk_ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
}  // namespace

template <int BN, int BM, int WN, int WM, int NSTAGE, int EPI, int SBK>
__global__ void __launch_bounds__(64 * WN * WM) skinny_gemm_kernel(SkinnyGemmParams P) {
  constexpr int NW = WN * WM;   // waves per workgroup (4 or 8)
  constexpr int RW = BN / WN;   // weight rows per wave
  constexpr int CW = BM / WM;   // token rows per wave
  constexpr int NTW = RW / 16, MTW = CW / 16;
  constexpr int CPR = SBK / 8;          // 16-B chunks per LDS row
  constexpr int RPI = 64 / CPR;         // rows per 1-KiB DMA instruction (8 or 16)
  constexpr int KSS = SBK / 32;         // 32-deep MFMA k-steps per stage (2 or 1)
  static_assert(SBK == 64 || SBK == 32, "stage depth");
  static_assert((NW == 4 || NW == 8) && NTW >= 1 && MTW >= 1, "tile");
  static_assert(BN % (RPI * NW) == 0 && BM % (RPI * NW) == 0, "every wave stages whole DMA pieces");
  static_assert(EPI != 2 || NTW % 2 == 0, "SwiGLU pairs gate / up tiles inside a wave");
  static_assert(NSTAGE >= 2 && NSTAGE <= 4, "stage count");
  constexpr int W_GL = BN / (RPI * NW), X_GL = BM / (RPI * NW);   // DMA instructions per wave per stage
  constexpr int NPS = W_GL + X_GL;
  constexpr int STAGE = (BN + BM) * SBK;          // uint16 elements per stage
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSTAGE * STAGE];

  const int nblk = P.nN * P.nM * P.split;
  const int pb = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, x8 = pb % 8;
  const int L = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + pb / 8;
  const int mi = L % P.nM;
  const int ks = (L / P.nM) % P.split;
  const int nb = L / (P.nM * P.split);
  const int nk_all = P.K / SBK;
  const int kb = ks * nk_all / P.split;
  const int nk = (ks + 1) * nk_all / P.split - kb;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wn = wv % WN, wm = wv / WN;
  const int col = lane & 15, h = lane >> 4;

  // per-lane DMA sources (fixed over K): instruction i of wave wv fills LDS rows
  // [RPI (wv * N + i), +RPI) lane-linearly; lane l lands in row + l / CPR, physical chunk
  // l % CPR, which holds logical chunk (l % CPR) ^ swizzle(row)
  constexpr int RSH = SBK == 64 ? 1 : 2;
  const uint16_t* wsrc[W_GL];
#pragma unroll
  for (int i = 0; i < W_GL; ++i) {
    const int r = (wv * W_GL + i) * RPI + lane / CPR;
    const int ch = (lane % CPR) ^ ((r >> RSH) & (CPR - 1));
    int wrow;
    if constexpr (EPI == 2) {
      const int rr = r % RW;
      const int f = nb * (BN / 2) + (r / RW) * (RW / 2) + (rr >> 5) * 16 + (rr & 15);
      wrow = ((rr >> 4) & 1) ? P.N + f : f;
    } else {
      wrow = nb * BN + r;
      if (wrow >= P.N) wrow = P.N - 1;   // ragged last block: any valid row (not stored)
    }
    if (P.wpack)   // tile-packed weights [nN][K/64][BN][64]: a K step of a block is one contiguous tile
      wsrc[i] = P.w + ((int64_t)nb * nk_all + kb) * (BN * SBK) + r * SBK + ch * 8;
    else
      wsrc[i] = P.w + (int64_t)wrow * P.K + (int64_t)kb * SBK + ch * 8;
  }
  const uint16_t* xsrc[X_GL];
#pragma unroll
  for (int i = 0; i < X_GL; ++i) {
    const int r = (wv * X_GL + i) * RPI + lane / CPR;
    const int ch = (lane % CPR) ^ ((r >> RSH) & (CPR - 1));
    int t = mi * BM + r;
    if (t >= P.M) t = P.M - 1;           // padding token rows: any valid row (not stored)
    if (P.xpack)   // tile-packed activations [nM][K/64][BM][64] (rows past M are zero padding)
      xsrc[i] = P.x + ((int64_t)mi * nk_all + kb) * (BM * SBK) + r * SBK + ch * 8;
    else
      xsrc[i] = P.x + (int64_t)t * P.ldx + (int64_t)kb * SBK + ch * 8;
  }
  // krot: blocks walk their K range from different starting steps, so the blocks that share an
  // operand slice (x for every weight block, W for every token tile) do not all address the
  // same 128-B column of it at the same moment
  const int rot = P.krot ? (int)((unsigned)(nb * 7 + mi * 3) % (unsigned)nk) : 0;
  auto issue = [&](int kt, int buf) {
    uint16_t* base = smem + buf * STAGE;
    int ke = kt + rot;
    if (ke >= nk) ke -= nk;
    const int k0 = ke * SBK;
    const int64_t wk0 = P.wpack ? (int64_t)ke * (BN * SBK) : (int64_t)k0;
    // weights with the default cache policy: non-temporal weight DMA measured within noise
#pragma unroll
    for (int i = 0; i < W_GL; ++i) glds16(wsrc[i] + wk0, base + (wv * W_GL + i) * RPI * SBK);
    const int64_t xk0 = P.xpack ? (int64_t)ke * (BM * SBK) : (int64_t)k0;
#pragma unroll
    for (int i = 0; i < X_GL; ++i) glds16(xsrc[i] + xk0, base + BN * SBK + (wv * X_GL + i) * RPI * SBK);
  };

  f32x4 acc[NTW][MTW];
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = (f32x4)(0.f);

  bf16x8 af[2][NTW], bfr[2][MTW];
  auto read_frags = [&](const uint16_t* ws, int s) {
    const uint16_t* xs = ws + BN * SBK;
    const int ch = 4 * s + h;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
      bfr[s][mt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&xs[sk_swz<SBK>(wm * CW + mt * 16 + col, ch)]));
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
      af[s][nt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&ws[sk_swz<SBK>(wn * RW + nt * 16 + col, ch)]));
  };
  auto mfmas = [&](int s) {
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt) acc[nt][mt] = mfma16(af[s][nt], bfr[s][mt], acc[nt][mt]);
  };
  constexpr int NR = NTW + MTW, NM = NTW * MTW;   // reads / MFMAs per 32-deep k-step
  constexpr int GR = NR >= 4 ? NR / 4 : 1, GM = NM >= 4 ? NM / 4 : 1;

#pragma unroll
  for (int st = 0; st < NSTAGE - 1; ++st)
    if (st < nk) issue(st, st);
  for (int kt = 0; kt < nk; ++kt) {
    // retire stage kt (this wave's DMA); later stages stay in flight. The count is the DMA of
    // the stages issued after kt: NSTAGE - 2 of them in the steady state, fewer at the tail.
    const int after = min(nk - 1 - kt, NSTAGE - 2);
    if (after >= 2) sk_wait_vm<2 * NPS>();
    else if (after == 1) sk_wait_vm<NPS>();
    else sk_wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const uint16_t* ws = smem + (kt % NSTAGE) * STAGE;
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    if constexpr (KSS == 2) {
      // k-step 0's fragments first; then its MFMAs with k-step 1's reads interleaved
      read_frags(ws, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_frags(ws, 1);
      mfmas(0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, GM, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, GR, 0);   // DS read
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(1);
    } else {
      // one 32-deep k-step per stage: its fragments, then its MFMAs
      read_frags(ws, 0);
      __builtin_amdgcn_sched_barrier(0);
      mfmas(0);
    }
  }
  sk_wait_vm<0>();   // no DMA may still target this CU's LDS when the workgroup ends

  // epilogue: acc[nt][mt][r] = out[token (16-tile mt, col)][feature (16-tile nt, 4h + r)]
  const int t_base = mi * BM + wm * CW;
  const int n_base = nb * BN + wn * RW;
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
    const int t = t_base + mt * 16 + col;
    if (t >= P.M) continue;
    if constexpr (EPI == 0) {
      uint16_t* op = reinterpret_cast<uint16_t*>(P.out) + (int64_t)t * P.ldo;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n = n_base + nt * 16 + 4 * h;
        if (n >= P.N) continue;
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(acc[nt][mt][r]);
        *reinterpret_cast<u16x4*>(op + n) = v;
      }
    } else if constexpr (EPI == 1) {
      float* op = reinterpret_cast<float*>(P.out) + ((int64_t)ks * P.M + t) * P.N;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n = n_base + nt * 16 + 4 * h;
        if (n >= P.N) continue;
        *reinterpret_cast<f32x4*>(op + n) = acc[nt][mt];
      }
    } else {
      uint16_t* op = reinterpret_cast<uint16_t*>(P.out) + (int64_t)t * P.ldo;
#pragma unroll
      for (int g = 0; g < NTW / 2; ++g) {
        const int f = nb * (BN / 2) + wn * (RW / 2) + g * 16 + 4 * h;
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(sk_silu(acc[2 * g][mt][r]) * acc[2 * g + 1][mt][r]);
        *reinterpret_cast<u16x4*>(op + f) = v;
      }
    }
  }
}

// out[m, n] = bf16(sum_s P[s, m, n]); 8 features per thread
__global__ void splitk_reduce_kernel(const float* __restrict__ P, int S, int M, int N,
                                     uint16_t* __restrict__ out, int64_t ldo) {
  const int nv = N / 8;
  const int64_t total = (int64_t)M * nv;
  const int64_t slab = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / nv;
    const int c = (int)(i - m * nv) * 8;
    const float* p = P + m * N + c;
    f32x4 a0 = sk_ld4(p), a1 = sk_ld4(p + 4);
    for (int s = 1; s < S; ++s) {
      a0 += sk_ld4(p + s * slab);
      a1 += sk_ld4(p + s * slab + 4);
    }
    u16x8 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[q] = f2bf(a0[q]);
      o[4 + q] = f2bf(a1[q]);
    }
    store8(out + m * ldo + c, o);
  }
}

// out[m, f] = bf16(silu(sum_s P[s, m, f]) * sum_s P[s, m, F + f]): the K-split gate / up
// projection (slabs in the standard [gate | up] column order) summed by its SwiGLU consumer
__global__ void splitk_swiglu_kernel(const float* __restrict__ P, int S, int M, int F,
                                     uint16_t* __restrict__ out, int64_t ldo) {
  const int nv = F / 8;
  const int64_t total = (int64_t)M * nv;
  const int64_t slab = (int64_t)M * 2 * F;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / nv;
    const int c = (int)(i - m * nv) * 8;
    const float* p = P + m * 2 * F + c;
    f32x4 g0 = sk_ld4(p), g1 = sk_ld4(p + 4);
    f32x4 u0 = sk_ld4(p + F), u1 = sk_ld4(p + F + 4);
    for (int s = 1; s < S; ++s) {
      const float* q = p + s * slab;
      g0 += sk_ld4(q);
      g1 += sk_ld4(q + 4);
      u0 += sk_ld4(q + F);
      u1 += sk_ld4(q + F + 4);
    }
    u16x8 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = f2bf(sk_silu(g0[r]) * u0[r]);
      o[4 + r] = f2bf(sk_silu(g1[r]) * u1[r]);
    }
    store8(out + m * ldo + c, o);
  }
}

// resid += sum_s P[s] (one rounding to the bf16 residual); out = rmsnorm(resid) * w.
// One workgroup per row, 8 features per lane (the add_rmsnorm kernel with the split-K sum of
// the producing GEMM folded into its load).
__global__ void __launch_bounds__(1024) splitk_add_rmsnorm_kernel(const float* __restrict__ P, int S,
                                                                  int M, uint16_t* __restrict__ resid,
                                                                  const uint16_t* __restrict__ w,
                                                                  float eps, int H,
                                                                  uint16_t* __restrict__ out) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int c = threadIdx.x * 8;
  const bool active = c < H;
  const int64_t slab = (int64_t)M * H;
  float x[8];
  float ss = 0.f;
  if (active) {
    const float* p = P + row * H + c;
    f32x4 a0 = sk_ld4(p), a1 = sk_ld4(p + 4);
    for (int s = 1; s < S; ++s) {
      a0 += sk_ld4(p + s * slab);
      a1 += sk_ld4(p + s * slab + 4);
    }
    const u16x8 v = load8(resid + row * H + c);
    u16x8 st;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      st[i] = f2bf(bf2f(v[i]) + (i < 4 ? a0[i] : a1[i - 4]));
      x[i] = bf2f(st[i]);   // normalise what is stored (bf16 residual stream)
      ss += x[i] * x[i];
    }
    store8(resid + row * H + c, st);
  }
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)H + eps);
  if (active) {
    const u16x8 wv = load8(w + c);
    u16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2bf(x[i] * r * bf2f(wv[i]));
    store8(out + row * H + c, o);
  }
}

// ------------------------------------------------------------------ launchers
// tile configurations: {BN, BM, WN, WM, NSTAGE} (WN x WM waves). Measured and dropped: two-stage
// tiles small enough for 2-3 workgroups (16-24 waves) per CU — {128,128,2,4,2}, {256,64,4,2,2},
// {128,64,2,4,2} — 10-70 % slower than the table's picks (profiles/r4_skinny/sweep_more_waves.jsonl); the
// next stage's DMA pieces spread one by one between the MFMAs instead of issued together at the
// barrier (5-30 % slower at every tile; 256 x 256 collapsed; profiles/r4_headline_ab/sweep_il.jsonl)
#define NGA_SKINNY_CFGS(X)       \
  X(0, 256, 128, 2, 2, 3, 64)   \
  X(1, 128, 128, 2, 2, 3, 64)   \
  X(2, 128, 64, 2, 2, 3, 64)    \
  X(3, 64, 64, 2, 2, 4, 64)     \
  X(4, 128, 256, 2, 2, 2, 64)   \
  X(5, 64, 256, 1, 4, 3, 64)    \
  X(6, 256, 64, 4, 1, 3, 64)    \
  X(7, 128, 32, 4, 1, 4, 64)    \
  X(8, 256, 32, 4, 1, 3, 64)    \
  X(9, 64, 128, 1, 4, 3, 64)    \
  X(10, 128, 128, 2, 2, 4, 64)  \
  X(11, 128, 128, 2, 2, 2, 64)  \
  X(12, 256, 256, 4, 2, 2, 64)  \
  X(13, 256, 128, 4, 2, 3, 64)  \
  X(14, 128, 256, 2, 4, 2, 64)  \
  X(15, 64, 64, 2, 2, 2, 64)    \
  X(16, 256, 128, 2, 4, 3, 64)  \
  X(17, 256, 256, 4, 2, 4, 32)  \
  X(18, 256, 256, 2, 4, 4, 32)  \
  X(19, 256, 256, 4, 2, 3, 32)  \
  X(20, 256, 128, 4, 2, 4, 32)  \
  X(21, 128, 256, 2, 4, 4, 32)  \
  X(22, 128, 128, 2, 2, 4, 32)  \
  X(23, 128, 128, 2, 4, 4, 32)  \
  X(24, 256, 128, 4, 2, 2, 32)  \
  X(25, 256, 128, 2, 4, 3, 32)  \
  X(26, 128, 256, 2, 4, 3, 32)  \
  X(27, 224, 128, 1, 4, 3, 64)

int skinny_gemm_cfg_count() {
  int n = 0;
#define NGA_COUNT(ID, BN, BM, WN, WM, NS, BK) ++n;
  NGA_SKINNY_CFGS(NGA_COUNT)
#undef NGA_COUNT
  return n;
}

// {BN, BM, WN, WM, NSTAGE, BK} of a configuration, or zeros
void skinny_gemm_cfg_info(int cfg, int* info) {
  info[0] = info[1] = info[2] = info[3] = info[4] = info[5] = 0;
#define NGA_INFO(ID, BN, BM, WN, WM, NS, BK) \
  if (cfg == ID) {                           \
    info[0] = BN;                            \
    info[1] = BM;                            \
    info[2] = WN;                            \
    info[3] = WM;                            \
    info[4] = NS;                            \
    info[5] = BK;                            \
    return;                                  \
  }
  NGA_SKINNY_CFGS(NGA_INFO)
#undef NGA_INFO
}

void launch_skinny_gemm(const SkinnyGemmParams& p, int cfg, int epi, hipStream_t stream) {
  const int nblk = p.nN * p.nM * p.split;
  dim3 grid(nblk);
#define NGA_LAUNCH(ID, BN, BM, WN, WM, NS, BK)                                                        \
  if (cfg == ID) {                                                                                        \
    if (nblk == 0) return;                                                                                \
    const dim3 block(64 * WN * WM);                                                                       \
    if (epi == 0) skinny_gemm_kernel<BN, BM, WN, WM, NS, 0, BK><<<grid, block, 0, stream>>>(p);       \
    else if (epi == 1) skinny_gemm_kernel<BN, BM, WN, WM, NS, 1, BK><<<grid, block, 0, stream>>>(p);  \
    else skinny_gemm_kernel<BN, BM, WN, WM, NS, 2, BK><<<grid, block, 0, stream>>>(p);                \
    return;                                                                                               \
  }
  NGA_SKINNY_CFGS(NGA_LAUNCH)
#undef NGA_LAUNCH
}

void launch_splitk_reduce(const float* P, int S, int M, int N, uint16_t* out, int64_t ldo,
                          hipStream_t stream) {
  if (M == 0) return;
  int64_t g = ((int64_t)M * (N / 8) + 255) / 256;
  if (g > 2048) g = 2048;
  splitk_reduce_kernel<<<(unsigned)g, 256, 0, stream>>>(P, S, M, N, out, ldo);
}

void launch_splitk_swiglu(const float* P, int S, int M, int F, uint16_t* out, int64_t ldo,
                          hipStream_t stream) {
  if (M == 0) return;
  int64_t g = ((int64_t)M * (F / 8) + 255) / 256;
  if (g > 2048) g = 2048;
  splitk_swiglu_kernel<<<(unsigned)g, 256, 0, stream>>>(P, S, M, F, out, ldo);
}

void launch_splitk_add_rmsnorm(const float* P, int S, int M, uint16_t* resid, const uint16_t* w,
                               float eps, int H, uint16_t* out, hipStream_t stream) {
  if (M == 0) return;
  int t = (H / 8 + 63) / 64 * 64;
  if (t < 64) t = 64;
  splitk_add_rmsnorm_kernel<<<M, t, 0, stream>>>(P, S, M, resid, w, eps, H, out);
}

}  // namespace nga
