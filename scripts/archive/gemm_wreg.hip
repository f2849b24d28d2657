// ARCHIVED (round 5, not built): measured slower than gemm_skinny.hip's LDS tiles on every
// llama3-8b projection at M = 64-256, consumers included (profiles/r5_wreg/: e.g. gate/up at
// M = 256 85-118 us vs 82.7 us, down 56-75 vs 50.8, o 25.7-38 vs 23.4). Weights in registers cut
// the LDS traffic but not the L2 -> CU intake: with BN = M = 256 per CU and split-K to fill the
// chip the per-CU intake still caps near 40-44 GB/s, as in the LDS form. Kept as the record of
// the experiment (it was wired in as skinny cfg IDs 17-38 for the sweep).
// Decode-shape projection GEMM, weight-in-registers form (K6, M <= 256 per token tile):
//
//   out[M, N] = x[M, K] . W[N, K]^T          (nn.Linear layout: both operands K-contiguous)
//
// Why a second decode-shape kernel: gemm_skinny.hip stages BOTH operands through LDS, so every
// block re-reads its weight tile once per token tile and its token tile once per weight tile:
// the CU intake is 2KMN (1/BM + 1/BN) bytes, and with three LDS stages of (BN + BM) x 64 the
// tile cannot grow past 256 x 128 (profiles/r4_pmc: the intake, not HBM, bounds it at ~9 TB/s).
// Here the weights never touch LDS: each wave streams its own weight rows global -> VGPR and
// uses every fragment against ALL of the block's token rows (BM = M up to 256), so each weight
// byte crosses L2 -> CU exactly once and LDS holds only the token tile (32 KiB per 64-deep stage
// at M = 256: four stages fit where the LDS form fit two or three). Intake = 2KN (1 + M / BN).
//
// MFMA: mfma_f32_32x32x16_bf16, A = 32 weight rows (register-resident), B = 32 token rows (LDS).
// A 64-deep K chunk feeds four MFMA k-steps. The MFMA's 16 k slots are a dummy index, so each
// lane takes CONTIGUOUS weights: lane (r = l & 31, h = l >> 5) loads W[row r][k0 + 32h .. +32)
// (64 B, four dwordx4 per chunk; two lanes cover a row's 128-B line) and k-step j uses its
// elements [8j, 8j + 8). The token fragment of k-step j is therefore x[t][k0 + 32h + 8j .. +8]:
// LDS chunk 4h + j of the token row, XOR-swizzled (chunk ^ ((row >> 1) & 7)) so the
// ds_read_b128 of a 16-lane group hits 16 distinct 4-bank groups.
//
// Accumulators: lane holds, per (32-row tile, 32-token tile), register j = feature
// (j & 3) + 4h + 8 (j >> 2) of token l & 31 — 4 consecutive features per register quad
// (8-B bf16 / 16-B fp32 stores). SwiGLU (EPI 2): a tile's rows are [gate f..f+15 | up f..f+15],
// so gate register j < 8 pairs with up register j + 8 in the same lane.
//
// Pipeline: NS steps in flight. Step s = the token-tile DMA of chunk s (global_load_lds into LDS
// stage s % NS) + the weight loads of chunk s (into register buffer s % NS); the loop is
// unrolled by NS so both rings index statically. One raw s_barrier per chunk after a counted
// vmcnt that retires only this chunk's DMA (the weight registers are waited for by the
// compiler's own counters when first used).
//
// Grid: nN x nM x split blocks remapped to contiguous ranges per XCD, weight block fastest:
// an XCD's blocks share one (token tile, K slice) of x in their L2.
//
// Epilogues as gemm_skinny.hip: 0 bf16 [M, N]; 1 fp32 K-split slabs [split, M, N] (summed by the
// consumer); 2 SwiGLU bf16 [M, F] (gate rows [0, F), up rows [F, 2F) of W).
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int wr_swz(int row, int ch) {  // 16-B chunk of a 128-B LDS row
  return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3);
}

// s_waitcnt vmcnt(N) alone (gfx9 encoding; expcnt / lgkmcnt left at "no wait")
template <int N>
__device__ __forceinline__ void wr_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ float wr_silu(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ bf16x8 u4_bf(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// Weight loads as inline asm: the compiler's wait insertion treats a mix of LDS-DMA and plain
// loads as out of order and would drain vmcnt to 0 before every first use of a weight register
// (killing the prefetch); the kernel waits for them itself with counted vmcnts (in order on
// hardware), so the compiler must not see them as loads.
template <int OFF>
__device__ __forceinline__ uint4 wr_load16(const uint16_t* p) {
  uint4 r;
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(r) : "v"(p), "n"(OFF));
  return r;
}
}  // namespace

template <int RT, int NW, int MT, int NS, int BPF, int EPI>
__global__ void __launch_bounds__(64 * NW) wreg_gemm_kernel(SkinnyGemmParams P) {
  constexpr int BN = 32 * RT * NW;          // weight rows per block
  constexpr int BM = 32 * MT;               // token rows per block
  constexpr int XP = BM / 8;                // 8-row DMA pieces per token stage
  constexpr int X_GL = (XP + NW - 1) / NW;  // pieces per wave (surplus waves repeat the last one)
  constexpr int W_GL = 4 * RT;              // dwordx4 weight loads per wave per chunk
  constexpr int STEP = X_GL + W_GL;         // vector-memory instructions per pipeline step
  constexpr int STAGE = BM * 64;            // uint16 per LDS stage
  static_assert(NS >= 2 && NS <= 4, "stages");
  static_assert((NS - 1) * STEP < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NS * STAGE];

  const int nblk = P.nN * P.nM * P.split;
  const int pb = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, x8 = pb % 8;
  const int L = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + pb / 8;
  const int nb = L % P.nN;
  const int mi = (L / P.nN) % P.nM;
  const int ks = L / (P.nN * P.nM);
  const int nk_all = P.K / 64;
  const int kb = ks * nk_all / P.split;
  const int nk = (ks + 1) * nk_all / P.split - kb;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;

  // this lane's weight row in each of its 32-row tiles (64 contiguous bytes per chunk)
  const uint16_t* wsrc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int tile = wv * RT + rt;
    int wrow;
    if constexpr (EPI == 2) {
      const int f = nb * (BN / 2) + tile * 16 + (l32 & 15);
      wrow = l32 >= 16 ? P.N + f : f;
    } else {
      wrow = nb * BN + tile * 32 + l32;
      if (wrow >= P.N) wrow = P.N - 1;   // ragged last block: any valid row (not stored)
    }
    wsrc[rt] = P.w + (int64_t)wrow * P.K + (int64_t)kb * 64 + 32 * h;
  }
  // token-tile DMA: piece p fills LDS rows [8p, 8p + 8) lane-linearly; lane l lands in row
  // 8p + l / 8, physical chunk l % 8, which holds logical chunk (l % 8) ^ swizzle(row)
  const uint16_t* xsrc[X_GL];
  int xdst[X_GL];
#pragma unroll
  for (int i = 0; i < X_GL; ++i) {
    const int p = min(wv + i * NW, XP - 1);
    const int r = p * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((r >> 1) & 7);
    int t = mi * BM + r;
    if (t >= P.M) t = P.M - 1;           // padding token rows: any valid row (not stored)
    xsrc[i] = P.x + (int64_t)t * P.ldx + (int64_t)kb * 64 + ch * 8;
    xdst[i] = p * 8 * 64;
  }

  uint4 wreg[NS][W_GL];
  auto issue = [&](int kt, int buf) {
    uint16_t* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < X_GL; ++i) glds16(xsrc[i] + kt * 64, base + xdst[i]);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const uint16_t* src = wsrc[rt] + kt * 64;
      wreg[buf][rt * 4 + 0] = wr_load16<0>(src);
      wreg[buf][rt * 4 + 1] = wr_load16<16>(src);
      wreg[buf][rt * 4 + 2] = wr_load16<32>(src);
      wreg[buf][rt * 4 + 3] = wr_load16<48>(src);
    }
  };

  f32x16 acc[RT][MT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = (f32x16)(0.f);

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
  __builtin_amdgcn_sched_barrier(0);

  auto compute = [&](int u) {
    const uint16_t* xs = smem + u * STAGE;
    if constexpr (BPF) {
      // token fragments of k-step j + 1 requested before k-step j's MFMAs (one wave per SIMD has
      // no partner wave to cover the LDS latency)
      bf16x8 b[2][MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        b[0][mt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&xs[wr_swz(mt * 32 + l32, 4 * h)]));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < 3) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            b[(j + 1) & 1][mt] =
                as_bf16x8(*reinterpret_cast<const u16x8*>(&xs[wr_swz(mt * 32 + l32, 4 * h + j + 1)]));
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const bf16x8 a = u4_bf(wreg[u][rt * 4 + j]);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = mfma32x16(a, b[j & 1][mt], acc[rt][mt]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x8 b[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          b[mt] = as_bf16x8(*reinterpret_cast<const u16x8*>(&xs[wr_swz(mt * 32 + l32, 4 * h + j)]));
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const bf16x8 a = u4_bf(wreg[u][rt * 4 + j]);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = mfma32x16(a, b[mt], acc[rt][mt]);
        }
      }
    }
  };

  // steady state: every chunk of an NS-group issues its step kt + NS - 1 unconditionally, so the
  // vector-memory counts are static (the compiler's own waits on the weight registers stay exact)
  int kt0 = 0;
  for (; kt0 + 2 * NS - 2 < nk; kt0 += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      wr_wait_vm<(NS - 2) * STEP + W_GL>();   // step kt's DMA retired; later steps in flight
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      issue(kt0 + u + NS - 1, (u + NS - 1) % NS);
      wr_wait_vm<(NS - 1) * STEP>();           // step kt's weight registers landed
      __builtin_amdgcn_sched_barrier(0);
      compute(u);
    }
  }
  // tail: at most 2 NS - 2 chunks, issuing only the steps that exist
  for (; kt0 < nk; kt0 += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int kt = kt0 + u;
      if (kt < nk) {
        const int after = min(nk - 1, kt + NS - 2) - kt;   // steps issued after step kt
        if (after >= NS - 2) wr_wait_vm<(NS - 2) * STEP + W_GL>();
        else if (NS >= 4 && after == 1) wr_wait_vm<(NS >= 4 ? STEP + W_GL : 0)>();
        else wr_wait_vm<W_GL>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + NS - 1 < nk) issue(kt + NS - 1, (u + NS - 1) % NS);
        wr_wait_vm<0>();   // tail: everything issued so far (weights of step kt included)
        __builtin_amdgcn_sched_barrier(0);
        compute(u);
      }
    }
  }
  wr_wait_vm<0>();   // no DMA may still target this CU's LDS when the workgroup ends

  // epilogue: acc[rt][mt][j] = out[token mt * 32 + l32][feature tile_base + (j & 3) + 4h + 8 (j >> 2)]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int t = mi * BM + mt * 32 + l32;
    if (t >= P.M) continue;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int tile = wv * RT + rt;
      if constexpr (EPI == 2) {
        uint16_t* op = reinterpret_cast<uint16_t*>(P.out) + (int64_t)t * P.ldo;
        const int fb = nb * (BN / 2) + tile * 16 + 4 * h;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          u16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = f2bf(wr_silu(acc[rt][mt][4 * g + r]) * acc[rt][mt][8 + 4 * g + r]);
          *reinterpret_cast<u16x4*>(op + fb + 8 * g) = v;
        }
      } else {
        const int nbase = nb * BN + tile * 32 + 4 * h;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = nbase + 8 * g;
          if (n >= P.N) continue;
          if constexpr (EPI == 0) {
            u16x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = f2bf(acc[rt][mt][4 * g + r]);
            *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(P.out) + (int64_t)t * P.ldo + n) = v;
          } else {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[rt][mt][4 * g + r];
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.out) + ((int64_t)ks * P.M + t) * P.N + n) = v;
          }
        }
      }
    }
  }
}

// configurations {RT, NW, MT, NS}: RT 32-row weight tiles per wave, NW waves, MT 32-token
// tiles (BM = 32 MT), NS pipeline steps in flight. IDs continue gemm_skinny.hip's list.
#define NGA_WREG_CFGS(X) \
  X(17, 1, 8, 8, 3, 0)      \
  X(18, 2, 4, 8, 3, 0)      \
  X(19, 1, 4, 8, 3, 0)      \
  X(20, 1, 8, 8, 2, 0)      \
  X(21, 1, 4, 8, 4, 0)      \
  X(22, 1, 8, 4, 3, 0)      \
  X(23, 2, 4, 4, 3, 0)      \
  X(24, 1, 4, 4, 4, 0)      \
  X(25, 1, 8, 4, 4, 0)      \
  X(26, 1, 8, 2, 4, 0)      \
  X(27, 2, 4, 2, 4, 0)      \
  X(28, 1, 4, 2, 4, 0)      \
  X(29, 1, 4, 1, 4, 0)      \
  X(30, 2, 4, 1, 4, 0)      \
  X(31, 1, 8, 6, 3, 0)      \
  X(32, 2, 4, 6, 3, 0)      \
  X(33, 1, 8, 8, 4, 0)      \
  X(34, 2, 4, 8, 4, 0)      \
  X(35, 1, 4, 8, 3, 1)      \
  X(36, 2, 4, 8, 3, 1)      \
  X(37, 1, 4, 8, 4, 1)      \
  X(38, 2, 4, 8, 4, 1)

int wreg_gemm_cfg_count() {
  int n = 0;
#define NGA_COUNT(ID, RT, NW, MT, NS, BPF) ++n;
  NGA_WREG_CFGS(NGA_COUNT)
#undef NGA_COUNT
  return n;
}

bool wreg_gemm_cfg_info(int cfg, int* info) {
#define NGA_INFO(ID, RT, NW, MT, NS, BPF) \
  if (cfg == ID) {                   \
    info[0] = 32 * RT * NW;          \
    info[1] = 32 * MT;               \
    info[2] = NW;                    \
    info[3] = 1;                     \
    info[4] = NS;                    \
    info[5] = 1;                     \
    return true;                     \
  }
  NGA_WREG_CFGS(NGA_INFO)
#undef NGA_INFO
  return false;
}

bool launch_wreg_gemm(const SkinnyGemmParams& p, int cfg, int epi, hipStream_t stream) {
  const int nblk = p.nN * p.nM * p.split;
#define NGA_LAUNCH(ID, RT, NW, MT, NS, BPF)                                                        \
  if (cfg == ID) {                                                                              \
    if (nblk == 0) return true;                                                                 \
    const dim3 grid(nblk), block(64 * NW);                                                      \
    if (epi == 0) wreg_gemm_kernel<RT, NW, MT, NS, BPF, 0><<<grid, block, 0, stream>>>(p);           \
    else if (epi == 1) wreg_gemm_kernel<RT, NW, MT, NS, BPF, 1><<<grid, block, 0, stream>>>(p);      \
    else wreg_gemm_kernel<RT, NW, MT, NS, BPF, 2><<<grid, block, 0, stream>>>(p);                    \
    return true;                                                                                \
  }
  NGA_WREG_CFGS(NGA_LAUNCH)
#undef NGA_LAUNCH
  return false;
}

}  // namespace nga
