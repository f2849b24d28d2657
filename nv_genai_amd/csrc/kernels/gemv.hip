// Weight-streaming GEMV for the smallest decode batches (M = 1..4 token rows):
//
//   out[m, n] = sum_k x[m, k] . W[n, k]        (nn.Linear layout, both K-contiguous)
//
// At M <= 4 a projection is a pure weight stream (Llama-3-8B: 436 MB per layer, ~67 us at
// 6.5 TB/s) and MFMA tiles would be 75-94 % padding. Here x (M x K bf16, at most 160 KiB) is
// staged once per workgroup in LDS; each wave then streams R weight rows with lane-linear
// 16-B loads (one 1-KiB wave instruction per row and 512-element K step, non-temporal: every
// weight byte is read exactly once), multiplies them against the LDS copy of x in fp32 and
// reduces across the wave at the end. Nothing is shared between waves after the x stage, so
// there is no barrier in the stream; many small workgroups per CU keep the loads in flight.
//
// Epilogues: 0 = bf16 out [M, ldo]; 1 = fp32 out [M, ldo] (LM-head logits); 2 = SwiGLU bf16
// out [M, F] from a [gate | up] weight of 2F rows (feature f's gate and up rows in one wave).
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int GV_WAVES = 4;

__device__ __forceinline__ u16x8 load8_nt(const uint16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(p));
}

__device__ __forceinline__ float gv_silu(float x) { return x / (1.f + __expf(-x)); }
}  // namespace

template <int M, int R, int EPI>
__global__ void __launch_bounds__(64 * GV_WAVES) gemv_kernel(GemvParams P) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];   // [M][K]
  const int K = P.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int f0 = (blockIdx.x * GV_WAVES + wv) * R;   // first output feature of this wave
  constexpr int NR = EPI == 2 ? 2 * R : R;   // weight rows streamed per wave
  const uint16_t* wr[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    int f = min(f0 + (r % R), P.N - 1);           // ragged last wave: any valid row, not stored
    const int row = (EPI == 2 && r >= R) ? P.N + f : f;
    wr[r] = P.w + (int64_t)row * K + lane * 8;
  }
  // the first K step's weights are requested before x is staged: the stage's L2 round trip
  // and the weights' HBM round trip overlap instead of running back to back
  u16x8 wcur[NR];
  if (f0 < P.N && lane * 8 < K) {
#pragma unroll
    for (int r = 0; r < NR; ++r) wcur[r] = load8_nt(wr[r]);
  }
  {
    const int per_row = K / 8;
    for (int i = tid; i < M * per_row; i += 64 * GV_WAVES) {
      const int m = i / per_row, c = (i - m * per_row) * 8;
      store8(xs + m * K + c, load8(P.x + (int64_t)m * P.ldx + c));
    }
  }
  __syncthreads();
  if (f0 >= P.N) return;
  float acc[NR][M];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;

#pragma unroll 2
  for (int k = 0; k < K; k += 512) {
    if (k + lane * 8 >= K) break;                 // K % 512 != 0: the tail step's idle lanes
    const bool more = k + 512 + lane * 8 < K;
    u16x8 wnext[NR];
    if (more) {                                   // one K step of weights in flight ahead
#pragma unroll
      for (int r = 0; r < NR; ++r) wnext[r] = load8_nt(wr[r] + k + 512);
    }
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const u16x8 xv = *reinterpret_cast<const u16x8*>(xs + m * K + k + lane * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) xf[m][j] = bf2f(xv[j]);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float wf = bf2f(wcur[r][j]);
#pragma unroll
        for (int m = 0; m < M; ++m) acc[r][m] = __builtin_fmaf(wf, xf[m][j], acc[r][m]);
      }
    if (more) {
#pragma unroll
      for (int r = 0; r < NR; ++r) wcur[r] = wnext[r];
    }
  }
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float v = acc[r][m];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[r][m] = v;
    }
  // lane (r * M + m) writes output (row f0 + r, token m): one store per lane
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (lane != r * M + m || f0 + r >= P.N) continue;
      const int f = f0 + r;
      if constexpr (EPI == 1) {
        reinterpret_cast<float*>(P.out)[(int64_t)m * P.ldo + f] = acc[r][m];
      } else if constexpr (EPI == 2) {
        reinterpret_cast<uint16_t*>(P.out)[(int64_t)m * P.ldo + f] = f2bf(gv_silu(acc[r][m]) * acc[R + r][m]);
      } else {
        reinterpret_cast<uint16_t*>(P.out)[(int64_t)m * P.ldo + f] = f2bf(acc[r][m]);
      }
    }
}

template <int M, int R, int EPI>
static void gemv_launch(const GemvParams& p, hipStream_t stream) {
  const size_t lds = (size_t)M * p.K * 2;
  if (lds > 64 * 1024) {   // only x images past the default limit need the attribute (it loads the kernel)
    static bool attr = [] {
      (void)hipFuncSetAttribute((const void*)gemv_kernel<M, R, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      return true;
    }();
    (void)attr;
  }
  const int waves = (p.N + R - 1) / R;
  dim3 grid((waves + GV_WAVES - 1) / GV_WAVES);
  gemv_kernel<M, R, EPI><<<grid, 64 * GV_WAVES, lds, stream>>>(p);
}

// Rows per wave R: as many as keep >= 2,048 waves (8 per CU) in the grid, at most 4 (EPI 2:
// R features = 2R weight rows). Fewer, longer waves leave too few loads in flight per CU.
bool launch_gemv(const GemvParams& p, int epi, hipStream_t stream) {
  if (p.M < 1 || p.M > 4 || p.N == 0) return false;
  if ((size_t)p.M * p.K * 2 > 160 * 1024) return false;
  const int rows = epi == 2 ? 2 * p.N : p.N;
  const int r = rows >= 4 * 2048 ? 4 : rows >= 2 * 2048 ? 2 : 1;
#define NGA_GV(MM)                                                                 \
  do {                                                                             \
    if (epi == 2) {                                                                \
      if (r == 4) gemv_launch<MM, 2, 2>(p, stream);                                \
      else gemv_launch<MM, 1, 2>(p, stream);                                       \
    } else if (epi == 1) {                                                         \
      if (r == 4) gemv_launch<MM, 4, 1>(p, stream);                                \
      else if (r == 2) gemv_launch<MM, 2, 1>(p, stream);                           \
      else gemv_launch<MM, 1, 1>(p, stream);                                       \
    } else {                                                                       \
      if (r == 4) gemv_launch<MM, 4, 0>(p, stream);                                \
      else if (r == 2) gemv_launch<MM, 2, 0>(p, stream);                           \
      else gemv_launch<MM, 1, 0>(p, stream);                                       \
    }                                                                              \
  } while (0)
  switch (p.M) {
    case 1: NGA_GV(1); break;
    case 2: NGA_GV(2); break;
    case 3: NGA_GV(3); break;
    default: NGA_GV(4); break;
  }
#undef NGA_GV
  return true;
}

}  // namespace nga
