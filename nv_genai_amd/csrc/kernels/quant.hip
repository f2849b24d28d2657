// Row-wise FP8 (OCP e4m3fn, gfx950's native FP8) activation quantisation for the W8A8
// serving mode: the GEMM inputs of a layer (normed hidden, attention output, SwiGLU output)
// are quantised per token row, y = cvt_e4m3(x / s) with s = max|x| / 448, so a row-scaled
// hipBLASLt FP8 GEMM (torch._scaled_mm, scale_a[M,1] x scale_b[1,N]) reproduces x @ W^T.
// Weights are quantised once per output channel at load time.
//
// One 256-thread block per row, two passes over the row (absmax, then convert; the second
// read hits L2): 16-B bf16 loads, packed conversions (v_cvt_pk_fp8_f32, round-to-nearest-even,
// inputs clamped to +-448 first so nothing saturates to NaN), 8-B stores.
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr float FP8_MAX = 448.f;

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, FP8_MAX, -FP8_MAX);
  b = __builtin_amdgcn_fmed3f(b, FP8_MAX, -FP8_MAX);
  c = __builtin_amdgcn_fmed3f(c, FP8_MAX, -FP8_MAX);
  d = __builtin_amdgcn_fmed3f(d, FP8_MAX, -FP8_MAX);
  uint32_t r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }
}  // namespace

// x: [rows, H] bf16 (row stride ldx) -> y: [rows, H] fp8 (contiguous), scale[row]
// mode 0: y = q(x); mode 1 (SwiGLU): x is [rows, 2H] = [gate | up], y = q(silu(gate) * up)
template <int MODE>
__global__ void __launch_bounds__(256) quant_fp8_rows_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                             int H, uint8_t* __restrict__ y,
                                                             float* __restrict__ scale) {
  __shared__ float red[8];
  const int64_t r = blockIdx.x;
  const uint16_t* xr = x + r * ldx;
  auto val8 = [&](int c, float* v) {
    const u16x8 a = load8(xr + c);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
    } else {
      const u16x8 u = load8(xr + H + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = silu(bf2f(a[j])) * bf2f(u[j]);
    }
  };
  float amax = 0.f;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    float v[8];
    val8(c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
  }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-12f) / FP8_MAX;
  const float inv = 1.f / s;
  uint8_t* yr = y + r * (int64_t)H;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    float v[8];
    val8(c, v);
    uint2 o;
    o.x = pack4_fp8(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
    o.y = pack4_fp8(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
    *reinterpret_cast<uint2*>(yr + c) = o;
  }
  if (threadIdx.x == 0) scale[r] = s;
}

void launch_quant_fp8_rows(const uint16_t* x, int64_t ldx, int64_t rows, int H, int mode, uint8_t* y,
                           float* scale, hipStream_t stream) {
  if (rows == 0) return;
  if (mode == 0)
    quant_fp8_rows_kernel<0><<<(unsigned)rows, 256, 0, stream>>>(x, ldx, H, y, scale);
  else
    quant_fp8_rows_kernel<1><<<(unsigned)rows, 256, 0, stream>>>(x, ldx, H, y, scale);
}

}  // namespace nga
