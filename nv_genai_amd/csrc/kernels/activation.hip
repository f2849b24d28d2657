// Elementwise activations (K5 SwiGLU / GeGLU, K11 bias+GELU). Memory-bound, 16-B vectors,
// grid-stride with a capped grid (Guideline 11).
#include "common.h"
#include "kernels.h"

namespace nga {

// in: [T, 2F] = [gate | up]; out: [T, F] = silu(gate) * up
__global__ void silu_mul_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ in,
                                int64_t T, int F) {
  const int64_t vec_per_row = F / 8;
  const int64_t total = T * vec_per_row;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / vec_per_row;
    const int64_t c = (i - t * vec_per_row) * 8;
    u16x8 g = load8(in + t * 2 * F + c);
    u16x8 u = load8(in + t * 2 * F + F + c);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      const float s = gf / (1.f + __expf(-gf));
      o[j] = f2bf(s * bf2f(u[j]));
    }
    store8(out + t * F + c, o);
  }
}

// tanh-form GELU, 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))), with tanh(u) written
// as 1 - 2 / (1 + e^{2u}) so it costs one exp and one reciprocal
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x - x / (1.f + __expf(2.f * u));
}

// in: [T, 2F] = [gate | up]; out: [T, F] = gelu_tanh(gate) * up   (Gemma GeGLU)
__global__ void gelu_tanh_mul_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ in,
                                     int64_t T, int F) {
  const int64_t vec_per_row = F / 8;
  const int64_t total = T * vec_per_row;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / vec_per_row;
    const int64_t c = (i - t * vec_per_row) * 8;
    u16x8 g = load8(in + t * 2 * F + c);
    u16x8 u = load8(in + t * 2 * F + F + c);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(gelu_tanh(bf2f(g[j])) * bf2f(u[j]));
    store8(out + t * F + c, o);
  }
}

// x: [T, F] inout; x = gelu(x + bias): MODE 0 erf form, 1 tanh approximation, 2 CLIP's
// quick_gelu x * sigmoid(1.702 x)
template <int MODE>
__global__ void bias_gelu_kernel(uint16_t* __restrict__ x, const uint16_t* __restrict__ bias,
                                 int64_t T, int F) {
  const int64_t vec_per_row = F / 8;
  const int64_t total = T * vec_per_row;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / vec_per_row;
    const int64_t c = (i - t * vec_per_row) * 8;
    u16x8 v = load8(x + t * F + c);
    u16x8 b;
    if (bias) b = load8(bias + c);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = bf2f(v[j]) + (bias ? bf2f(b[j]) : 0.f);
      float y;
      if (MODE == 1) y = gelu_tanh(f);
      else if (MODE == 2) y = f / (1.f + __expf(-1.702f * f));
      else y = 0.5f * f * (1.f + erff(f * 0.70710678118654752f));
      o[j] = f2bf(y);
    }
    store8(x + t * F + c, o);
  }
}

static dim3 ew_grid(int64_t vecs) {
  int64_t g = (vecs + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return dim3((unsigned)g);
}

void launch_silu_mul(uint16_t* out, const uint16_t* in, int64_t T, int F, hipStream_t stream) {
  if (T == 0) return;
  silu_mul_kernel<<<ew_grid(T * F / 8), 256, 0, stream>>>(out, in, T, F);
}

void launch_gelu_tanh_mul(uint16_t* out, const uint16_t* in, int64_t T, int F, hipStream_t stream) {
  if (T == 0) return;
  gelu_tanh_mul_kernel<<<ew_grid(T * F / 8), 256, 0, stream>>>(out, in, T, F);
}

void launch_bias_gelu(uint16_t* x, const uint16_t* bias, int64_t T, int F, int mode,
                      hipStream_t stream) {
  if (T == 0) return;
  if (mode == 1)
    bias_gelu_kernel<1><<<ew_grid(T * F / 8), 256, 0, stream>>>(x, bias, T, F);
  else if (mode == 2)
    bias_gelu_kernel<2><<<ew_grid(T * F / 8), 256, 0, stream>>>(x, bias, T, F);
  else
    bias_gelu_kernel<0><<<ew_grid(T * F / 8), 256, 0, stream>>>(x, bias, T, F);
}

}  // namespace nga
