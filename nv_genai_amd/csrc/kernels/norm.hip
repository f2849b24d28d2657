// RMSNorm (+ fused residual add) for the Llama decoder and LayerNorm
// (+ fused residual add) for the BERT-class encoder.
//
// Memory-bound: one workgroup per row, one 16-B (8 x bf16) vector per lane,
// the row stays in registers between the reduction and the write, so every
// byte is read once and written once (K3 / K11 in SURVEY.md §2.C).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace nga {

// resid (inout, optional) += delta;  out = resid * rsqrt(mean(resid^2) + eps) * w
template <bool ADD>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(uint16_t* __restrict__ out,
                                                       uint16_t* __restrict__ resid,
                                                       const uint16_t* __restrict__ delta,
                                                       const uint16_t* __restrict__ w, float eps,
                                                       int H, int64_t in_stride, int64_t out_stride) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int c = threadIdx.x * 8;
  const bool active = c < H;
  float x[8];
  float ss = 0.f;
  if (active) {
    u16x8 v = load8(resid + row * in_stride + c);
    if (ADD) {
      u16x8 d = load8(delta + row * in_stride + c);
      u16x8 s;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        x[i] = bf2f(v[i]) + bf2f(d[i]);
        s[i] = f2bf(x[i]);
        x[i] = bf2f(s[i]);  // normalise what is stored (matches a bf16 residual stream)
      }
      store8(resid + row * in_stride + c, s);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = bf2f(v[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += x[i] * x[i];
  }
  ss = block_sum(ss, red);
  const float r = rsqrtf(ss / (float)H + eps);
  if (active) {
    u16x8 wv = load8(w + c);
    u16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2bf(x[i] * r * bf2f(wv[i]));
    store8(out + row * out_stride + c, o);
  }
}

// MODE 0: out = LN(x) * g + b
// MODE 1: out = LN(x + resid) * g + b            (BERT post-LN blocks; nothing written back)
// MODE 2: x += resid (stored, bf16); out = LN(x)  (pre-LN decoders: StarCoder2's residual
//         stream, x is the residual and `resid` the block output being added)
template <int MODE>
__global__ void __launch_bounds__(1024) layernorm_kernel(uint16_t* __restrict__ out,
                                                         uint16_t* __restrict__ x_in,
                                                         const uint16_t* __restrict__ resid,
                                                         const uint16_t* __restrict__ g,
                                                         const uint16_t* __restrict__ b, float eps,
                                                         int H) {
  constexpr bool ADD = MODE != 0;
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int c = threadIdx.x * 8;
  const bool active = c < H;
  float x[8];
  float s = 0.f;
  if (active) {
    u16x8 v = load8(x_in + row * H + c);
    if (ADD) {
      u16x8 d = load8(resid + row * H + c);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = bf2f(v[i]) + bf2f(d[i]);
      if (MODE == 2) {
        u16x8 sv;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          sv[i] = f2bf(x[i]);
          x[i] = bf2f(sv[i]);  // normalise the stored bf16 residual
        }
        store8(x_in + row * H + c, sv);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = bf2f(v[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
  }
  const float mean = block_sum(s, red) / (float)H;
  float vs = 0.f;
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = x[i] - mean;
      vs += d * d;
    }
  }
  const float rstd = rsqrtf(block_sum(vs, red) / (float)H + eps);
  if (active) {
    u16x8 gv = load8(g + c), bv = load8(b + c), o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2bf((x[i] - mean) * rstd * bf2f(gv[i]) + bf2f(bv[i]));
    store8(out + row * H + c, o);
  }
}

static int row_threads(int H) {
  int t = (H / 8 + 63) / 64 * 64;
  return t < 64 ? 64 : t;
}

void launch_rmsnorm(uint16_t* out, uint16_t* resid, const uint16_t* delta, const uint16_t* w,
                    float eps, int64_t rows, int H, int64_t in_stride, int64_t out_stride,
                    hipStream_t stream) {
  if (rows == 0) return;
  // One workgroup per row. A wave-per-row form (a row in one wave's registers, 4 rows per
  // workgroup) measured slower at every step size of the headline (add + RMSNorm, 4,096 wide:
  // 1,426 rows 7.2 vs 6.7 us, 4,352 rows 22.5 vs 21.3 us, 256 rows 3.9 both;
  // profiles/r3_decode_step/kb_norm.json) and was removed.
  dim3 grid((unsigned)rows), block(row_threads(H));
  if (delta)
    rmsnorm_kernel<true><<<grid, block, 0, stream>>>(out, resid, delta, w, eps, H, in_stride,
                                                      out_stride);
  else
    rmsnorm_kernel<false><<<grid, block, 0, stream>>>(out, resid, delta, w, eps, H, in_stride,
                                                       out_stride);
}

void launch_layernorm(uint16_t* out, const uint16_t* x, const uint16_t* resid, const uint16_t* g,
                      const uint16_t* b, float eps, int64_t rows, int H, hipStream_t stream) {
  if (rows == 0) return;
  dim3 grid((unsigned)rows), block(row_threads(H));
  uint16_t* xm = const_cast<uint16_t*>(x);  // read-only in modes 0 / 1
  if (resid)
    layernorm_kernel<1><<<grid, block, 0, stream>>>(out, xm, resid, g, b, eps, H);
  else
    layernorm_kernel<0><<<grid, block, 0, stream>>>(out, xm, resid, g, b, eps, H);
}

void launch_add_layernorm(uint16_t* out, uint16_t* resid, const uint16_t* delta, const uint16_t* g,
                          const uint16_t* b, float eps, int64_t rows, int H, hipStream_t stream) {
  if (rows == 0) return;
  dim3 grid((unsigned)rows), block(row_threads(H));
  layernorm_kernel<2><<<grid, block, 0, stream>>>(out, resid, delta, g, b, eps, H);
}

}  // namespace nga
