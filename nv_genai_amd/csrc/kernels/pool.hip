// Sentence-embedding pooling + L2 normalisation (K12): CLS or masked-mean pooling over
// packed variable-length sequences (no padding tokens are ever materialised), fp32 output.
#include "common.h"
#include "kernels.h"

namespace nga {

// hidden: [T, H] bf16 packed; cu: [B+1]; out: [B, H] fp32. mode 0 = CLS, 1 = mean.
__global__ void __launch_bounds__(1024) pool_l2norm_kernel(const uint16_t* __restrict__ hidden,
                                                           const int32_t* __restrict__ cu, int H,
                                                           int mode, int normalize,
                                                           float* __restrict__ out) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int s0 = cu[b], s1 = cu[b + 1];
  const int c = threadIdx.x * 8;
  const bool active = c < H;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (active && s1 > s0) {
    if (mode == 0) {
      u16x8 v = load8(hidden + (int64_t)s0 * H + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = bf2f(v[j]);
    } else {
      for (int t = s0; t < s1; ++t) {
        u16x8 v = load8(hidden + (int64_t)t * H + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
      }
      const float inv = 1.f / (float)(s1 - s0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) ss += acc[j] * acc[j];
  ss = block_sum(ss, red);
  const float r = normalize ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
  if (active) {
    f32x4 o0, o1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o0[j] = acc[j] * r;
      o1[j] = acc[4 + j] * r;
    }
    float* dst = out + (int64_t)b * H + c;
    *reinterpret_cast<f32x4*>(dst) = o0;
    *reinterpret_cast<f32x4*>(dst + 4) = o1;
  }
}

// rows of X (bf16) -> squared L2 norm (fp32), used for L2-metric bias and k-means.
__global__ void row_sqnorm_kernel(const uint16_t* __restrict__ X, int64_t N, int D,
                                  float* __restrict__ out) {
  const int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  float s = 0.f;
  for (int c = lane * 8; c < D; c += 64 * 8) {
    u16x8 v = load8(X + row * D + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = bf2f(v[j]);
      s += f * f;
    }
  }
  s = wave_sum(s);
  if (lane == 0) out[row] = s;
}

void launch_pool_l2norm(const uint16_t* hidden, const int32_t* cu, int B, int H, int mode,
                        int normalize, float* out, hipStream_t stream) {
  if (B == 0) return;
  int threads = (H / 8 + 63) / 64 * 64;
  if (threads < 64) threads = 64;
  pool_l2norm_kernel<<<B, threads, 0, stream>>>(hidden, cu, H, mode, normalize, out);
}

void launch_row_sqnorm(const uint16_t* X, int64_t N, int D, float* out, hipStream_t stream) {
  if (N == 0) return;
  row_sqnorm_kernel<<<(unsigned)((N + 3) / 4), 256, 0, stream>>>(X, N, D, out);
}

// Timeline markers: one-thread kernels whose names bracket a region in a kernel trace
// (bench.py's timed window; scripts/summarize_prof.py restricts its busy / gap accounting to
// the span between the end of the begin marker and the start of the end marker). The store
// keeps the kernel from being empty; `sink` is a 4-byte device scratch word.
__global__ void region_begin_marker_kernel(int* sink) { *sink = 1; }
__global__ void region_end_marker_kernel(int* sink) { *sink = 2; }

void launch_region_marker(int end, int* sink, hipStream_t stream) {
  if (end) region_end_marker_kernel<<<1, 1, 0, stream>>>(sink);
  else region_begin_marker_kernel<<<1, 1, 0, stream>>>(sink);
}

}  // namespace nga
