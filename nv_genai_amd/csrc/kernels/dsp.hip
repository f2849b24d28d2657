// Software-defined-radio front end of the FM-ASR streaming RAG (K18, SURVEY.md §2.B N8;
// experimental/fm-asr-streaming-rag/sdr-holoscan/operators.py:53-84,236-352): complex
// baseband I/Q at 1 MS/s -> FIR low-pass -> FM demodulation -> polyphase decimation to the
// ASR rate -> gain -> 16-bit PCM. Three kernels per burst on the caller's stream.
//
// * fir_c64: y[i] = sum_k h[k] x[i-k] over complex64 samples with real taps; a workgroup
//   stages its 1024-output window plus the (ntaps-1) halo in LDS (history from the previous
//   burst, or zeros, in front of sample 0), so every input sample is read from HBM once.
// * fm_demod: y[i] = arg(x[i] * conj(x[i-1])) — the principal-value phase difference, which
//   is exactly diff(unwrap(angle(x))) without a sequential unwrap pass.
// * resample_pcm: decimating FIR (up = 1): y[m] = sum_k h[k] x[(m + pre) * down - k], then
//   gain and clip(y * 32768) -> int16 (truncation toward zero like numpy's astype).
#include "common.h"
#include "kernels.h"

namespace nga {

constexpr int FIR_TILE = 1024;
constexpr int FIR_MAX_TAPS = 1024;

__global__ void __launch_bounds__(256) fir_c64_kernel(const float2* __restrict__ x, int n,
                                                      const float* __restrict__ taps, int ntaps,
                                                      const float2* __restrict__ hist,
                                                      float2* __restrict__ y) {
  extern __shared__ float smem[];
  float* h = smem;                                        // [ntaps]
  float2* xs = reinterpret_cast<float2*>(smem + ((ntaps + 1) & ~1));  // [FIR_TILE + ntaps - 1]
  const int base = blockIdx.x * FIR_TILE;
  const int halo = ntaps - 1;
  for (int k = threadIdx.x; k < ntaps; k += blockDim.x) h[k] = taps[k];
  for (int j = threadIdx.x; j < FIR_TILE + halo; j += blockDim.x) {
    const int src = base - halo + j;
    float2 v = make_float2(0.f, 0.f);
    if (src >= 0 && src < n) {
      v = x[src];
    } else if (src < 0 && hist != nullptr) {
      v = hist[halo + src];  // hist holds the previous burst's last `halo` samples
    }
    xs[j] = v;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < FIR_TILE; o += blockDim.x) {
    const int i = base + o;
    if (i >= n) break;
    float re = 0.f, im = 0.f;
    // output o uses xs[o + halo - k], k = 0..ntaps-1
    const float2* xp = xs + o + halo;
    for (int k = 0; k < ntaps; ++k) {
      const float2 v = xp[-k];
      re = fmaf(h[k], v.x, re);
      im = fmaf(h[k], v.y, im);
    }
    y[i] = make_float2(re, im);
  }
}

__global__ void fm_demod_kernel(const float2* __restrict__ x, int n, float2 prev, int has_prev,
                                float* __restrict__ y) {
  // has_prev: n outputs (sample 0 differenced against `prev`); else n-1 outputs
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  const int nout = has_prev ? n : n - 1;
  if (o >= nout) return;
  const int i = has_prev ? o : o + 1;
  const float2 a = x[i];
  const float2 b = i > 0 ? x[i - 1] : prev;
  // a * conj(b)
  const float re = a.x * b.x + a.y * b.y;
  const float im = a.y * b.x - a.x * b.y;
  y[o] = atan2f(im, re);
}

__global__ void resample_pcm_kernel(const float* __restrict__ x, int n, const float* __restrict__ h,
                                    int nh, int down, int pre, int nout, float gain,
                                    float* __restrict__ yf, int16_t* __restrict__ yi) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nout) return;
  const int64_t c = (int64_t)(m + pre) * down;  // full-convolution index
  // k ranges over taps with 0 <= c - k < n
  int k0 = (int)max<int64_t>(0, c - (n - 1));
  int k1 = (int)min<int64_t>(nh - 1, c);
  float acc = 0.f;
  for (int k = k0; k <= k1; ++k) acc = fmaf(h[k], x[c - k], acc);
  const float v = gain * acc;
  if (yf) yf[m] = v;
  if (yi) {
    float s = v * 32768.f;
    s = fminf(fmaxf(s, -32768.f), 32767.f);
    yi[m] = (int16_t)s;  // truncation toward zero
  }
}

void launch_fir_c64(const float* x, int n, const float* taps, int ntaps, const float* hist, float* y,
                    hipStream_t stream) {
  if (n <= 0) return;
  const size_t lds = (size_t)((ntaps + 1) & ~1) * sizeof(float) + (size_t)(FIR_TILE + ntaps - 1) * sizeof(float2);
  const int blocks = (n + FIR_TILE - 1) / FIR_TILE;
  hipLaunchKernelGGL(fir_c64_kernel, dim3(blocks), dim3(256), lds, stream,
                     reinterpret_cast<const float2*>(x), n, taps, ntaps,
                     reinterpret_cast<const float2*>(hist), reinterpret_cast<float2*>(y));
}

void launch_fm_demod(const float* x, int n, float prev_re, float prev_im, int has_prev, float* y,
                     hipStream_t stream) {
  const int nout = has_prev ? n : n - 1;
  if (nout <= 0) return;
  hipLaunchKernelGGL(fm_demod_kernel, dim3((nout + 255) / 256), dim3(256), 0, stream,
                     reinterpret_cast<const float2*>(x), n, make_float2(prev_re, prev_im), has_prev, y);
}

void launch_resample_pcm(const float* x, int n, const float* h, int nh, int down, int pre, int nout,
                         float gain, float* yf, int16_t* yi, hipStream_t stream) {
  if (nout <= 0) return;
  hipLaunchKernelGGL(resample_pcm_kernel, dim3((nout + 127) / 128), dim3(128), 0, stream, x, n, h, nh,
                     down, pre, nout, gain, yf, yi);
}

}  // namespace nga
