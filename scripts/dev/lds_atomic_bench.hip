// Micro-benchmark: cost of an LDS histogram pass over 256 rows x 128K fp32 values (one
// 1024-thread workgroup per row), by atomic flavour. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int NT = 1024, NB = 2048, V = 128256, B = 256;

__device__ __forceinline__ float hash_norm(uint32_t i) {
  uint32_t a = i * 2654435761u ^ 0x9e3779b9u, b = (i + 7u) * 2246822519u ^ 0x85ebca6bu;
  a ^= a >> 15; a *= 0x2c1b3c6du; a ^= a >> 12; b ^= b >> 13; b *= 0x297a2d39u; b ^= b >> 16;
  const float u1 = ((a >> 8) + 1) * (1.f / 16777217.f), u2 = (b >> 8) * (1.f / 16777216.f);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
}

__global__ void fill(float* x, float scale) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (size_t)B * V) x[i] = scale * hash_norm((uint32_t)i);
}

template <int MODE>
__global__ void __launch_bounds__(NT) hist(const float* __restrict__ xs, float M, float* out) {
  __shared__ float hf[NB];
  __shared__ uint32_t hu[NB];
  __shared__ float hp[16][NB / 4];
  __shared__ unsigned long long hq[NB];
  const int t = threadIdx.x;
  for (int i = t; i < NB; i += NT) { hf[i] = 0.f; hu[i] = 0u; hq[i] = 0ull; }
  for (int i = t; i < 16 * NB / 4; i += NT) (&hp[0][0])[i] = 0.f;
  __syncthreads();
  const float4* x4 = reinterpret_cast<const float4*>(xs + (size_t)blockIdx.x * V);
  float acc = 0.f;
  for (int j = t; j < V / 4; j += NT) {
    const float4 v4 = x4[j];
    const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = M - vv[e];
      if (d < 16.f) {
        const int b = NB - 1 - min((int)(d * 128.f), NB - 1);
        const float w = __expf(-d);
        if (MODE == 0) acc += w * (float)b;
        if (MODE == 1) atomicAdd(&hf[b], w);
        if (MODE == 2) atomicAdd(&hu[b], 1u);
        if (MODE == 3) atomicAdd(&hp[t >> 6][b >> 2], w);   // per-wave copy, 512 bins
        if (MODE == 4) atomicAdd(&hf[b], 1.f);
        if (MODE == 5) atomicAdd(&hq[b], (unsigned long long)(w * 1099511627776.f));
      }
    }
  }
  __syncthreads();
  if (t == 0) out[blockIdx.x] = acc + hf[t] + hu[t] + hp[0][t] + (float)hq[t];
}

template <int MODE>
float run(const float* x, float M, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hist<MODE><<<B, NT>>>(x, M, out);
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) hist<MODE><<<B, NT>>>(x, M, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 20 * 1e3f;
}

int main() {
  float *x, *out;
  hipMalloc(&x, sizeof(float) * (size_t)B * V);
  hipMalloc(&out, sizeof(float) * B);
  const float scales[3] = {0.5f, 3.f, 15.f};
  for (float s : scales) {
    fill<<<((size_t)B * V + 255) / 256, 256>>>(x, s);
    const float M = 4.3f * s;
    printf("{\"sigma\": %.1f, \"none_us\": %.1f, \"f32_us\": %.1f, \"u32_us\": %.1f, \"perwave_f32_us\": %.1f, \"f32_ones_us\": %.1f, \"u64_fixed_us\": %.1f}\n",
           s, run<0>(x, M, out), run<1>(x, M, out), run<2>(x, M, out), run<3>(x, M, out), run<4>(x, M, out), run<5>(x, M, out));
  }
  hipFree(x); hipFree(out);
  return 0;
}
