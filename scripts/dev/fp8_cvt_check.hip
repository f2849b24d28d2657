// Standalone check of the fp8 (e4m3fn) -> bf16 widening used by the KV-cache kernels.
#include <cstdio>
#include "../../nv_genai_amd/csrc/kernels/common.h"
using namespace nga;
__global__ void k(const uint8_t* in, uint16_t* out) {
  const u16x8 v = load8_fp8(in + 8 * threadIdx.x);
  for (int j = 0; j < 8; ++j) out[8 * threadIdx.x + j] = v[j];
}
int main() {
  uint8_t h[256];
  for (int i = 0; i < 256; ++i) h[i] = (uint8_t)i;
  uint8_t* d; uint16_t* o;
  hipMalloc(&d, 256); hipMalloc(&o, 512);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  k<<<1, 32>>>(d, o);
  uint16_t r[256];
  hipMemcpy(r, o, 512, hipMemcpyDeviceToHost);
  for (int i = 0; i < 256; ++i) {
    union { uint32_t u; float f; } c; c.u = (uint32_t)r[i] << 16;
    printf("%d %g\n", i, c.f);
  }
  return 0;
}
