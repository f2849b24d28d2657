// Micro-benchmark: HBM read bandwidth of a KV-page-shaped stream by access pattern, to find
// the ceiling the paged decode attention kernel (attention_decode.hip) is measured against.
// Each wave streams 16 KiB units (one K or V^T page of 64 x 128 bf16) with all of a unit's
// loads in flight before it waits, as the decode kernel does per page:
//   pattern 0: lane-linear 16-B loads (one wave instruction = 1 KiB contiguous)
//   pattern 1: the decode kernel's MFMA-fragment order (one instruction = 16 rows x 64 B)
//   pattern 2: LDS-DMA (global_load_lds_dwordx4, lane-linear) into a per-wave 16 KiB slot
// NT = 1: non-temporal loads. Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/rbw read_bw_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int UNIT = 16384;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

template <int PATTERN, int NT, int UPI>
__global__ void __launch_bounds__(256) rd(const char* __restrict__ buf, long n_units, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char lds[PATTERN == 2 ? 4 * UNIT : 16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long gw = (long)blockIdx.x * 4 + w, nw = (long)gridDim.x * 4;
  unsigned acc = 0;
  for (long u = gw * UPI; u < n_units; u += nw * UPI) {
    if constexpr (PATTERN == 2) {
      const char* base = buf + u * UNIT;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_global_load_lds((gptr_t)(base + i * 1024 + lane * 16),
                                         (lptr_t)(lds + w * UNIT + i * 1024), 16, 0, NT ? 2 : 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc ^= *reinterpret_cast<const unsigned*>(lds + w * UNIT + lane * 16);
    } else {
      u32x4 v[UPI][16];
#pragma unroll
      for (int k = 0; k < UPI; ++k) {
        const char* base = buf + (u + k) * UNIT;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          long off;
          if constexpr (PATTERN == 0) {
            off = i * 1024 + lane * 16;
          } else {   // tile ti = i >> 2 (16 rows), d-step s = i & 3; lane: row l & 15, 16-B chunk l >> 4
            const int row = 16 * (i >> 2) + (lane & 15);
            off = row * 256 + (i & 3) * 64 + (lane >> 4) * 16;
          }
          const u32x4* p = reinterpret_cast<const u32x4*>(base + off);
          v[k][i] = NT ? __builtin_nontemporal_load(p) : *p;
        }
      }
#pragma unroll
      for (int k = 0; k < UPI; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= v[k][i][0] ^ v[k][i][3];
    }
  }
  out[(long)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int P, int NT, int UPI>
double run(const char* buf, long n_units, unsigned* out, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  rd<P, NT, UPI><<<grid, 256>>>(buf, n_units, out);
  CK(hipDeviceSynchronize());
  const int it = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < it; ++i) rd<P, NT, UPI><<<grid, 256>>>(buf, n_units, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return (double)n_units * UNIT * it / (ms * 1e-3) / 1e12;
}

int main() {
  const long n_units = 131072;   // 2 GiB
  char* buf;
  unsigned* out;
  CK(hipMalloc(&buf, n_units * UNIT));
  CK(hipMemset(buf, 1, n_units * UNIT));
  CK(hipMalloc(&out, 65536L * 256 * 4));
  printf("{");
  const int grids[] = {1024, 2048, 4096, 8192};
  bool first = true;
  for (int g : grids) {
    double r[8] = {run<0, 0, 1>(buf, n_units, out, g), run<0, 0, 2>(buf, n_units, out, g),
                   run<1, 0, 1>(buf, n_units, out, g), run<1, 0, 2>(buf, n_units, out, g),
                   run<0, 1, 2>(buf, n_units, out, g), run<1, 1, 2>(buf, n_units, out, g),
                   run<2, 0, 1>(buf, n_units, out, g), run<2, 1, 1>(buf, n_units, out, g)};
    printf("%s\"grid%d\": {\"linear_1u\": %.2f, \"linear_2u\": %.2f, \"mfma_1u\": %.2f, \"mfma_2u\": %.2f, "
           "\"linear_2u_nt\": %.2f, \"mfma_2u_nt\": %.2f, \"glds_1u\": %.2f, \"glds_1u_nt\": %.2f}",
           first ? "" : ", ", g, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
    first = false;
  }
  printf("}\n");
  return 0;
}
