// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * bf16 tensors are passed as raw uint16_t storage; conversion goes through
//     clang's __bf16 so hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
//   * bf16 global traffic is always vectorised to 16 B per lane (8 x bf16).
//   * MFMA tiles use __builtin_amdgcn_mfma_f32_16x16x32_bf16; operand maps
//     (lane l, h = l >> 4):  A[row l&15][k 8h..8h+7],  B[k 8h..8h+7][col l&15],
//     C/D: col = l&15, row = 4h + reg.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nga {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ u16x8 load8(const uint16_t* p) {
  return *reinterpret_cast<const u16x8*>(p);
}

__device__ __forceinline__ void store8(uint16_t* p, u16x8 v) {
  *reinterpret_cast<u16x8*>(p) = v;
}

__device__ __forceinline__ bf16x8 as_bf16x8(u16x8 v) {
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// FP8 (OCP e4m3fn) KV cache helpers. 8 cache bytes <-> 8 bf16 values; every e4m3 value is
// exact in bf16, so reads are lossless. Writes saturate to +-448 (the format has no inf).
// (fp8 -> f32 pairs, then bf16: exact. The one-step v_cvt_scalef32_pk_bf16_fp8 gave the even
// byte's value for the odd one of each pair in a device check, scripts/dev/fp8_cvt_check.hip.)
__device__ __forceinline__ u16x8 fp8x8_to_bf16x8(uint2 w) {
  u16x8 r;
  const uint32_t ws[2] = {w.x, w.y};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(ws[i], false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(ws[i], true);
    r[4 * i] = f2bf(lo[0]);
    r[4 * i + 1] = f2bf(lo[1]);
    r[4 * i + 2] = f2bf(hi[0]);
    r[4 * i + 3] = f2bf(hi[1]);
  }
  return r;
}

__device__ __forceinline__ u16x8 load8_fp8(const uint8_t* p) {
  return fp8x8_to_bf16x8(*reinterpret_cast<const uint2*>(p));
}

__device__ __forceinline__ float fp8_sat(float x) { return fminf(fmaxf(x, -448.f), 448.f); }

// two floats -> two fp8 bytes in the low half of the result
__device__ __forceinline__ uint32_t f32x2_to_fp8(float a, float b) {
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(fp8_sat(a), fp8_sat(b), 0, false) & 0xffffu;
}

__device__ __forceinline__ uint8_t f32_to_fp8(float a) { return (uint8_t)(f32x2_to_fp8(a, 0.f) & 0xffu); }

// LDS-DMA: 16 B per lane global -> LDS; the wave's 64 lanes fill lds_wave_base + lane * 16
// (the LDS address is wave-uniform, it goes through M0). Completion is tracked by vmcnt, not
// lgkmcnt; other waves see the bytes after the issuing wave's vmcnt wait + a barrier.
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
__device__ __forceinline__ void glds16(const uint16_t* src, uint16_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)(src), (lptr_t)(lds_wave_base), 16, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `red` must hold >= blockDim.x/64 floats. All threads get the result.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Counter-based RNG (splitmix64 finaliser) -> uniform in (0, 1].
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return ((float)(z >> 40) + 1.0f) * (1.0f / 16777216.0f);
}

}  // namespace nga
