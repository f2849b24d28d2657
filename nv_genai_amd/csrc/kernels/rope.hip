// Rotary embedding (Llama-3, rotate-half form, theta = 500000 folded into the
// host-built cos/sin table) fused with the paged KV-cache write (K4 + K9).
//
// Cache layout (chosen for the decode/prefill attention kernels' MFMA operand maps):
//   K  cache: [num_blocks, Hkv, BS, D]   (a page of one head = BS rows of D, contiguous)
//   Vt cache: [num_blocks, Hkv, D, BS]   (V stored transposed: keys contiguous per d, so the
//                                          P.V MFMA operand is one 16-B load per lane)
// qkv: [T, (Hq + 2*Hkv) * D] (the fused QKV projection output); q and k are rotated in place.
// The caches hold bf16, or fp8 e4m3fn (half the KV bytes; k / v multiplied by 1 / scale
// before rounding, the attention kernels fold the scales back in).
#include "common.h"
#include "kernels.h"

namespace nga {

// CT = cache element: uint16_t (bf16) or uint8_t (fp8 e4m3fn, values multiplied by
// inv_ks / inv_vs before rounding: the per-layer K / V scales)
template <typename CT>
__device__ __forceinline__ void put4(CT* dst, u16x4 v, float inv_s) {
  if constexpr (sizeof(CT) == 2) {
    *reinterpret_cast<u16x4*>(dst) = v;
  } else {
    *reinterpret_cast<uint32_t*>(dst) =
        f32x2_to_fp8(bf2f(v[0]) * inv_s, bf2f(v[1]) * inv_s) |
        (f32x2_to_fp8(bf2f(v[2]) * inv_s, bf2f(v[3]) * inv_s) << 16);
  }
}

template <typename CT>
__device__ __forceinline__ void put8(CT* dst, u16x8 v, float inv_s) {
  if constexpr (sizeof(CT) == 2) {
    store8(dst, v);
  } else {
    uint2 w;
    w.x = f32x2_to_fp8(bf2f(v[0]) * inv_s, bf2f(v[1]) * inv_s) |
          (f32x2_to_fp8(bf2f(v[2]) * inv_s, bf2f(v[3]) * inv_s) << 16);
    w.y = f32x2_to_fp8(bf2f(v[4]) * inv_s, bf2f(v[5]) * inv_s) |
          (f32x2_to_fp8(bf2f(v[6]) * inv_s, bf2f(v[7]) * inv_s) << 16);
    *reinterpret_cast<uint2*>(dst) = w;
  }
}

template <typename CT>
__device__ __forceinline__ void put1(CT* dst, uint16_t v, float inv_s) {
  if constexpr (sizeof(CT) == 2) *dst = v;
  else *dst = f32_to_fp8(bf2f(v) * inv_s);
}

template <int D, typename CT>
__global__ void rope_cache_kernel(uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos,
                                  const float* __restrict__ cos_sin,
                                  const int32_t* __restrict__ slots, CT* __restrict__ kc,
                                  CT* __restrict__ vc, int Hq, int Hkv, int BS, float inv_ks,
                                  float inv_vs) {
  constexpr int HALF = D / 2;
  constexpr int G4 = HALF / 4;  // 4-element groups per half
  const int64_t t = blockIdx.x;
  const int64_t row = (int64_t)(Hq + 2 * Hkv) * D;
  uint16_t* base = qkv + t * row;
  const int p = pos[t];
  const float* cs = cos_sin + (int64_t)p * D;
  const int slot = slots ? slots[t] : -1;
  const int64_t blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;

  const int n_rot = (Hq + Hkv) * G4;
  const int n_v = Hkv * (D / 8);
  for (int w = threadIdx.x; w < n_rot + n_v; w += blockDim.x) {
    if (w < n_rot) {
      const int h = w / G4;  // 0..Hq+Hkv-1 (q heads then k heads, contiguous in qkv)
      const int i0 = (w % G4) * 4;
      uint16_t* x = base + (int64_t)h * D;
      u16x4 a = *reinterpret_cast<const u16x4*>(x + i0);
      u16x4 b = *reinterpret_cast<const u16x4*>(x + HALF + i0);
      u16x4 oa, ob;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = cs[i0 + j], s = cs[HALF + i0 + j];
        const float x1 = bf2f(a[j]), x2 = bf2f(b[j]);
        oa[j] = f2bf(x1 * c - x2 * s);
        ob[j] = f2bf(x2 * c + x1 * s);
      }
      *reinterpret_cast<u16x4*>(x + i0) = oa;
      *reinterpret_cast<u16x4*>(x + HALF + i0) = ob;
      if (h >= Hq && slot >= 0) {
        const int kh = h - Hq;
        CT* dst = kc + ((blk * Hkv + kh) * BS + off) * D;
        put4(dst + i0, oa, inv_ks);
        put4(dst + HALF + i0, ob, inv_ks);
      }
    } else if (slot >= 0) {
      const int r = w - n_rot;
      const int vh = r / (D / 8);
      const int d0 = (r % (D / 8)) * 8;
      u16x8 v = load8(base + (int64_t)(Hq + Hkv + vh) * D + d0);
      CT* dst = vc + ((blk * Hkv + vh) * D + d0) * BS + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) put1(dst + (int64_t)j * BS, v[j], inv_vs);
    }
  }
}

// Tiled form for multi-token steps: grid = (token tiles of 64, Hq + 2*Hkv heads). A q/k head
// block rotates its 64 tokens with 16-B loads/stores (8-element chunks of each half, cos/sin
// as two float4 pairs) and writes k heads to the K cache; a v head block stages the 64 tokens
// x D tile in LDS and writes the transposed page rows with lanes = tokens, so the consecutive
// slots of a prefill chunk become one 128-B store per d row instead of 64 scattered 2-B ones
// per token (the per-token kernel above wrote Vt at ~2 TB/s effective).
constexpr int RT = 64;  // tokens per tile

template <int D, typename CT>
__global__ void __launch_bounds__(256) rope_cache_tiled_kernel(
    uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos, const float* __restrict__ cos_sin,
    const int32_t* __restrict__ slots, CT* __restrict__ kc, CT* __restrict__ vc,
    int64_t T, int Hq, int Hkv, int BS, float inv_ks, float inv_vs) {
  constexpr int HALF = D / 2;
  constexpr int CH = HALF / 8;       // 8-element chunks per half
  constexpr int LDP = D + 2;         // padded LDS row (bank-conflict-free column reads)
  __shared__ uint16_t tile[RT * LDP];
  const int64_t t0 = (int64_t)blockIdx.x * RT;
  const int h = blockIdx.y;
  const int64_t row = (int64_t)(Hq + 2 * Hkv) * D;
  if (h < Hq + Hkv) {
    for (int i = threadIdx.x; i < RT * CH; i += blockDim.x) {
      const int64_t t = t0 + i / CH;
      if (t >= T) break;
      const int i0 = (i % CH) * 8;
      uint16_t* x = qkv + t * row + (int64_t)h * D;
      const float* cs = cos_sin + (int64_t)pos[t] * D;
      const u16x8 a = load8(x + i0), b = load8(x + HALF + i0);
      const float4 c0 = *reinterpret_cast<const float4*>(cs + i0);
      const float4 c1 = *reinterpret_cast<const float4*>(cs + i0 + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(cs + HALF + i0);
      const float4 s1 = *reinterpret_cast<const float4*>(cs + HALF + i0 + 4);
      const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      u16x8 oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x1 = bf2f(a[j]), x2 = bf2f(b[j]);
        oa[j] = f2bf(x1 * c[j] - x2 * sn[j]);
        ob[j] = f2bf(x2 * c[j] + x1 * sn[j]);
      }
      store8(x + i0, oa);
      store8(x + HALF + i0, ob);
      const int slot = (slots && h >= Hq) ? slots[t] : -1;
      if (slot >= 0) {
        CT* dst = kc + (((int64_t)(slot / BS) * Hkv + (h - Hq)) * BS + slot % BS) * D;
        put8(dst + i0, oa, inv_ks);
        put8(dst + HALF + i0, ob, inv_ks);
      }
    }
    return;
  }
  if (slots == nullptr) return;
  const int vh = h - Hq - Hkv;
  // stage V[t0:t0+64, vh, :] (4-byte pairs; padded rows keep 4-B alignment)
  for (int i = threadIdx.x; i < RT * (D / 2); i += blockDim.x) {
    const int r = i / (D / 2), c2 = i % (D / 2);
    const int64_t t = t0 + r;
    uint32_t v = 0;
    if (t < T) v = *reinterpret_cast<const uint32_t*>(qkv + t * row + (int64_t)(Hq + Hkv + vh) * D + 2 * c2);
    *reinterpret_cast<uint32_t*>(tile + r * LDP + 2 * c2) = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t t = t0 + lane;
  const int slot = t < T ? slots[t] : -1;
  if (slot < 0) return;
  CT* dst = vc + ((int64_t)(slot / BS) * Hkv + vh) * D * BS + slot % BS;
  for (int d = w; d < D; d += nw) put1(dst + (int64_t)d * BS, tile[lane * LDP + d], inv_vs);
}

template <typename CT>
static void rope_dispatch(uint16_t* qkv, const int32_t* pos, const float* cos_sin,
                          const int32_t* slots, CT* kc, CT* vc, int64_t T, int Hq, int Hkv, int D,
                          int BS, float inv_ks, float inv_vs, hipStream_t stream) {
  if (T >= RT) {
    dim3 grid((unsigned)((T + RT - 1) / RT), (unsigned)(Hq + 2 * Hkv)), block(256);
#define NGA_RT(DD) rope_cache_tiled_kernel<DD, CT><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, T, Hq, Hkv, BS, inv_ks, inv_vs)
    if (D == 128) NGA_RT(128); else if (D == 256) NGA_RT(256); else if (D == 64) NGA_RT(64);
#undef NGA_RT
    return;
  }
  dim3 grid((unsigned)T), block(256);
#define NGA_R1(DD) rope_cache_kernel<DD, CT><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, BS, inv_ks, inv_vs)
  if (D == 128) NGA_R1(128); else if (D == 256) NGA_R1(256); else if (D == 64) NGA_R1(64);
#undef NGA_R1
}

void launch_rope_cache(uint16_t* qkv, const int32_t* pos, const float* cos_sin,
                       const int32_t* slots, void* kc, void* vc, int64_t T, int Hq,
                       int Hkv, int D, int BS, bool kv_fp8, float inv_ks, float inv_vs,
                       hipStream_t stream) {
  if (T == 0) return;
  if (kv_fp8)
    rope_dispatch(qkv, pos, cos_sin, slots, static_cast<uint8_t*>(kc), static_cast<uint8_t*>(vc), T,
                  Hq, Hkv, D, BS, inv_ks, inv_vs, stream);
  else
    rope_dispatch(qkv, pos, cos_sin, slots, static_cast<uint16_t*>(kc), static_cast<uint16_t*>(vc),
                  T, Hq, Hkv, D, BS, 1.f, 1.f, stream);
}

}  // namespace nga
