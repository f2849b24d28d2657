// Rotary embedding (Llama-3, rotate-half form, theta = 500000 folded into the
// host-built cos/sin table) fused with the paged KV-cache write (K4 + K9).
//
// Cache layout (chosen for the decode/prefill attention kernels' MFMA operand maps):
//   K  cache: [num_blocks, Hkv, BS, D]   (a page of one head = BS rows of D, contiguous)
//   Vt cache: [num_blocks, Hkv, D, BS]   (V stored transposed: keys contiguous per d, so the
//                                          P.V MFMA operand is one 16-B load per lane)
// qkv: [T, (Hq + 2*Hkv) * D] (the fused QKV projection output); q and k are rotated in place.
#include "common.h"
#include "kernels.h"

namespace nga {

template <int D>
__global__ void rope_cache_kernel(uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos,
                                  const float* __restrict__ cos_sin,
                                  const int32_t* __restrict__ slots, uint16_t* __restrict__ kc,
                                  uint16_t* __restrict__ vc, int Hq, int Hkv, int BS) {
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
        uint16_t* dst = kc + ((blk * Hkv + kh) * BS + off) * D;
        *reinterpret_cast<u16x4*>(dst + i0) = oa;
        *reinterpret_cast<u16x4*>(dst + HALF + i0) = ob;
      }
    } else if (slot >= 0) {
      const int r = w - n_rot;
      const int vh = r / (D / 8);
      const int d0 = (r % (D / 8)) * 8;
      u16x8 v = load8(base + (int64_t)(Hq + Hkv + vh) * D + d0);
      uint16_t* dst = vc + ((blk * Hkv + vh) * D + d0) * BS + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[(int64_t)j * BS] = v[j];
    }
  }
}

void launch_rope_cache(uint16_t* qkv, const int32_t* pos, const float* cos_sin,
                       const int32_t* slots, uint16_t* kc, uint16_t* vc, int64_t T, int Hq,
                       int Hkv, int D, int BS, hipStream_t stream) {
  if (T == 0) return;
  dim3 grid((unsigned)T), block(256);
  if (D == 128)
    rope_cache_kernel<128><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, BS);
  else if (D == 64)
    rope_cache_kernel<64><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, BS);
}

}  // namespace nga
