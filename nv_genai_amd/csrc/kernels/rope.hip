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

template <typename CT, bool NT = false>
__device__ __forceinline__ void put1(CT* dst, uint16_t v, float inv_s) {
  // NT: a non-temporal store — one token's V^T column touches a different 128-B page row per d,
  // 2 bytes each, and those rows are not in the cache (kernel form rope_vnt, A/B)
  if constexpr (sizeof(CT) == 2) {
    if constexpr (NT) __builtin_nontemporal_store(v, dst);
    else *dst = v;
  } else {
    const CT b = f32_to_fp8(bf2f(v) * inv_s);
    if constexpr (NT) __builtin_nontemporal_store(b, dst);
    else *dst = b;
  }
}

// Source of the qkv values: the bf16 projection output, or (part != nullptr) the S fp32 K-split
// partial slabs of the skinny GEMM [S, T, row], summed here and rounded to bf16 exactly as the
// materialised projection would be — the rotated / copied result is written to qkv either way,
// so the projection output never makes a separate bf16 round trip.
struct QkvSrc {
  const float* part;
  int S;
  int64_t slab;   // T * row
};

__device__ __forceinline__ u16x8 ld8(const uint16_t* qkv, const QkvSrc& src, int64_t i) {
  if (src.part == nullptr) return load8(qkv + i);
  const float* p = src.part + i;
  f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  for (int s = 1; s < src.S; ++s) {
    a += *reinterpret_cast<const f32x4*>(p + s * src.slab);
    b += *reinterpret_cast<const f32x4*>(p + s * src.slab + 4);
  }
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = f2bf(a[j]);
    r[4 + j] = f2bf(b[j]);
  }
  return r;
}

__device__ __forceinline__ u16x4 ld4(const uint16_t* qkv, const QkvSrc& src, int64_t i) {
  if (src.part == nullptr) return *reinterpret_cast<const u16x4*>(qkv + i);
  const float* p = src.part + i;
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  for (int s = 1; s < src.S; ++s) a += *reinterpret_cast<const f32x4*>(p + s * src.slab);
  u16x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = f2bf(a[j]);
  return r;
}

__device__ __forceinline__ uint32_t ld2(const uint16_t* qkv, const QkvSrc& src, int64_t i) {
  if (src.part == nullptr) return *reinterpret_cast<const uint32_t*>(qkv + i);
  const float* p = src.part + i;
  f32x2 a = *reinterpret_cast<const f32x2*>(p);
  for (int s = 1; s < src.S; ++s) a += *reinterpret_cast<const f32x2*>(p + s * src.slab);
  return (uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16);
}

template <int D, typename CT, bool NT = false>
__global__ void rope_cache_kernel(uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos,
                                  const float* __restrict__ cos_sin,
                                  const int32_t* __restrict__ slots, CT* __restrict__ kc,
                                  CT* __restrict__ vc, int Hq, int Hkv, int BS, float inv_ks,
                                  float inv_vs, QkvSrc src) {
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
      const int64_t xi = t * row + (int64_t)h * D;
      u16x4 a = ld4(qkv, src, xi + i0);
      u16x4 b = ld4(qkv, src, xi + HALF + i0);
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
    } else if (slot >= 0 || src.part != nullptr) {
      const int r = w - n_rot;
      const int vh = r / (D / 8);
      const int d0 = (r % (D / 8)) * 8;
      const int64_t vi = (int64_t)(Hq + Hkv + vh) * D + d0;
      u16x8 v = ld8(qkv, src, t * row + vi);
      if (src.part != nullptr) store8(base + vi, v);
      if (slot >= 0) {
        CT* dst = vc + ((blk * Hkv + vh) * D + d0) * BS + off;
#pragma unroll
        for (int j = 0; j < 8; ++j) put1<CT, NT>(dst + (int64_t)j * BS, v[j], inv_vs);
      }
    }
  }
}

// Tiled form for multi-token steps: a workgroup covers RT = 4096 / D tokens (32 at head_dim
// 128) and either a group of `hg` rotary heads (q, then k) or one v head.
// * rotary group: thread = (token, 8-element chunk of each half); it loads its cos/sin once
//   and rotates the chunk in every head of the group (the loads of all heads issued before
//   the math), writing k heads to the K cache too. (One workgroup per head re-read the
//   fp32 cos/sin rows — twice the bytes of the activations — once per head.)
// * v head: stages the RT tokens x D tile in LDS and writes the transposed page rows with
//   lanes = tokens, so the consecutive slots of a prefill chunk become one store per d row
//   instead of scattered 2-B ones per token.
template <int D, typename CT, int NTM = 0>
__global__ void __launch_bounds__(256) rope_cache_tiled_kernel(
    uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos, const float* __restrict__ cos_sin,
    const int32_t* __restrict__ slots, CT* __restrict__ kc, CT* __restrict__ vc,
    int64_t T, int Hq, int Hkv, int BS, int hg, float inv_ks, float inv_vs, QkvSrc src) {
  constexpr int HALF = D / 2;
  constexpr int CH = HALF / 8;       // 8-element chunks per half
  constexpr int RT = 256 / CH;       // tokens per tile (one thread per token and chunk)
  constexpr int LDP = D + 2;         // padded LDS row (bank-conflict-free column reads)
  constexpr int HGMAX = 8;
  __shared__ uint16_t tile[RT * LDP];
  const int64_t t0 = (int64_t)blockIdx.x * RT;
  const int nrot = Hq + Hkv;
  const int ngroups = (nrot + hg - 1) / hg;
  const int64_t row = (int64_t)(Hq + 2 * Hkv) * D;
  if ((int)blockIdx.y < ngroups) {
    const int64_t t = t0 + threadIdx.x / CH;
    if (t >= T) return;
    const int i0 = (threadIdx.x % CH) * 8;
    const int h0 = blockIdx.y * hg, h1 = min(nrot, h0 + hg);
    const float* cs = cos_sin + (int64_t)pos[t] * D;
    const float4 c0 = *reinterpret_cast<const float4*>(cs + i0);
    const float4 c1 = *reinterpret_cast<const float4*>(cs + i0 + 4);
    const float4 s0 = *reinterpret_cast<const float4*>(cs + HALF + i0);
    const float4 s1 = *reinterpret_cast<const float4*>(cs + HALF + i0 + 4);
    uint16_t* xr = qkv + t * row + i0;
    const int64_t xi = t * row + i0;
    u16x8 a[HGMAX], b[HGMAX];
#pragma unroll
    for (int j = 0; j < HGMAX; ++j)
      if (h0 + j < h1) {
        a[j] = ld8(qkv, src, xi + (int64_t)(h0 + j) * D);
        b[j] = ld8(qkv, src, xi + (int64_t)(h0 + j) * D + HALF);
      }
    const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const int slot = slots ? slots[t] : -1;
#pragma unroll
    for (int j = 0; j < HGMAX; ++j) {
      const int h = h0 + j;
      if (h >= h1) break;
      u16x8 oa, ob;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x1 = bf2f(a[j][e]), x2 = bf2f(b[j][e]);
        oa[e] = f2bf(x1 * c[e] - x2 * sn[e]);
        ob[e] = f2bf(x2 * c[e] + x1 * sn[e]);
      }
      store8(xr + (int64_t)h * D, oa);
      store8(xr + (int64_t)h * D + HALF, ob);
      if (h >= Hq && slot >= 0) {
        CT* dst = kc + (((int64_t)(slot / BS) * Hkv + (h - Hq)) * BS + slot % BS) * D + i0;
        put8(dst, oa, inv_ks);
        put8(dst + HALF, ob, inv_ks);
      }
    }
    return;
  }
  if (slots == nullptr && src.part == nullptr) return;
  const int vh = blockIdx.y - ngroups;
  // stage V[t0:t0+RT, vh, :] (4-byte pairs; padded rows keep 4-B alignment); from partial
  // slabs the summed bf16 V is also written back to qkv
  for (int i = threadIdx.x; i < RT * (D / 2); i += blockDim.x) {
    const int r = i / (D / 2), c2 = i % (D / 2);
    const int64_t t = t0 + r;
    uint32_t v = 0;
    if (t < T) {
      const int64_t vi = t * row + (int64_t)(Hq + Hkv + vh) * D + 2 * c2;
      v = ld2(qkv, src, vi);
      if (src.part != nullptr) *reinterpret_cast<uint32_t*>(qkv + vi) = v;
    }
    *reinterpret_cast<uint32_t*>(tile + r * LDP + 2 * c2) = v;
  }
  if (slots == nullptr) return;
  __syncthreads();
  // lane -> (token = lane % RT, d-phase = lane / RT): RT lanes store one d row's tokens
  constexpr int PH = 64 / RT;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int tl = lane % RT, ph = lane / RT;
  const int64_t t = t0 + tl;
  const int slot = t < T ? slots[t] : -1;
  if (slot < 0) return;
  CT* dst = vc + ((int64_t)(slot / BS) * Hkv + vh) * D * BS + slot % BS;
  // NTM 1: every V^T store non-temporal; 2: only a token with no neighbour in the same page row
  // (a decode row: its 2-byte column would leave a dirty partial line in L2 for each of its D
  // page rows), while runs of consecutive slots (prefill chunks) keep cached stores, which the
  // L2 merges into whole lines
  bool nt = NTM == 1;
  if constexpr (NTM == 2) {
    const int sp = t > 0 ? slots[t - 1] : -2, sn = t + 1 < T ? slots[t + 1] : -2;
    nt = !((sp >= 0 && sp + 1 == slot && sp / BS == slot / BS) || (sn == slot + 1 && sn / BS == slot / BS));
  }
  if (nt) {
    for (int d = w * PH + ph; d < D; d += nw * PH) put1<CT, true>(dst + (int64_t)d * BS, tile[tl * LDP + d], inv_vs);
  } else {
    for (int d = w * PH + ph; d < D; d += nw * PH) put1<CT, false>(dst + (int64_t)d * BS, tile[tl * LDP + d], inv_vs);
  }
}

template <typename CT>
static void rope_dispatch(uint16_t* qkv, const int32_t* pos, const float* cos_sin,
                          const int32_t* slots, CT* kc, CT* vc, int64_t T, int Hq, int Hkv, int D,
                          int BS, float inv_ks, float inv_vs, QkvSrc src, hipStream_t stream) {
  const int rt = 4096 / D;   // tokens per tile of the tiled kernel
  const int nt = kernel_form(KF_ROPE_VNT);
  if (T >= rt) {
    // rotary heads per workgroup: enough workgroups to fill the chip, up to 8 heads sharing
    // one cos/sin load
    const int64_t tiles = (T + rt - 1) / rt;
    const int nrot = Hq + Hkv;
    int hg = 8;
    while (hg > 1 && tiles * ((nrot + hg - 1) / hg) < 512) hg /= 2;
    dim3 grid((unsigned)tiles, (unsigned)((nrot + hg - 1) / hg + Hkv)), block(256);
#define NGA_RT(DD)                                                                                      \
  do {                                                                                                  \
    if (nt == 1) rope_cache_tiled_kernel<DD, CT, 1><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, T, Hq, Hkv, BS, hg, inv_ks, inv_vs, src); \
    else if (nt == 2) rope_cache_tiled_kernel<DD, CT, 2><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, T, Hq, Hkv, BS, hg, inv_ks, inv_vs, src); \
    else rope_cache_tiled_kernel<DD, CT><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, T, Hq, Hkv, BS, hg, inv_ks, inv_vs, src); \
  } while (0)
    if (D == 128) NGA_RT(128); else if (D == 256) NGA_RT(256); else if (D == 64) NGA_RT(64);
#undef NGA_RT
    return;
  }
  dim3 grid((unsigned)T), block(256);
#define NGA_R1(DD)                                                                                      \
  do {                                                                                                  \
    if (nt) rope_cache_kernel<DD, CT, true><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, BS, inv_ks, inv_vs, src); \
    else rope_cache_kernel<DD, CT><<<grid, block, 0, stream>>>(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, BS, inv_ks, inv_vs, src); \
  } while (0)
  if (D == 128) NGA_R1(128); else if (D == 256) NGA_R1(256); else if (D == 64) NGA_R1(64);
#undef NGA_R1
}

void launch_rope_cache(uint16_t* qkv, const int32_t* pos, const float* cos_sin,
                       const int32_t* slots, void* kc, void* vc, int64_t T, int Hq,
                       int Hkv, int D, int BS, bool kv_fp8, float inv_ks, float inv_vs,
                       hipStream_t stream, const float* part, int S) {
  if (T == 0) return;
  const QkvSrc src{part, S, T * (int64_t)(Hq + 2 * Hkv) * D};
  if (kv_fp8)
    rope_dispatch(qkv, pos, cos_sin, slots, static_cast<uint8_t*>(kc), static_cast<uint8_t*>(vc), T,
                  Hq, Hkv, D, BS, inv_ks, inv_vs, src, stream);
  else
    rope_dispatch(qkv, pos, cos_sin, slots, static_cast<uint16_t*>(kc), static_cast<uint16_t*>(vc),
                  T, Hq, Hkv, D, BS, 1.f, 1.f, src, stream);
}

}  // namespace nga
