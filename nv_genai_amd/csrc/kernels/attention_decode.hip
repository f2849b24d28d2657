// Paged decode attention with GQA on MFMA (K2 in SURVEY.md §2.C), head_dim 128 / 256,
// optional sliding window.
//
// One query token per sequence. For a (sequence, kv-head) pair the G = Hq/Hkv query rows
// that share the kv head form the 16 columns of an MFMA tile (padded with zero rows), so
// K and V are read from HBM exactly once per (sequence, kv-head) — the kernel is bound by
// the KV stream, which is ~half the bytes of a Llama-3-8B decode step at RAG context lengths.
//
// Per 64-key page (= one KV-cache block, BS = 64) and per wave:
//   S^T[key, q] = K[key, :] . Q[q, :]^T       4 tiles x 4 d-steps of mfma_f32_16x16x32_bf16
//   online softmax over keys (exp2 domain), keys of a q column live in 4 lanes x 16 regs
//   O^T[d, q]  += Vt[d, key] . P^T[key, q]     2 key-groups x 8 d-tiles
// The S accumulator is consumed as the P^T B-operand with no lane movement: tile rows are
// mapped to physical keys as key = 32*g + 8*(row>>2) + 4*t1 + (row&3) so that lane group h
// holds keys 32g+8h .. 32g+8h+7 — exactly the 8 consecutive keys the Vt A-operand load
// (one 16-B load from the transposed V page) provides.
//
// Work split: grid = (seqs, kv_heads, partitions); 4 waves per workgroup stride over the
// partition's pages; waves combine through LDS; partitions (flash-decoding split-K, used
// when seqs*kv_heads is too small to fill 256 CUs) combine in a second small kernel. A
// sequence's pages are divided evenly over the partitions at run time (pages_per_part only
// sizes the grid), so the split adapts to each sequence's real context length.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int BS = 64;
constexpr int NW = 4;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float RESCALE_LOG2 = 8.f;
}  // namespace

// D = head_dim (128 or 256). For D = 128 a page's 64 keys are loaded and softmaxed in one
// pass (KH = 2 key groups of 32); for D = 256 the K / Vt fragments of a whole page would need
// 256 VGPRs, so the page is processed as two 32-key passes with their own online-softmax
// update (KH = 1). WINDOW > 0 (sliding-window attention): the query at position ctx - 1 sees
// keys (ctx - 1 - window, ctx - 1]; pages wholly before the window are never read.
// CT = cache element: uint16_t (bf16) or uint8_t (fp8 e4m3fn: 8-byte fragment loads widened
// to bf16 in registers; the K scale is folded into `scale` by the launcher, the V scale
// multiplies the output)
template <int D, typename CT>
__global__ void __launch_bounds__(256) decode_attn_kernel(
    uint16_t* __restrict__ out, int64_t out_stride, const uint16_t* __restrict__ q,
    int64_t q_stride, const CT* __restrict__ kc, const CT* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks,
    const int32_t* __restrict__ ctx_lens, int Hq, int Hkv, float scale, int pages_per_part,
    float* __restrict__ part_ml, float* __restrict__ part_o, int window, float v_scale, int skip_empty,
    int nt_loads) {
  // fp8 pages at head_dim 128: 16-byte loads (half as many load instructions as 8-byte ones).
  // Each lane's 16 K bytes cover two d-steps (Q is loaded with the same d order, the dot
  // product does not care) and its 16 Vt bytes cover 16 consecutive keys of both key
  // groups: tile rows map to keys as key = 16 (row >> 2) + 8 g + 4 t1 + (row & 3), so lane
  // group h holds keys 16h + 8g .. 16h + 8g + 7 (bf16 pages keep the 32g + 8h + ... order).
  constexpr bool F8 = sizeof(CT) == 1;
  constexpr bool W16 = F8 && D == 128;
  constexpr int DS = D / 32;   // d-steps of the QK^T MFMA
  constexpr int DT = D / 16;   // d-tiles of the PV MFMA
  constexpr int KH = D <= 128 ? 2 : 1;  // 32-key groups per softmax pass
  constexpr int NPASS = 2 / KH;
  const int b = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z, nparts = gridDim.z;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int ctx = ctx_lens[b];
  const int n_pages = (ctx + BS - 1) / BS;
  const int key_lo = window > 0 ? max(0, ctx - window) : 0;   // first visible key
  const int p_lo = key_lo / BS;
  // each sequence's own (visible) pages split evenly over the grid's partitions, so a split
  // sized for the batch (hipGraph-captured with the worst-case context) still divides short
  // contexts — but never below one page per wave: a partition of 1-2 pages leaves most of
  // its waves idle and pays the workgroup's fixed cost for nothing (the surplus partitions
  // of a short context just report empty)
  const int ppp = max(NW, (n_pages - p_lo + nparts - 1) / nparts);
  const int p_begin = p_lo + part * ppp;
  const int p_end = min(n_pages, p_begin + ppp);

  __shared__ float o_s[NW][16][D + 4];
  __shared__ float m_s[NW][16], l_s[NW][16];
  if (p_begin >= p_end) {
    // empty partition (or an empty padding sequence, ctx = 0). skip_empty: a ctx-0 row is not
    // this launch's row at all (a mixed-step graph covers a bucket of rows, the ones past the
    // step's decode rows belong to its prefill tokens) and is left untouched
    if (skip_empty && ctx == 0) return;
    if (nparts == 1) {
      for (int i = threadIdx.x; i < G * D; i += blockDim.x)
        out[(int64_t)b * out_stride + (int64_t)(kvh * G) * D + i] = 0;
    } else {
      for (int i = threadIdx.x; i < G; i += blockDim.x) {
        const int64_t idx = ((int64_t)b * Hq + kvh * G + i) * nparts + part;
        part_ml[2 * idx] = -INFINITY;
        part_ml[2 * idx + 1] = 0.f;
      }
    }
    return;
  }

  // Q^T as the B operand: lane holds Q[q=col][d = 32s + 8h + j]
  bf16x8 qf[DS];
  {
    const bool qv = col < G;
    const uint16_t* qp = q + (int64_t)b * q_stride + (int64_t)(kvh * G + (qv ? col : 0)) * D;
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      u16x8 v = load8(qp + (W16 ? 64 * (s >> 1) + 16 * h + 8 * (s & 1) : 32 * s + 8 * h));
      if (!qv) v = (u16x8)(0);
      qf[s] = as_bf16x8(v);
    }
  }

  const float sl2 = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4)(0.f);

  const int32_t* bt = block_tables + (int64_t)b * max_blocks;
  for (int p = p_begin + w; p < p_end; p += NW) {
    const int64_t blk = bt[p];
    const CT* kp = kc + (blk * Hkv + kvh) * (int64_t)(BS * D);
    const CT* vp = vc + (blk * Hkv + kvh) * (int64_t)(D * BS);
    const int kbase = p * BS;
    const bool full = kbase + BS <= ctx && kbase >= key_lo;
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
      // K operand loads: tile tau (g = tau>>1, t1 = tau&1), row = col
      // bf16 fragments, or the raw fp8 words: widened right before their MFMA, so the loads
      // in flight take half the registers
      u16x8 kf[2 * KH][DS];
      u16x8 vf[KH][DT];
      uint2 kw[2 * KH][DS], vw[KH][DT];
      if constexpr (W16) {
        const uint8_t* kb = reinterpret_cast<const uint8_t*>(kp);
        const uint8_t* vb = reinterpret_cast<const uint8_t*>(vp);
#pragma unroll
        for (int ti = 0; ti < 2 * KH; ++ti) {
          const int key = 16 * (col >> 2) + 8 * (ti >> 1) + 4 * (ti & 1) + (col & 3);
#pragma unroll
          for (int pp = 0; pp < DS / 2; ++pp) {
            const uint4 w = *reinterpret_cast<const uint4*>(kb + key * D + 64 * pp + 16 * h);
            kw[ti][2 * pp] = make_uint2(w.x, w.y);
            kw[ti][2 * pp + 1] = make_uint2(w.z, w.w);
          }
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const uint4 w = *reinterpret_cast<const uint4*>(vb + (16 * dt + col) * BS + 16 * h);
          vw[0][dt] = make_uint2(w.x, w.y);
          vw[1][dt] = make_uint2(w.z, w.w);
        }
      } else {
#pragma unroll
        for (int ti = 0; ti < 2 * KH; ++ti) {
          const int tau = 2 * KH * pass + ti;
          const int key = 32 * (tau >> 1) + 8 * (col >> 2) + 4 * (tau & 1) + (col & 3);
#pragma unroll
          for (int s = 0; s < DS; ++s) {
            const CT* src = kp + key * D + 32 * s + 8 * h;
            if constexpr (F8) kw[ti][s] = *reinterpret_cast<const uint2*>(src);
            else kf[ti][s] = nt_loads ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(src))
                                      : load8(src);
          }
        }
#pragma unroll
        for (int gi = 0; gi < KH; ++gi) {
          const int g = KH * pass + gi;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const CT* src = vp + (16 * dt + col) * BS + 32 * g + 8 * h;
            if constexpr (F8) vw[gi][dt] = *reinterpret_cast<const uint2*>(src);
            else vf[gi][dt] = nt_loads ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(src))
                                       : load8(src);
          }
        }
      }

      f32x4 sacc[2 * KH];
#pragma unroll
      for (int ti = 0; ti < 2 * KH; ++ti) {
        sacc[ti] = (f32x4)(0.f);
#pragma unroll
        for (int s = 0; s < DS; ++s)
          sacc[ti] = mfma16(as_bf16x8(F8 ? fp8x8_to_bf16x8(kw[ti][s]) : kf[ti][s]), qf[s], sacc[ti]);
      }
      // mask (the sequence's last, partial page; the window's first page); lane's keys:
      // 32g + 8h + 4t1 + r for tile tau = 2g + t1, reg r. Raw scores: the softmax scale is
      // folded into the exp2 FMA.
      float mloc = -INFINITY;
      if (full) {
#pragma unroll
        for (int ti = 0; ti < 2 * KH; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, sacc[ti][r]);
      } else {
#pragma unroll
        for (int ti = 0; ti < 2 * KH; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int tau = 2 * KH * pass + ti;
            const int key = kbase + (W16 ? 16 * h + 8 * (tau >> 1) : 32 * (tau >> 1) + 8 * h) +
                            4 * (tau & 1) + r;
            const float sv = (key < ctx && key >= key_lo) ? sacc[ti][r] : -INFINITY;
            sacc[ti][r] = sv;
            mloc = fmaxf(mloc, sv);
          }
      }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      mloc *= sl2;  // scale > 0: max commutes with it
      // Lazy rescaling (as in the prefill kernel): the running max only moves, and O / l are
      // only rescaled, when a pass's max exceeds it by more than 2^RESCALE_LOG2; until then
      // P = 2^(s - m) <= 2^8 stays harmless in fp32 l / O and bf16 P. m starts at -inf, so
      // the first pass with a visible key rescales (alpha = 2^-inf = 0 on the all-zero O). A
      // pass can be fully masked (D = 256 halves, window edges): m may still be -inf then, so
      // the exponent offset uses 0 instead (2^-inf = 0 either way).
      if (mloc > m + RESCALE_LOG2) {
        const float alpha = __builtin_amdgcn_exp2f(m - mloc);
        m = mloc;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      }
      const float mo = m == -INFINITY ? 0.f : -m;
      bf16x8 pf[KH];
#pragma unroll
      for (int gi = 0; gi < KH; ++gi)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(sacc[2 * gi + (j >> 2)][j & 3], sl2, mo));  // 2^-inf = 0
          l += pv;
          pf[gi][j] = (__bf16)pv;
        }
#pragma unroll
      for (int gi = 0; gi < KH; ++gi)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          o[dt] = mfma16(as_bf16x8(F8 ? fp8x8_to_bf16x8(vw[gi][dt]) : vf[gi][dt]), pf[gi], o[dt]);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  // wave partials -> LDS. O^T layout: lane holds O[q=col][d = 16dt + 4h + r]
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) o_s[w][col][16 * dt + 4 * h + r] = o[dt][r];
  if (h == 0) {
    m_s[w][col] = m;
    l_s[w][col] = l;
  }
  __syncthreads();

  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int qi = i / D, d = i % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, m_s[ww][qi]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float f = (m_s[ww][qi] == -INFINITY) ? 0.f : exp2f(m_s[ww][qi] - M);
      L += f * l_s[ww][qi];
      acc += f * o_s[ww][qi][d];
    }
    acc *= v_scale;
    const int hq = kvh * G + qi;
    if (nparts == 1) {
      out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
    } else {
      const int64_t idx = ((int64_t)b * Hq + hq) * nparts + part;
      part_o[idx * D + d] = acc;
      if (d == 0) {
        part_ml[2 * idx] = M;
        part_ml[2 * idx + 1] = L;
      }
    }
  }
}

// LDS-DMA form for bf16 head_dim-128 pages (the serving shape). The register form above
// loads each MFMA fragment straight from HBM: one wave instruction reads 16 rows x 64 B, half
// of each 128-B line, and a page-shaped stream in that order tops out near 6.0 TB/s, while
// lane-linear 1-KiB instructions reach 6.9 TB/s with non-temporal loads and LDS-DMA 6.5-6.8
// (scripts/dev/read_bw_probe.hip, profiles/r3_bw/read_bw.json). Here each wave streams its
// page's K and V^T (32 KiB) by non-temporal LDS-DMA, one contiguous 1 KiB per instruction,
// into its own LDS slot, XOR-swizzled through the source address (the prefill kernels'
// swizzles, bank-conflict-free fragment reads); reads the fragments with ds_read_b128; and
// issues the next page's DMA before computing this one. A wave only touches its own slot, so
// the page loop has no barrier. 128 KiB of LDS: one workgroup (4 waves) per CU.
namespace {
constexpr int DSLOT = 2 * BS * 128;   // elements of one wave's slot: K page + V^T page
constexpr int DMA_MAX_PAGES = 1024;   // block ids of a workgroup's partition staged in LDS
__device__ __forceinline__ int dkswz(int row) { return (row & 3) | (((row >> 3) & 3) << 2); }
__device__ __forceinline__ int dvswz(int row) { return (row >> 1) & 7; }
}  // namespace

// RING = true (NGA_DECODE_DMA=2): the wave's K and V^T buffers are refilled separately. With
// one whole-page DMA the wave waits for K and V^T together, reads both and only then issues the
// next page, so nothing of its own is in flight while it reads. In the ring form the next K
// goes out once this K is in registers and the next V^T once this V^T is, so one 16-KiB DMA is
// always in flight. (A half-page ring, 32-key units, read each V^T row's 128-B line in two
// 64-B halves and ran at 4.7 TB/s against 6.7.)
// AUX: cache policy of the KV-page DMA loads (form decode_dma_aux): 2 = nt (each page is read
// once per step), 0 = default policy
template <bool RING, int AUX>
__global__ void __launch_bounds__(256, 1) decode_attn_dma_kernel(
    uint16_t* __restrict__ out, int64_t out_stride, const uint16_t* __restrict__ q,
    int64_t q_stride, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks,
    const int32_t* __restrict__ ctx_lens, int Hq, int Hkv, float scale,
    float* __restrict__ part_ml, float* __restrict__ part_o, int window, int skip_empty) {
  constexpr int D = 128, DS = 4, DT = 8;
  // ONE LDS object (a second one makes the compiler drain the DMA before fragment reads):
  // the waves' page slots, reused by the wave combine after the loop
  __shared__ __attribute__((aligned(16))) uint16_t smem[NW * DSLOT + 2 * DMA_MAX_PAGES];
  const int b = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z, nparts = gridDim.z;
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int ctx = ctx_lens[b];
  const int n_pages = (ctx + BS - 1) / BS;
  const int key_lo = window > 0 ? max(0, ctx - window) : 0;
  const int p_lo = key_lo / BS;
  const int ppp = max(NW, (n_pages - p_lo + nparts - 1) / nparts);
  const int p_begin = p_lo + part * ppp;
  const int p_end = min(n_pages, p_begin + ppp);
  if (p_begin >= p_end) {   // as decode_attn_kernel
    if (skip_empty && ctx == 0) return;
    if (nparts == 1) {
      for (int i = threadIdx.x; i < G * D; i += blockDim.x)
        out[(int64_t)b * out_stride + (int64_t)(kvh * G) * D + i] = 0;
    } else {
      for (int i = threadIdx.x; i < G; i += blockDim.x) {
        const int64_t idx = ((int64_t)b * Hq + kvh * G + i) * nparts + part;
        part_ml[2 * idx] = -INFINITY;
        part_ml[2 * idx + 1] = 0.f;
      }
    }
    return;
  }

  uint16_t* const ks = smem + w * DSLOT;
  uint16_t* const vs = ks + BS * D;
  const int32_t* bt = block_tables + (int64_t)b * max_blocks;
  // DMA instruction i fills slot bytes [1 KiB i, +1 KiB): K keys 4i .. 4i+3 (lane: key
  // 4i + (l >> 4), 16-B position l & 15 holding logical chunk (l & 15) ^ kswz(key)); V^T rows
  // 8i .. 8i+7 (lane: row 8i + (l >> 3), position l & 7 holding chunk (l & 7) ^ vswz(row))
  auto issue = [&](int64_t blk) {
    const char* kp = reinterpret_cast<const char*>(kc + (blk * Hkv + kvh) * (int64_t)(BS * D));
    const char* vp = reinterpret_cast<const char*>(vc + (blk * Hkv + kvh) * (int64_t)(D * BS));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 4 * i + (lane >> 4);
      __builtin_amdgcn_global_load_lds((gptr_t)(kp + key * 256 + (((lane & 15) ^ dkswz(key)) << 4)),
                                       (lptr_t)(ks + i * 512), 16, 0, AUX);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 8 * i + (lane >> 3);
      __builtin_amdgcn_global_load_lds((gptr_t)(vp + row * 128 + (((lane & 7) ^ dvswz(row)) << 4)),
                                       (lptr_t)(vs + i * 512), 16, 0, AUX);
    }
  };

  const float sl2 = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4)(0.f);

  // the partition's block ids in LDS: a VMEM block-id load in the loop would be sunk past the
  // page wait by the compiler and then waited for on its own before every next-page DMA
  int32_t* const sbt = reinterpret_cast<int32_t*>(smem + NW * DSLOT);
  for (int i = threadIdx.x; i < p_end - p_begin; i += blockDim.x) sbt[i] = bt[p_begin + i];
  __syncthreads();
  if constexpr (RING) {
    // the slot as a ring of two 16-KiB DMA units, the wave's page k's K (buffer ks) and V^T
    // (buffer vs): K(k+1) is issued as soon as K(k) is in registers, so it streams during page
    // k's scores and softmax; V(k+1) as soon as V(k) is, during page k's P.V
    const int my_pages = p_begin + w < p_end ? (p_end - 1 - (p_begin + w)) / NW + 1 : 0;
    auto blk_of = [&](int k) { return (int64_t)sbt[w + NW * k]; };
    auto issue_k = [&](int64_t blk) {
      const char* kp = reinterpret_cast<const char*>(kc + (blk * Hkv + kvh) * (int64_t)(BS * D));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = 4 * i + (lane >> 4);
        __builtin_amdgcn_global_load_lds((gptr_t)(kp + key * 256 + (((lane & 15) ^ dkswz(key)) << 4)),
                                         (lptr_t)(ks + i * 512), 16, 0, AUX);
      }
    };
    auto issue_v = [&](int64_t blk) {
      const char* vp = reinterpret_cast<const char*>(vc + (blk * Hkv + kvh) * (int64_t)(D * BS));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = 8 * i + (lane >> 3);
        __builtin_amdgcn_global_load_lds((gptr_t)(vp + row * 128 + (((lane & 7) ^ dvswz(row)) << 4)),
                                         (lptr_t)(vs + i * 512), 16, 0, AUX);
      }
    };
    if (my_pages > 0) {
      issue_k(blk_of(0));
      issue_v(blk_of(0));
    }
    bf16x8 qf[DS];
    {
      const bool qv = col < G;
      const uint16_t* qp = q + (int64_t)b * q_stride + (int64_t)(kvh * G + (qv ? col : 0)) * D;
#pragma unroll
      for (int s = 0; s < DS; ++s) {
        u16x8 v = load8(qp + 32 * s + 8 * h);
        if (!qv) v = (u16x8)(0);
        qf[s] = as_bf16x8(v);
      }
    }
    // Q is consumed here, so the compiler's wait for it (a full vmcnt drain beside the DMAs)
    // lands before the loop and not inside it
#pragma unroll
    for (int s = 0; s < DS; ++s) asm volatile("" ::"v"(qf[s]));
    for (int k = 0; k < my_pages; ++k) {
      const bool more = k + 1 < my_pages;
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // K(k) landed (V(k) may not have)
      u16x8 kf[4][DS];
#pragma unroll
      for (int ti = 0; ti < 4; ++ti) {
        const int key = 32 * (ti >> 1) + 8 * (col >> 2) + 4 * (ti & 1) + (col & 3);
#pragma unroll
        for (int s = 0; s < DS; ++s)
          kf[ti][s] = *reinterpret_cast<const u16x8*>(ks + key * D + (((4 * s + h) ^ dkswz(key)) << 3));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // K buffer free
      if (more) issue_k(blk_of(k + 1));

      const int kbase = (p_begin + w + NW * k) * BS;
      const bool full = kbase + BS <= ctx && kbase >= key_lo;
      f32x4 sacc[4];
#pragma unroll
      for (int ti = 0; ti < 4; ++ti) {
        sacc[ti] = (f32x4)(0.f);
#pragma unroll
        for (int s = 0; s < DS; ++s) sacc[ti] = mfma16(as_bf16x8(kf[ti][s]), qf[s], sacc[ti]);
      }
      float mloc = -INFINITY;
      if (full) {
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, sacc[ti][r]);
      } else {
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kbase + 32 * (ti >> 1) + 8 * h + 4 * (ti & 1) + r;
            const float sv = (key < ctx && key >= key_lo) ? sacc[ti][r] : -INFINITY;
            sacc[ti][r] = sv;
            mloc = fmaxf(mloc, sv);
          }
      }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      mloc *= sl2;
      if (mloc > m + RESCALE_LOG2) {
        const float alpha = __builtin_amdgcn_exp2f(m - mloc);
        m = mloc;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      }
      const float mo = m == -INFINITY ? 0.f : -m;
      bf16x8 pf[2];
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(sacc[2 * g + (j >> 2)][j & 3], sl2, mo));
          l += pv;
          pf[g][j] = (__bf16)pv;
        }
      // V(k) landed: K(k+1), if issued, is the only younger DMA
      if (more) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u16x8 vf[2][DT];
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int row = 16 * dt + col;
          vf[g][dt] = *reinterpret_cast<const u16x8*>(vs + row * BS + (((4 * g + h) ^ dvswz(row)) << 3));
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // V buffer free
      if (more) issue_v(blk_of(k + 1));
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] = mfma16(as_bf16x8(vf[g][dt]), pf[g], o[dt]);
    }
  } else {
  int p = p_begin + w;
  if (p < p_end) issue(sbt[p - p_begin]);
  // Q after the first DMA: its wait is the first page's anyway
  bf16x8 qf[DS];
  {
    const bool qv = col < G;
    const uint16_t* qp = q + (int64_t)b * q_stride + (int64_t)(kvh * G + (qv ? col : 0)) * D;
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      u16x8 v = load8(qp + 32 * s + 8 * h);
      if (!qv) v = (u16x8)(0);
      qf[s] = as_bf16x8(v);
    }
  }
  for (; p < p_end; p += NW) {
    const int pn = p + NW;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u16x8 kf[4][DS], vf[2][DT];
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
      const int key = 32 * (ti >> 1) + 8 * (col >> 2) + 4 * (ti & 1) + (col & 3);
#pragma unroll
      for (int s = 0; s < DS; ++s)
        kf[ti][s] = *reinterpret_cast<const u16x8*>(ks + key * D + (((4 * s + h) ^ dkswz(key)) << 3));
    }
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int row = 16 * dt + col;
        vf[g][dt] = *reinterpret_cast<const u16x8*>(vs + row * BS + (((4 * g + h) ^ dvswz(row)) << 3));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot is free: next page's DMA
    if (pn < p_end) issue(sbt[pn - p_begin]);

    const int kbase = p * BS;
    const bool full = kbase + BS <= ctx && kbase >= key_lo;
    f32x4 sacc[4];
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
      sacc[ti] = (f32x4)(0.f);
#pragma unroll
      for (int s = 0; s < DS; ++s) sacc[ti] = mfma16(as_bf16x8(kf[ti][s]), qf[s], sacc[ti]);
    }
    float mloc = -INFINITY;
    if (full) {
#pragma unroll
      for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, sacc[ti][r]);
    } else {
#pragma unroll
      for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kbase + 32 * (ti >> 1) + 8 * h + 4 * (ti & 1) + r;
          const float sv = (key < ctx && key >= key_lo) ? sacc[ti][r] : -INFINITY;
          sacc[ti][r] = sv;
          mloc = fmaxf(mloc, sv);
        }
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    mloc *= sl2;
    if (mloc > m + RESCALE_LOG2) {   // lazy rescale, as decode_attn_kernel
      const float alpha = __builtin_amdgcn_exp2f(m - mloc);
      m = mloc;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    }
    const float mo = m == -INFINITY ? 0.f : -m;
    bf16x8 pf[2];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(sacc[2 * g + (j >> 2)][j & 3], sl2, mo));
        l += pv;
        pf[g][j] = (__bf16)pv;
      }
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = mfma16(as_bf16x8(vf[g][dt]), pf[g], o[dt]);
  }
  }   // RING
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);

  // wave partials -> LDS (the page slots are free: every wave waited for its last DMA)
  __syncthreads();
  float* o_s = reinterpret_cast<float*>(smem);              // [NW][16][D + 4]
  float* m_s = o_s + NW * 16 * (D + 4);                     // [NW][16]
  float* l_s = m_s + NW * 16;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) o_s[(w * 16 + col) * (D + 4) + 16 * dt + 4 * h + r] = o[dt][r];
  if (h == 0) {
    m_s[w * 16 + col] = m;
    l_s[w * 16 + col] = l;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int qi = i / D, d = i % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, m_s[ww * 16 + qi]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float mw = m_s[ww * 16 + qi];
      const float f = mw == -INFINITY ? 0.f : exp2f(mw - M);
      L += f * l_s[ww * 16 + qi];
      acc += f * o_s[(ww * 16 + qi) * (D + 4) + d];
    }
    const int hq = kvh * G + qi;
    if (nparts == 1) {
      out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
    } else {
      const int64_t idx = ((int64_t)b * Hq + hq) * nparts + part;
      part_o[idx * D + d] = acc;
      if (d == 0) {
        part_ml[2 * idx] = M;
        part_ml[2 * idx + 1] = L;
      }
    }
  }
}

// Combine of the split-K partitions, one workgroup per (sequence, query head), one thread per
// output dimension. Wave 0 turns the partitions' (m, l) into normalised weights in LDS (all
// (m, l) loads in flight at once); then every thread sums its d over the partitions with the
// O loads issued 8 at a time. (The first version walked the partitions with one dependent
// load chain per thread: ~6 us per call at 16 x 1,400, profiles/r3_pmc/decode_fetch.txt.)
constexpr int REDUCE_MAX_PARTS = 256;
template <int D>
__global__ void __launch_bounds__(D) decode_attn_reduce_kernel(
    uint16_t* __restrict__ out, int64_t out_stride, const float* __restrict__ part_ml,
    const float* __restrict__ part_o, int Hq, int nparts, const int32_t* __restrict__ ctx_lens,
    int skip_empty) {
  __shared__ float w_s[REDUCE_MAX_PARTS];
  __shared__ float inv_s;
  const int b = blockIdx.x, hq = blockIdx.y;
  if (skip_empty && ctx_lens[b] == 0) return;
  const int64_t base = ((int64_t)b * Hq + hq) * nparts;
  if (threadIdx.x < 64) {
    float M = -INFINITY;
    for (int p = threadIdx.x; p < nparts; p += 64) M = fmaxf(M, part_ml[2 * (base + p)]);
    M = wave_max(M);
    float L = 0.f;
    for (int p = threadIdx.x; p < nparts; p += 64) {
      const float mp = part_ml[2 * (base + p)];
      const float f = mp == -INFINITY ? 0.f : exp2f(mp - M);   // empty partition: weight 0
      L += f * part_ml[2 * (base + p) + 1];
      w_s[p] = f;
    }
    L = wave_sum(L);
    if (threadIdx.x == 0) inv_s = L > 0.f ? 1.f / L : 0.f;
  }
  __syncthreads();
  const int d = threadIdx.x;
  const float* po = part_o + base * D + d;
  float acc = 0.f;
  int p = 0;
  // unconditional loads (an empty partition's O slot holds stale bytes: the select, not the
  // multiply, drops it — 0 x NaN would not)
  for (; p + 8 <= nparts; p += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = po[(int64_t)(p + j) * D];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += w_s[p + j] != 0.f ? w_s[p + j] * v[j] : 0.f;
  }
  for (; p < nparts; ++p) {
    const float v = po[(int64_t)p * D];
    acc += w_s[p] != 0.f ? w_s[p] * v : 0.f;
  }
  out[(int64_t)b * out_stride + (int64_t)hq * D + d] = f2bf(acc * inv_s);
}

int decode_attn_pages_per_part(int num_seqs, int Hkv, int max_ctx) {
  // Aim for >= ~1024 workgroups (4 per CU) so the KV stream has enough loads in flight.
  const int pages = (max_ctx + BS - 1) / BS;
  const int items = num_seqs * Hkv;
  int want_parts = (1024 + items - 1) / items;
  if (want_parts < 1) want_parts = 1;
  int ppp = (pages + want_parts - 1) / want_parts;
  if (ppp < NW) ppp = NW;  // at least one page per wave
  return ppp;
}

void launch_decode_attention(uint16_t* out, int64_t out_stride, const uint16_t* q,
                             int64_t q_stride, const void* kc, const void* vc,
                             const int32_t* block_tables, int max_blocks, const int32_t* ctx_lens,
                             int num_seqs, int Hq, int Hkv, int D, int max_ctx, float scale,
                             int pages_per_part, float* part_ml, float* part_o, int window,
                             bool kv_fp8, float k_scale, float v_scale, hipStream_t stream,
                             bool skip_empty) {
  if (num_seqs == 0) return;
  int pages = (max_ctx + BS - 1) / BS;
  if (window > 0) pages = min(pages, (window + BS - 1) / BS + 1);  // visible pages at most
  const int nparts = (pages + pages_per_part - 1) / pages_per_part;
  dim3 grid(num_seqs, Hkv, nparts);
  dim3 g2(num_seqs, Hq);
  if (!kv_fp8) k_scale = v_scale = 1.f;
  // form decode_nt: nt KV loads (each page is streamed once per step) — 1 always, 2 (default)
  // bf16 pages only: a bf16 decode step on this kernel runs 0.6-1.2 % faster with them, the
  // fp8-KV headline 0.5-0.9 % slower (profiles/r5_decode_nt/)
  const int ntf = kernel_form(KF_DECODE_NT);
  const int nt = ntf == 1 || (ntf == 2 && !kv_fp8) ? 1 : 0;
  const float sc = scale * k_scale;
#define NGA_DEC(DD, CT)                                                                        \
  decode_attn_kernel<DD, CT><<<grid, 256, 0, stream>>>(                                        \
      out, out_stride, q, q_stride, static_cast<const CT*>(kc), static_cast<const CT*>(vc),   \
      block_tables, max_blocks, ctx_lens, Hq, Hkv, sc, pages_per_part, part_ml, part_o, window, \
      v_scale, skip_empty ? 1 : 0, nt)
  if (D == 256) {
    if (kv_fp8) NGA_DEC(256, uint8_t); else NGA_DEC(256, uint16_t);
    if (nparts > 1)
      decode_attn_reduce_kernel<256><<<g2, 256, 0, stream>>>(out, out_stride, part_ml, part_o, Hq, nparts,
                                                             ctx_lens, skip_empty ? 1 : 0);
  } else {
    // bf16 pages run the LDS-DMA kernel at every batch size. It holds one workgroup per CU,
    // so DecodeWorkspace sizes its split for ~256 busy workgroups (one per CU) rather than the
    // register kernel's ~2,048 (graph replay, profiles/r3_search_dma/kb_decode_small_sweep.json):
    // 16 x 1,400 22.1 -> 18.6 us (2 partitions), 64 x 1,400 81.5 -> 59.6 us (1 partition),
    // 4 x 1,400 9.6 -> 8.1 us, the 70B TP=8 rank's 32 x 1,400 9.9 -> 8.8 us; 256 x 1,400
    // 257 -> 224 us (profiles/r3_dma). Form KF_DECODE_DMA (NGA_DECODE_DMA): 0 forces the register
    // kernel, 1 the whole-page DMA form, 2 (default) its K / V^T refill ring (profiles/r5_dma_ring/).
    const int dma = kernel_form(KF_DECODE_DMA);
    if (kv_fp8) NGA_DEC(128, uint8_t);
    else if (dma && (pages + nparts - 1) / nparts <= DMA_MAX_PAGES) {
#define NGA_DMA(RING, AUX)                                                                                   \
  decode_attn_dma_kernel<RING, AUX><<<grid, 256, 0, stream>>>(                                              \
      out, out_stride, q, q_stride, static_cast<const uint16_t*>(kc), static_cast<const uint16_t*>(vc), \
      block_tables, max_blocks, ctx_lens, Hq, Hkv, sc, part_ml, part_o, window, skip_empty ? 1 : 0)
      const bool cached = kernel_form(KF_DECODE_DMA_AUX) == 0;
      if (dma == 2) {
        if (cached) NGA_DMA(true, 0); else NGA_DMA(true, 2);
      } else {
        if (cached) NGA_DMA(false, 0); else NGA_DMA(false, 2);
      }
#undef NGA_DMA
    } else NGA_DEC(128, uint16_t);
    if (nparts > 1)
      decode_attn_reduce_kernel<128><<<g2, 128, 0, stream>>>(out, out_stride, part_ml, part_o, Hq, nparts,
                                                             ctx_lens, skip_empty ? 1 : 0);
  }
#undef NGA_DEC
}

}  // namespace nga
