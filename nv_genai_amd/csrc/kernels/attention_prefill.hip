// Flash-style prefill / encoder attention on MFMA (K1 causal-GQA over the paged KV cache,
// K10 bidirectional encoder attention over packed variable-length sequences).
//
// Workgroup = 4 waves = a 64-row query tile of one query head; each wave owns 16 query
// rows, which are the 16 columns of its mfma_f32_16x16x32_bf16 tiles. Per 64-key tile the
// workgroup stages K [64][D] and V^T [D][64] in LDS (XOR-swizzled 16-B chunks so the
// ds_read_b128 operand reads are bank-conflict-free), then every wave computes
//   S^T = K . Q^T (key rows on the MFMA A side, Q^T kept in registers as the B operand),
//   an online softmax per query column (exp2 domain, keys of a column in 4 lanes x 16 regs),
//   O^T += V^T . P^T (the S accumulator is the P^T B operand with no lane movement — same
//   key<->row mapping as attention_decode.hip).
// The next tile's K/V are loaded into registers before the current tile's MFMAs and written
// to LDS after the barrier (issue-early / write-late, guide §5.5 T14).
//
// PAGED: K from the [blocks, Hkv, 64, D] cache, V^T from the [blocks, Hkv, D, 64] cache,
//        queries are the last q_len positions of a ctx_len context (chunked prefill and
//        prefix-cache hits work unchanged).  Otherwise: K and V rows come from packed
//        [T, H, D] tensors with per-sequence offsets (cu_q), V is transposed while staging.
// D is 64 or 128 (either mode), 256 (paged: Gemma) or 32 (packed mode only: the
// all-MiniLM-L6-v2 encoder). Paged caches may be fp8 e4m3fn (P.kv_fp8): widened to bf16 in
// registers before staging; P.scale carries the K scale, P.v_scale the V scale. P.window > 0: sliding-window causal attention (query i sees keys
// (i - window, i]); key tiles wholly before every query's window are skipped.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr float LOG2E_P = 1.4426950408889634f;
constexpr float RESCALE_LOG2 = 8.f;

__device__ __forceinline__ int row_swz(int row) {  // 4-bit key: distinct over a tile's 16 rows
  return (row & 3) | (((row >> 3) & 3) << 2);
}
}  // namespace

template <int D, bool PAGED, bool CAUSAL, int NCG>
__device__ __forceinline__ void v1_tile(const PrefillParams& P, uint16_t* k_s, uint16_t* v_s, int b, int hq,
                                        int tile) {
  // NCG query column-groups (16 rows each) per wave: the K and V^T fragments read from LDS
  // for one key tile feed NCG MFMAs each, and the tile's staging + barriers are amortised
  // over a 64*NCG-row query tile.
  constexpr int KT = 64;          // keys per tile (= KV page size when PAGED)
  constexpr int NCH_K = D / 8;    // 16-B chunks per K row
  constexpr int DS = D / 32;      // d-steps of the QK^T MFMA
  constexpr int DT = D / 16;      // d-tiles of the PV MFMA
  constexpr int K_CHUNKS = KT * NCH_K;   // = V chunks too
  constexpr int PER_T = K_CHUNKS / 256;  // chunks per thread per operand
  constexpr int QT = 64 * NCG;           // query rows per workgroup

  // K-row swizzle: XOR the 16-B chunk index with up to 4 bits of the row (fewer for short
  // rows: the XOR value must stay below the chunk count)
  constexpr int SWS = NCH_K >= 16 ? 0 : NCH_K == 8 ? 1 : 2;
  const int q0 = P.cu_q[b], qlen = P.cu_q[b + 1] - q0;
  if (tile * QT >= qlen) return;
  const int ctx = PAGED ? P.ctx_lens[b] : qlen;
  const int G = P.Hq / P.Hkv;
  const int kvh = hq / G;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int col = lane & 15, h = lane >> 4;
  const int tid = threadIdx.x;

  // this lane's query rows (one per column group)
  int qr[NCG], qpos[NCG];
  bool row_ok[NCG];
  bf16x8 qf[NCG][DS];
#pragma unroll
  for (int cg = 0; cg < NCG; ++cg) {
    int r = tile * QT + w * 16 * NCG + cg * 16 + col;
    row_ok[cg] = r < qlen;
    if (!row_ok[cg]) r = qlen - 1;
    qr[cg] = r;
    qpos[cg] = ctx - qlen + r;  // absolute key index of this query
    const uint16_t* qp = P.q + (int64_t)(q0 + r) * P.q_stride + (int64_t)hq * D;
#pragma unroll
    for (int s2 = 0; s2 < DS; ++s2) qf[cg][s2] = as_bf16x8(load8(qp + 32 * s2 + 8 * h));
  }

  const int qpos_w0 = ctx - qlen + tile * QT + w * 16 * NCG;  // smallest query position of this wave
  const int qpos_w1 = qpos_w0 + 16 * NCG - 1;                  // largest (may exceed ctx: masked rows)
  const int W = CAUSAL ? P.window : 0;
  int last_key = ctx - 1;
  if (CAUSAL) {
    const int qmax = min(qlen - 1, tile * QT + QT - 1);
    last_key = min(last_key, ctx - qlen + qmax);
  }
  const int n_tiles = last_key / KT + 1;
  // sliding window: the workgroup's oldest visible key belongs to its first query row
  const int t_first = W > 0 ? max(0, ctx - qlen + tile * QT - W + 1) / KT : 0;

  // staging registers, one tile ahead (a second set, two tiles ahead, measured no faster
  // and costs 32 VGPRs that the accumulators need)
  u16x8 kA[PER_T], vA[PER_T];
  auto load_tile = [&](int t, u16x8 (&kreg)[PER_T], u16x8 (&vreg)[PER_T]) {
    if (PAGED) {
      const int64_t blk = P.block_tables[(int64_t)b * P.max_blocks + t];
      const int64_t pg = (blk * P.Hkv + kvh) * (int64_t)(KT * D);   // elements (= bytes for fp8)
      if (P.kv_fp8) {   // 8-byte fp8 chunks widened to bf16 before they are staged
        const uint8_t* kp = reinterpret_cast<const uint8_t*>(P.kc) + pg;
        const uint8_t* vp = reinterpret_cast<const uint8_t*>(P.vc) + pg;
#pragma unroll
        for (int i = 0; i < PER_T; ++i) {
          const int c = tid + 256 * i;
          kreg[i] = load8_fp8(kp + (int64_t)c * 8);
          vreg[i] = load8_fp8(vp + (int64_t)c * 8);
        }
      } else {
        const uint16_t* kp = P.kc + pg;
        const uint16_t* vp = P.vc + pg;
#pragma unroll
        for (int i = 0; i < PER_T; ++i) {
          const int c = tid + 256 * i;
          kreg[i] = load8(kp + (int64_t)c * 8);
          vreg[i] = load8(vp + (int64_t)c * 8);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int c = tid + 256 * i;
        const int key = t * KT + c / NCH_K, ch = c % NCH_K;
        if (key < ctx) {
          const int64_t off = (int64_t)(q0 + key) * P.kv_stride + (int64_t)kvh * D + ch * 8;
          kreg[i] = load8(P.k + off);
          vreg[i] = load8(P.v + off);
        } else {
          kreg[i] = (u16x8)(0);
          vreg[i] = (u16x8)(0);
        }
      }
    }
  };
  auto store_tile = [&](const u16x8 (&kreg)[PER_T], const u16x8 (&vreg)[PER_T]) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = tid + 256 * i;
      {  // K: row = key, chunk = d/8
        const int row = c / NCH_K, ch = c % NCH_K;
        const int sw = row_swz(row) >> SWS;
        *reinterpret_cast<u16x8*>(&k_s[row * D + ((ch ^ sw) * 8)]) = kreg[i];
      }
      if (PAGED) {  // Vt page is already [d][key]: row = d, chunk = key/8
        const int row = c / 8, ch = c % 8;
        *reinterpret_cast<u16x8*>(&v_s[row * KT + ((ch ^ ((row >> 1) & 7)) * 8)]) = vreg[i];
      } else {  // transpose: vreg holds V[key][d0..d0+7]
        const int key = c / NCH_K, d0 = (c % NCH_K) * 8;
        const int ch = key / 8, kin = key % 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = d0 + j;
          v_s[row * KT + ((ch ^ ((row >> 1) & 7)) * 8) + kin] = vreg[i][j];
        }
      }
    }
  };

  const float sl2 = P.scale * LOG2E_P;
  float m[NCG], l[NCG];
  f32x4 o[NCG][DT];
#pragma unroll
  for (int cg = 0; cg < NCG; ++cg) {
    m[cg] = -INFINITY;
    l[cg] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[cg][dt] = (f32x4)(0.f);
  }

  // (Tried: separate masked/unmasked instantiations of this body behind a wave-uniform
  // branch to drop the ~60 if-converted mask selects per tile. 39.3 -> 34.5 us at 1 x 1,196
  // but 658 -> 672 us at 27 x 1,200: the two bodies need 252 VGPRs, 3 -> 2 waves/SIMD, and
  // forcing 3 waves spills.)
  auto compute_tile = [&](int t) {
      f32x4 sacc[NCG][4];
#pragma unroll
      for (int tau = 0; tau < 4; ++tau) {
        const int row = 32 * (tau >> 1) + 8 * (col >> 2) + 4 * (tau & 1) + (col & 3);
        const int sw = row_swz(row) >> SWS;
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) sacc[cg][tau] = (f32x4)(0.f);
#pragma unroll
        for (int s2 = 0; s2 < DS; ++s2) {
          const int ch = 4 * s2 + h;
          bf16x8 a = as_bf16x8(*reinterpret_cast<const u16x8*>(&k_s[row * D + ((ch ^ sw) * 8)]));
#pragma unroll
          for (int cg = 0; cg < NCG; ++cg) sacc[cg][tau] = mfma16(a, qf[cg][s2], sacc[cg][tau]);
        }
      }
      const int kbase = t * KT;
      // masking is only needed on tiles that cross this wave's causal diagonal (or the end
      // of the context); the test is wave-uniform
      const bool need_mask = CAUSAL ? (kbase + KT - 1 > qpos_w0 || (W > 0 && kbase <= qpos_w1 - W))
                                    : (kbase + KT > ctx);
      bf16x8 pf[NCG][2];
#pragma unroll
      for (int cg = 0; cg < NCG; ++cg) {
        float mloc = -INFINITY;
#pragma unroll
        for (int tau = 0; tau < 4; ++tau)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float sv = sacc[cg][tau][r];  // raw score; the scale is folded into the exp
            if (need_mask) {
              const int key = kbase + 32 * (tau >> 1) + 8 * h + 4 * (tau & 1) + r;
              const bool ok = CAUSAL ? (key <= qpos[cg] && (W == 0 || key > qpos[cg] - W)) : (key < ctx);
              sv = ok ? sv : -INFINITY;
            }
            sacc[cg][tau][r] = sv;
            mloc = fmaxf(mloc, sv);
          }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        mloc *= sl2;  // scale > 0: max commutes with it
        // Lazy rescaling: the running max only moves (and O / l are only rescaled) when a
        // row's tile max exceeds it by more than 2^RESCALE_LOG2; until then P = 2^(s - m)
        // stays <= 2^8, harmless in fp32 accumulators and bf16 P. Keeps O in the MFMA
        // accumulators instead of a VALU round trip every tile. m starts at -inf, so the
        // first tile always rescales (alpha = 2^-inf = 0 on an all-zero O).
        const bool grow = mloc > m[cg] + RESCALE_LOG2;
        if (__ballot(grow)) {
          const float m_new = grow ? mloc : m[cg];
          // non-growing lanes keep their scale (and a still -inf m must not meet -inf - -inf)
          const float alpha = grow ? __builtin_amdgcn_exp2f(m[cg] - m_new) : 1.f;
          m[cg] = m_new;
          l[cg] *= alpha;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[cg][dt] *= alpha;
        }
        // exponent argument and row-sum in packed fp32 (v_pk_fma_f32 / v_pk_add_f32: two
        // scores per VALU op, two independent add chains instead of one 16-long chain).
        // Loop VALU 141 -> 128 instructions per tile at the same 148 VGPRs; kernel time within
        // run-to-run noise (633 us at 27 x 1,200, profiles/r1_prefill_valu).
        // a tile can be fully masked for a row (sliding window): m may still be -inf then,
        // and the offset must not become +inf (2^(-inf + inf) = NaN)
        const float mo = m[cg] == -INFINITY ? 0.f : -m[cg];
        const f32x2 sl2v = {sl2, sl2}, nmc = {mo, mo};
        f32x2 lsum = {0.f, 0.f};
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const f32x4& sv = sacc[cg][2 * g + (j >> 2)];
            f32x2 e = __builtin_elementwise_fma((f32x2){sv[j & 3], sv[(j & 3) + 1]}, sl2v, nmc);
            e[0] = __builtin_amdgcn_exp2f(e[0]);  // 2^-inf = 0
            e[1] = __builtin_amdgcn_exp2f(e[1]);
            lsum += e;
            pf[cg][g][j] = (__bf16)e[0];
            pf[cg][g][j + 1] = (__bf16)e[1];
          }
        l[cg] += lsum[0] + lsum[1];
      }
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int ch = 4 * g + h;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int row = 16 * dt + col;
          bf16x8 a = as_bf16x8(
              *reinterpret_cast<const u16x8*>(&v_s[row * KT + ((ch ^ ((row >> 1) & 7)) * 8)]));
#pragma unroll
          for (int cg = 0; cg < NCG; ++cg) o[cg][dt] = mfma16(a, pf[cg][g], o[cg][dt]);
        }
      }
  };

  load_tile(t_first, kA, vA);
  for (int t = t_first; t < n_tiles; ++t) {
    __syncthreads();  // previous tile's LDS reads are done
    store_tile(kA, vA);
    __syncthreads();
    if (t + 1 < n_tiles) load_tile(t + 1, kA, vA);
    compute_tile(t);
  }
#pragma unroll
  for (int cg = 0; cg < NCG; ++cg) {
    float ll = l[cg];
    ll += __shfl_xor(ll, 16, 64);
    ll += __shfl_xor(ll, 32, 64);
    if (row_ok[cg]) {
      const float inv = (ll > 0.f ? 1.f / ll : 0.f) * (PAGED && P.kv_fp8 ? P.v_scale : 1.f);
      uint16_t* op = P.out + (int64_t)(q0 + qr[cg]) * P.out_stride + (int64_t)hq * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(o[cg][dt][r] * inv);
        *reinterpret_cast<u16x4*>(op + 16 * dt + 4 * h) = v;
      }
    }
  }
}

// Grid modes (as attention_prefill_v2.hip): enumerated — workgroups dealt round-robin over
// the 8 XCDs, physical block p runs on XCD p % 8 and logical item L = (p % 8) * per_xcd + p / 8
// gives every XCD one contiguous range of the (sequence, kv head, q head, tile) order (the G
// query heads sharing a KV head read its pages through the same L2; longest causal tiles
// first) — or a host-planned work list of (sequence, 64-row tile) pairs walked by a fixed
// grid with q head it % Hq (graph-captured steps with fp8 KV pages or head_dim != 128).
template <int D, bool PAGED, bool CAUSAL, int NCG>
__global__ void __launch_bounds__(256) prefill_attn_kernel(PrefillParams P) {
  constexpr int KT = 64;
  __shared__ __attribute__((aligned(16))) uint16_t k_s[KT * D];
  __shared__ __attribute__((aligned(16))) uint16_t v_s[D * KT];
  if (P.items) {
    const int total = *P.n_items * P.Hq;
    for (int it = blockIdx.x; it < total; it += gridDim.x) {
      __syncthreads();
      const int k = it / P.Hq;
      v1_tile<D, PAGED, CAUSAL, NCG>(P, k_s, v_s, P.items[2 * k], it % P.Hq, P.items[2 * k + 1]);
    }
    return;
  }
  const int pblk = blockIdx.x;
  const int L = (pblk & 7) * P.per_xcd + (pblk >> 3);
  if (L >= P.total) return;
  const int tile = P.ntiles - 1 - L % P.ntiles;
  const int hq = (L / P.ntiles) % P.Hq;
  const int b = L / (P.ntiles * P.Hq);
  v1_tile<D, PAGED, CAUSAL, NCG>(P, k_s, v_s, b, hq, tile);
}

void launch_prefill_attention_v1_worklist(const PrefillParams& p, int grid, int D, bool causal,
                                          hipStream_t stream) {
  dim3 g(grid);
  if (D == 256) {
    if (causal) prefill_attn_kernel<256, true, true, 1><<<g, 256, 0, stream>>>(p);
    else prefill_attn_kernel<256, true, false, 1><<<g, 256, 0, stream>>>(p);
  } else if (D == 128) {
    if (causal) prefill_attn_kernel<128, true, true, 1><<<g, 256, 0, stream>>>(p);
    else prefill_attn_kernel<128, true, false, 1><<<g, 256, 0, stream>>>(p);
  } else {
    if (causal) prefill_attn_kernel<64, true, true, 1><<<g, 256, 0, stream>>>(p);
    else prefill_attn_kernel<64, true, false, 1><<<g, 256, 0, stream>>>(p);
  }
}

void launch_prefill_attention(const PrefillParams& p, int num_seqs, int max_q_len, int D,
                              bool paged, bool causal, hipStream_t stream) {
  if (num_seqs == 0 || max_q_len == 0) return;
  // large paged head_dim-128 prefills run the 32x32-MFMA kernel (attention_prefill_v2.hip)
  if (launch_prefill_attention_v2(p, num_seqs, max_q_len, D, paged, causal, stream)) return;
  // 64-row query tiles (a 128-row variant with two column groups per wave halved the LDS
  // fragment traffic per MFMA but needed ~300 VGPR+AGPR — one wave per SIMD — and measured
  // 1.4-1.5x slower on MI355X; removed)
  const int ncg = 1;
  PrefillParams pp = p;
  pp.ntiles = (max_q_len + 64 * ncg - 1) / (64 * ncg);
  const int64_t total = (int64_t)pp.ntiles * p.Hq * num_seqs;
  pp.total = (int)total;
  pp.per_xcd = (int)((total + 7) / 8);
  // 1-D grid of 8 * per_xcd workgroups (see the XCD mapping in the kernel)
  dim3 grid(8 * pp.per_xcd);
#define NGA_PF(DD, PG, CS)                                                    \
  do {                                                                        \
    if (ncg == 2) prefill_attn_kernel<DD, PG, CS, 2><<<grid, 256, 0, stream>>>(pp); \
    else prefill_attn_kernel<DD, PG, CS, 1><<<grid, 256, 0, stream>>>(pp);          \
  } while (0)
  if (D == 256 && paged) {   // Gemma (head_dim 256): paged causal prefill
    if (causal) NGA_PF(256, true, true); else NGA_PF(256, true, false);
  } else if (D == 128) {
    if (paged) {
      if (causal) NGA_PF(128, true, true); else NGA_PF(128, true, false);
    } else {
      if (causal) NGA_PF(128, false, true); else NGA_PF(128, false, false);
    }
  } else if (D == 64) {
    if (paged) {
      if (causal) NGA_PF(64, true, true); else NGA_PF(64, true, false);
    } else {
      if (causal) NGA_PF(64, false, true); else NGA_PF(64, false, false);
    }
  } else if (D == 32 && !paged) {  // small encoders (MiniLM: 12 heads x 32); one MFMA d-step
    if (causal) NGA_PF(32, false, true); else NGA_PF(32, false, false);
  }
#undef NGA_PF
}

}  // namespace nga
