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
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr float LOG2E_P = 1.4426950408889634f;

__device__ __forceinline__ int row_swz(int row) {  // 4-bit key: distinct over a tile's 16 rows
  return (row & 3) | (((row >> 3) & 3) << 2);
}
}  // namespace

template <int D, bool PAGED, bool CAUSAL>
__global__ void __launch_bounds__(256) prefill_attn_kernel(PrefillParams P) {
  constexpr int KT = 64;          // keys per tile (= KV page size when PAGED)
  constexpr int NCH_K = D / 8;    // 16-B chunks per K row
  constexpr int DS = D / 32;      // d-steps of the QK^T MFMA
  constexpr int DT = D / 16;      // d-tiles of the PV MFMA
  constexpr int K_CHUNKS = KT * NCH_K;   // = V chunks too
  constexpr int PER_T = K_CHUNKS / 256;  // chunks per thread per operand

  __shared__ __attribute__((aligned(16))) uint16_t k_s[KT * D];
  __shared__ __attribute__((aligned(16))) uint16_t v_s[D * KT];

  const int b = blockIdx.z, hq = blockIdx.y, tile = blockIdx.x;
  const int q0 = P.cu_q[b], qlen = P.cu_q[b + 1] - q0;
  if (tile * 64 >= qlen) return;
  const int ctx = PAGED ? P.ctx_lens[b] : qlen;
  const int G = P.Hq / P.Hkv;
  const int kvh = hq / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int tid = threadIdx.x;

  // this lane's query row (column of the MFMA tile)
  int qr = tile * 64 + w * 16 + col;
  const bool row_ok = qr < qlen;
  if (!row_ok) qr = qlen - 1;
  const int qpos = ctx - qlen + qr;  // absolute key index of this query

  bf16x8 qf[DS];
  {
    const uint16_t* qp = P.q + (int64_t)(q0 + qr) * P.q_stride + (int64_t)hq * D;
#pragma unroll
    for (int s = 0; s < DS; ++s) qf[s] = as_bf16x8(load8(qp + 32 * s + 8 * h));
  }

  int last_key = ctx - 1;
  if (CAUSAL) {
    const int qmax = min(qlen - 1, tile * 64 + 63);
    last_key = min(last_key, ctx - qlen + qmax);
  }
  const int n_tiles = last_key / KT + 1;

  // staging registers (one tile ahead)
  u16x8 kreg[PER_T], vreg[PER_T];
  auto load_tile = [&](int t) {
    if (PAGED) {
      const int64_t blk = P.block_tables[(int64_t)b * P.max_blocks + t];
      const uint16_t* kp = P.kc + (blk * P.Hkv + kvh) * (int64_t)(KT * D);
      const uint16_t* vp = P.vc + (blk * P.Hkv + kvh) * (int64_t)(D * KT);
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int c = tid + 256 * i;
        kreg[i] = load8(kp + (int64_t)c * 8);
        vreg[i] = load8(vp + (int64_t)c * 8);
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
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = tid + 256 * i;
      {  // K: row = key, chunk = d/8
        const int row = c / NCH_K, ch = c % NCH_K;
        const int sw = (NCH_K == 16) ? row_swz(row) : (row_swz(row) >> 1);
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
  float m = -INFINITY, l = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4)(0.f);

  load_tile(0);
  for (int t = 0; t < n_tiles; ++t) {
    __syncthreads();  // previous tile's LDS reads are done
    store_tile();
    __syncthreads();
    if (t + 1 < n_tiles) load_tile(t + 1);

    f32x4 sacc[4];
#pragma unroll
    for (int tau = 0; tau < 4; ++tau) {
      const int row = 32 * (tau >> 1) + 8 * (col >> 2) + 4 * (tau & 1) + (col & 3);
      const int sw = (NCH_K == 16) ? row_swz(row) : (row_swz(row) >> 1);
      sacc[tau] = (f32x4)(0.f);
#pragma unroll
      for (int s = 0; s < DS; ++s) {
        const int ch = 4 * s + h;
        bf16x8 a = as_bf16x8(*reinterpret_cast<const u16x8*>(&k_s[row * D + ((ch ^ sw) * 8)]));
        sacc[tau] = mfma16(a, qf[s], sacc[tau]);
      }
    }
    const int kbase = t * KT;
    float mloc = -INFINITY;
#pragma unroll
    for (int tau = 0; tau < 4; ++tau)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kbase + 32 * (tau >> 1) + 8 * h + 4 * (tau & 1) + r;
        float s = sacc[tau][r] * sl2;
        const bool ok = CAUSAL ? (key <= qpos) : (key < ctx);
        s = ok ? s : -INFINITY;
        sacc[tau][r] = s;
        mloc = fmaxf(mloc, s);
      }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m, mloc);  // finite: tile 0 always holds key 0 <= qpos
    const float alpha = exp2f(m - m_new);
    m = m_new;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    bf16x8 pf[2];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = exp2f(sacc[2 * g + (j >> 2)][j & 3] - m_new);
        l += pv;
        pf[g][j] = (__bf16)pv;
      }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int ch = 4 * g + h;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int row = 16 * dt + col;
        bf16x8 a = as_bf16x8(
            *reinterpret_cast<const u16x8*>(&v_s[row * KT + ((ch ^ ((row >> 1) & 7)) * 8)]));
        o[dt] = mfma16(a, pf[g], o[dt]);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (row_ok) {
    const float inv = 1.f / l;
    uint16_t* op = P.out + (int64_t)(q0 + qr) * P.out_stride + (int64_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = f2bf(o[dt][r] * inv);
      *reinterpret_cast<u16x4*>(op + 16 * dt + 4 * h) = v;
    }
  }
}

void launch_prefill_attention(const PrefillParams& p, int num_seqs, int max_q_len, int D,
                              bool paged, bool causal, hipStream_t stream) {
  if (num_seqs == 0 || max_q_len == 0) return;
  dim3 grid((max_q_len + 63) / 64, p.Hq, num_seqs);
#define NGA_PF(DD, PG, CS) prefill_attn_kernel<DD, PG, CS><<<grid, 256, 0, stream>>>(p)
  if (D == 128) {
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
  }
#undef NGA_PF
}

}  // namespace nga
