// Token embedding gather (K8 in SURVEY.md §2.C), vocab-parallel aware.
//
// out[t, :] = table[ids[t] - vocab_lo, :] * scale for ids in this rank's vocabulary shard
// [vocab_lo, vocab_lo + rows), zeros otherwise (the TP all-reduce then sums the one non-zero
// contribution). One wave per token row, 16-B loads and stores (8 bf16 per lane per step);
// the row index is loaded once per wave. `scale` != 1 (Gemma's sqrt(hidden)) is applied to
// the bf16 value in fp32 and rounded back to bf16, as a bf16 tensor multiply does.
#include "common.h"
#include "kernels.h"

namespace nga {

__global__ void __launch_bounds__(256) embedding_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ table,
                                                        const int32_t* __restrict__ ids, int T, int H,
                                                        int64_t vocab_lo, int64_t rows, float scale) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + w;
  if (t >= T) return;
  const int64_t r = (int64_t)ids[t] - vocab_lo;
  const bool ok = r >= 0 && r < rows;
  uint16_t* dst = out + (int64_t)t * H;
  const uint16_t* src = table + (ok ? r : 0) * (int64_t)H;
  for (int c = lane * 8; c < H; c += 64 * 8) {
    u16x8 v = (u16x8)(0);
    if (ok) {
      v = load8(src + c);
      if (scale != 1.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * scale);
      }
    }
    store8(dst + c, v);
  }
}

void launch_embedding(uint16_t* out, const uint16_t* table, const int32_t* ids, int T, int H, int64_t vocab_lo,
                      int64_t rows, float scale, hipStream_t stream) {
  if (T == 0) return;
  embedding_kernel<<<(T + 3) / 4, 256, 0, stream>>>(out, table, ids, T, H, vocab_lo, rows, scale);
}

}  // namespace nga
