// Token sampling over a full vocabulary row (up to 256K: Gemma) (K7 in SURVEY.md §2.C), one 1024-thread
// workgroup per sequence, no sort:
//   * repetition penalty (TRT-LLM semantics: divide positive / multiply negative logits of
//     every token seen in prompt+output) through an LDS bitmap of the row's history;
//   * temperature; greedy when temperature <= 0 or top_k == 1;
//   * top-k and top-p thresholds by a 3-level (11/11/10-bit) radix descent on order-preserving
//     float keys — top-k descends on counts, top-p on probability mass restricted to the
//     top-k set — so each costs 3 L2-resident passes over the row instead of a 128K sort;
//   * the draw itself is Gumbel-max over the kept tokens with a counter-based RNG keyed on
//     (seed, step, token): deterministic for a given seed, no global RNG state.
// Also returns the chosen token's log-probability under the temperature-scaled distribution.
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int NT = 1024;
constexpr int NBINS = 2048;

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Inclusive suffix scan (from the top bin) of NBINS values held 2 per thread; returns the
// bin where the running total first reaches `target`, and the total strictly above it.
template <typename T>
__device__ int find_crossing(T* bins, T target, T* above_out, T* scan) {
  const int t = threadIdx.x;
  // thread t owns bins (NBINS-1-2t) and (NBINS-2-2t): descending order
  const int b0 = NBINS - 1 - 2 * t, b1 = b0 - 1;
  T v0 = bins[b0], v1 = bins[b1];
  T mine = v0 + v1;
  scan[t] = mine;
  __syncthreads();
  for (int off = 1; off < NT; off <<= 1) {
    T add = t >= off ? scan[t - off] : (T)0;
    __syncthreads();
    scan[t] += add;
    __syncthreads();
  }
  const T incl = scan[t];
  const T excl = incl - mine;
  __shared__ int sel;
  __shared__ T sel_above;
  if (t == 0) {
    sel = -1;
    sel_above = (T)0;
  }
  __syncthreads();
  if (excl < target && incl >= target) {
    if (excl + v0 >= target) {
      sel = b0;
      sel_above = excl;
    } else {
      sel = b1;
      sel_above = excl + v0;
    }
  }
  __syncthreads();
  int s = sel;
  T a = sel_above;
  if (s < 0) {  // target beyond total (rounding): take the lowest populated bin
    s = 0;
    a = scan[NT - 1] - bins[0];
  }
  *above_out = a;
  __syncthreads();
  return s;
}

// Visit every element of a row: float4 loads for the body (rows of the [B, V] fp32 logits
// are 16-B aligned when V % 4 == 0), scalar loads for any tail. f(index, value).
template <typename F>
__device__ __forceinline__ void for_row(const float* __restrict__ x, int V, F f) {
  const int t = threadIdx.x;
  if ((V & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const int n4 = V >> 2;
    for (int j = t; j < n4; j += NT) {
      const float4 v = x4[j];
      f(4 * j, v.x);
      f(4 * j + 1, v.y);
      f(4 * j + 2, v.z);
      f(4 * j + 3, v.w);
    }
  } else {
    for (int i = t; i < V; i += NT) f(i, x[i]);
  }
}

struct ArgMax {
  float v;
  int i;
};

__device__ __forceinline__ ArgMax am_max(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

__device__ ArgMax block_argmax(ArgMax a, ArgMax* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b;
    b.v = __shfl_xor(a.v, o, 64);
    b.i = __shfl_xor(a.i, o, 64);
    a = am_max(a, b);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  ArgMax r = red[0];
  for (int k = 1; k < NT / 64; ++k) r = am_max(r, red[k]);
  return r;
}
}  // namespace

__global__ void __launch_bounds__(NT) sample_kernel(
    float* __restrict__ logits, int V, const float* __restrict__ temperature,
    const int32_t* __restrict__ top_k, const float* __restrict__ top_p,
    const float* __restrict__ rep_penalty, const int32_t* __restrict__ history, int hist_len,
    const int64_t* __restrict__ seeds, const int64_t* __restrict__ steps,
    int32_t* __restrict__ out_tok, float* __restrict__ out_logprob) {
  __shared__ uint32_t bitmap[8192];  // history bitmap, V <= 262144 (Gemma: 256000)
  __shared__ uint32_t hcnt[NBINS];
  __shared__ float hmass[NBINS];
  __shared__ uint32_t scan_u[NT];
  __shared__ float scan_f[NT];
  __shared__ float red[NT / 64];
  __shared__ ArgMax ared[NT / 64];

  const int row = blockIdx.x, t = threadIdx.x;
  float* x = logits + (int64_t)row * V;
  const float pen = rep_penalty ? rep_penalty[row] : 1.f;

  if (pen != 1.f && history != nullptr) {
    for (int i = t; i < 8192; i += NT) bitmap[i] = 0;
    __syncthreads();
    const int32_t* hs = history + (int64_t)row * hist_len;
    for (int i = t; i < hist_len; i += NT) {
      const int tok = hs[i];
      if (tok >= 0 && tok < V) atomicOr(&bitmap[tok >> 5], 1u << (tok & 31));
    }
    __syncthreads();
    for (int i = t; i < V; i += NT)
      if (bitmap[i >> 5] & (1u << (i & 31))) {
        const float v = x[i];
        x[i] = v > 0.f ? v / pen : v * pen;
      }
    __syncthreads();
  }

  const float temp = temperature[row];
  const int k = top_k ? top_k[row] : 0;
  const float p = top_p ? top_p[row] : 1.f;
  const bool greedy = !(temp > 0.f) || k == 1;
  const float inv_t = greedy ? 1.f : 1.f / temp;

  // one pass: argmax and the partition function (online: per-thread running max + rescaled sum)
  ArgMax am{-INFINITY, 0x7fffffff};
  float z = 0.f;
  for_row(x, V, [&](int i, float raw) {
    const float v = raw * inv_t;
    if (v > am.v) {
      z = z * __expf(am.v - v) + 1.f;
      am = ArgMax{v, i};
    } else if (v > -INFINITY) {
      z += __expf(v - am.v);
      if (v == am.v && i < am.i) am.i = i;
    }
  });
  const float m_thr = am.v;
  am = block_argmax(am, ared);
  const float M = am.v;
  const float Z = block_sum(m_thr == -INFINITY ? 0.f : z * __expf(m_thr - M), red);
  const float logZ = __logf(Z);

  if (greedy) {
    if (t == 0) {
      out_tok[row] = am.i;
      out_logprob[row] = 0.f - logZ;  // x[am] * inv_t - M == 0
    }
    return;
  }

  uint32_t thr = 0u;  // keep tokens with fkey(x * inv_t) >= thr
  float kept_mass = Z;
  if (k > 0 && k < V) {
    uint32_t prefix = 0, mask = 0;
    int remaining = k;
    const int shifts[3] = {21, 10, 0};
    const int widths[3] = {11, 11, 10};
    for (int lvl = 0; lvl < 3; ++lvl) {
      for (int i = t; i < NBINS; i += NT) hcnt[i] = 0;
      __syncthreads();
      const int sh = shifts[lvl];
      const uint32_t bm = (1u << widths[lvl]) - 1u;
      for_row(x, V, [&](int, float raw) {
        const uint32_t key = fkey(raw * inv_t);
        if ((key & mask) == prefix) atomicAdd(&hcnt[(key >> sh) & bm], 1u);
      });
      __syncthreads();
      uint32_t above;
      const int bin = find_crossing<uint32_t>(hcnt, (uint32_t)remaining, &above, scan_u);
      remaining -= (int)above;
      prefix |= ((uint32_t)bin) << sh;
      mask |= bm << sh;
    }
    thr = prefix;
    float km = 0.f;
    for_row(x, V, [&](int, float raw) {
      const float v = raw * inv_t;
      if (fkey(v) >= thr) km += __expf(v - M);
    });
    kept_mass = block_sum(km, red);
  }
  if (p < 1.f) {
    uint32_t prefix = 0, mask = 0;
    float remaining = p * kept_mass;
    const int shifts[3] = {21, 10, 0};
    const int widths[3] = {11, 11, 10};
    for (int lvl = 0; lvl < 3; ++lvl) {
      for (int i = t; i < NBINS; i += NT) hmass[i] = 0.f;
      __syncthreads();
      const int sh = shifts[lvl];
      const uint32_t bm = (1u << widths[lvl]) - 1u;
      for_row(x, V, [&](int, float raw) {
        const float v = raw * inv_t;
        const uint32_t key = fkey(v);
        if ((key & mask) == prefix && key >= thr) atomicAdd(&hmass[(key >> sh) & bm], __expf(v - M));
      });
      __syncthreads();
      float above;
      const int bin = find_crossing<float>(hmass, remaining, &above, scan_f);
      remaining -= above;
      prefix |= ((uint32_t)bin) << sh;
      mask |= bm << sh;
    }
    thr = prefix > thr ? prefix : thr;
  }

  // Gumbel-max draw over kept tokens
  const uint64_t seed = (uint64_t)seeds[row];
  const uint64_t base = (uint64_t)steps[row] * (uint64_t)V;
  ArgMax best{-INFINITY, 0x7fffffff};
  for_row(x, V, [&](int i, float raw) {
    const float v = raw * inv_t;
    if (fkey(v) >= thr) {
      const float u = hash_uniform(seed, base + i);
      const float g = -__logf(-__logf(u));
      best = am_max(best, ArgMax{v + g, i});
    }
  });
  best = block_argmax(best, ared);
  if (t == 0) {
    const int tok = best.i == 0x7fffffff ? am.i : best.i;
    out_tok[row] = tok;
    out_logprob[row] = x[tok] * inv_t - M - logZ;
  }
}

void launch_sample(float* logits, int B, int V, const float* temperature, const int32_t* top_k,
                   const float* top_p, const float* rep_penalty, const int32_t* history,
                   int hist_len, const int64_t* seeds, const int64_t* steps, int32_t* out_tok,
                   float* out_logprob, hipStream_t stream) {
  if (B == 0) return;
  sample_kernel<<<B, NT, 0, stream>>>(logits, V, temperature, top_k, top_p, rep_penalty, history,
                                      hist_len, seeds, steps, out_tok, out_logprob);
}

}  // namespace nga
