// Token sampling over a full vocabulary row (up to 256K: Gemma) (K7 in SURVEY.md §2.C), one 1024-thread
// workgroup per sequence, no full sort:
//   * repetition penalty (TRT-LLM semantics: divide positive / multiply negative logits of
//     every token seen in prompt+output) through an LDS bitmap of the row's history;
//   * temperature; greedy when temperature <= 0 or top_k == 1;
//   * top-k / top-p thresholds, fast path: one pass bins every token with v > M - 16 by its
//     distance to the row max (2048 linear bins, so the LDS atomics spread out instead of piling
//     onto a few exponent bins; the far tail takes no atomic), a scan finds the bin where the
//     running count / probability mass reaches the target, a second pass gathers that bin's keys
//     (at most 2048) into LDS, and a bitonic sort + scan there gives the exact threshold;
//   * exact fallback when the crossing lies in the far tail or its bin is too full (flat rows,
//     p close to 1): 3-level (11/11/10-bit) radix descent on order-preserving float keys;
//   * the draw itself is Gumbel-max over the kept tokens with a counter-based RNG keyed on
//     (seed, step, token): deterministic for a given seed, no global RNG state.
// Every pass over the row keeps eight 16-byte loads in flight per thread. Histogram weights are
// 64-bit fixed point (2^-40 units of exp(v - M)) so the LDS atomics are ds_add_u64: LDS
// ds_add_f32 measured ~8x slower on gfx950 (scripts/dev/lds_atomic_bench.hip).
// Also returns the chosen token's log-probability under the temperature-scaled distribution.
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int NT = 1024;
constexpr int NBINS = 2048;
constexpr int CAP = 2048;        // keys the fast path sorts in LDS
constexpr float DRANGE = 16.f;   // fast-path bins cover v in (M - DRANGE, M]
constexpr float DSCALE = NBINS / DRANGE;
constexpr int UNROLL = 8;

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float fval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

struct ArgMax {
  float v;
  int i;
};

constexpr double FIX = 1099511627776.0;  // 2^40: fixed-point unit of the mass histograms

struct Smem {
  union {
    uint32_t bitmap[8192];  // history bitmap (repetition penalty only), V <= 262144 (Gemma: 256000)
    struct {
      union {
        uint64_t q[NBINS];  // bin weights: counts or fixed-point mass
        float w[NBINS];     // candidate weights (fast path, after the bin scan)
      } h;
      uint32_t cand[CAP];
      union {
        uint64_t q[NT];
        float f[NT];
      } scan;
    } s;
  } u;
  float red[NT / 64];
  ArgMax ared[NT / 64];
  int ncand;
  int sel;
  float sel_above_f;
  uint64_t sel_above_q;
};

// Top-down crossing over nb <= 2*NT values (bins[nb-1] is the top): inclusive suffix scan,
// returns the bin where the running total first reaches `target` and the total strictly above
// it, or -1 (with the grand total in *above_out) when the total stays below target.
template <typename T>
__device__ __forceinline__ int find_crossing(const T* bins, int nb, T target, T* above_out, T* scan, Smem& sm) {
  const int t = threadIdx.x;
  // thread t owns bins (nb-1-2t) and (nb-2-2t): descending order
  const int b0 = nb - 1 - 2 * t, b1 = b0 - 1;
  const T v0 = b0 >= 0 ? bins[b0] : (T)0, v1 = b1 >= 0 ? bins[b1] : (T)0;
  const T mine = v0 + v1;
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
  if (t == 0) sm.sel = -1;
  __syncthreads();
  if (excl < target && incl >= target) {
    const bool first = excl + v0 >= target;
    sm.sel = first ? b0 : b1;
    const T a = first ? excl : excl + v0;
    if constexpr (sizeof(T) == 8)
      sm.sel_above_q = a;
    else
      sm.sel_above_f = a;
  }
  __syncthreads();
  const int s = sm.sel;
  T a;
  if constexpr (sizeof(T) == 8)
    a = sm.sel_above_q;
  else
    a = sm.sel_above_f;
  *above_out = s >= 0 ? a : scan[NT - 1];
  __syncthreads();
  return s;
}

// Visit every element of a row: UNROLL float4 loads in flight per thread for the body (rows
// of the [B, V] fp32 logits are 16-B aligned when V % 4 == 0), scalar loads for any tail.
// f(index, value) is called by every lane of the workgroup in step for the unrolled body.
template <typename F>
__device__ __forceinline__ void for_row(const float* __restrict__ x, int V, F f) {
  const int t = threadIdx.x;
  if ((V & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const int n4 = V >> 2;
    int j = t;
    for (; j + (UNROLL - 1) * NT < n4; j += UNROLL * NT) {
      float4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) v[u] = x4[j + u * NT];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int i = 4 * (j + u * NT);
        f(i, v[u].x);
        f(i + 1, v[u].y);
        f(i + 2, v[u].z);
        f(i + 3, v[u].w);
      }
    }
    for (; j < n4; j += NT) {
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

__device__ __forceinline__ int dist_bin(float d) { return min((int)(d * DSCALE), NBINS - 1); }

// exp(v - M) <= 1 in units of 2^-40; a row's total stays below 2^58
__device__ __forceinline__ uint64_t fixed_mass(float dv) {
  return (uint64_t)(__expf(dv) * (float)FIX);
}
template <bool MASS>
__device__ __forceinline__ uint64_t to_fixed(float w) {
  return MASS ? (uint64_t)((double)w * FIX) : (uint64_t)w;
}
template <bool MASS>
__device__ __forceinline__ float from_fixed(uint64_t q) {
  return MASS ? (float)((double)q * (1.0 / FIX)) : (float)q;
}

// Fast threshold: the largest key thr >= floor_key whose weight {key >= thr} reaches target,
// weight = 1 per token (MASS = false: top-k) or exp(v - M) (MASS = true: top-p). Also returns
// the probability mass (relative to exp(M)) kept by that threshold. Returns false, uniformly
// over the workgroup, when the caller must take the radix descent instead.
template <bool MASS>
__device__ __forceinline__ bool fast_select(const float* __restrict__ x, int V, float inv_t, float M,
                            uint32_t floor_key, float target, Smem& sm, uint32_t* thr_out,
                            float* kept_out) {
  const int t = threadIdx.x, lane = t & 63;
  for (int i = t; i < NBINS; i += NT) sm.u.s.h.q[i] = 0ull;
  if (t == 0) sm.ncand = 0;
  __syncthreads();
  for_row(x, V, [&](int, float raw) {
    const float v = raw * inv_t;
    const float d = M - v;
    if (d < DRANGE && fkey(v) >= floor_key)
      atomicAdd(&sm.u.s.h.q[NBINS - 1 - dist_bin(d)], MASS ? fixed_mass(v - M) : 1ull);
  });
  __syncthreads();
  uint64_t above_q;
  const int bin = find_crossing<uint64_t>(sm.u.s.h.q, NBINS, to_fixed<MASS>(target), &above_q,
                                          sm.u.s.scan.q, sm);
  if (bin < 0) return false;
  const float above = from_fixed<MASS>(above_q);
  const int cbin = NBINS - 1 - bin;  // crossing bin in distance order

  // gather the crossing bin's keys (wave-aggregated slots), and the mass of the bins above it
  float m_above = 0.f;
  for_row(x, V, [&](int, float raw) {
    const float v = raw * inv_t;
    const float d = M - v;
    const uint32_t key = fkey(v);
    bool want = false;
    if (d < DRANGE && key >= floor_key) {
      const int db = dist_bin(d);
      if (db < cbin) m_above += __expf(v - M);
      want = db == cbin;
    }
    const uint64_t m = __ballot(want);
    if (m != 0) {
      const int leader = __ffsll((unsigned long long)m) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(&sm.ncand, __popcll(m));
      base = __shfl(base, leader, 64);
      if (want) {
        const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
        if (pos < CAP) sm.u.s.cand[pos] = key;
      }
    }
  });
  m_above = block_sum(m_above, sm.red);  // starts and ends with a barrier
  const int n = sm.ncand;
  if (n > CAP || n == 0) return false;
  int sn = 2;
  while (sn < n) sn <<= 1;
  for (int i = n + t; i < sn; i += NT) sm.u.s.cand[i] = 0u;  // pads sort below every real key
  // bitonic sort, ascending
  for (int size = 2; size <= sn; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      if (t < (sn >> 1)) {
        const int i = 2 * t - (t & (stride - 1));
        const int j = i + stride;
        const uint32_t a = sm.u.s.cand[i], b = sm.u.s.cand[j];
        if ((a > b) == ((i & size) == 0)) {
          sm.u.s.cand[i] = b;
          sm.u.s.cand[j] = a;
        }
      }
    }
  __syncthreads();
  const int lo = sn - n;  // first real key
  for (int i = t; i < sn; i += NT)
    sm.u.s.h.w[i] = i < lo ? 0.f : (MASS ? __expf(fval(sm.u.s.cand[i]) - M) : 1.f);
  __syncthreads();
  float above2;
  int c = find_crossing<float>(sm.u.s.h.w, sn, target - above, &above2, sm.u.s.scan.f, sm);
  if (c < lo) c = lo;  // rounding: keep the whole bin
  const uint32_t thr = sm.u.s.cand[c];
  float km = 0.f;
  for (int i = lo + t; i < sn; i += NT)
    if (sm.u.s.cand[i] >= thr) km += __expf(fval(sm.u.s.cand[i]) - M);
  km = block_sum(km, sm.red);
  *thr_out = thr;
  *kept_out = m_above + km;
  return true;
}

// Exact radix descent (11/11/10 bits of the key) on counts (top-k) or fixed-point mass (top-p,
// restricted to key >= floor_key). Used when the fast path declines.
template <bool MASS>
__device__ __forceinline__ uint32_t radix_select(const float* __restrict__ x, int V, float inv_t,
                                                 float M, uint32_t floor_key, float target, Smem& sm) {
  const int t = threadIdx.x;
  uint32_t prefix = 0, mask = 0;
  uint64_t remaining = to_fixed<MASS>(target);
  for (int lvl = 0; lvl < 3; ++lvl) {
    for (int i = t; i < NBINS; i += NT) sm.u.s.h.q[i] = 0ull;
    __syncthreads();
    const int sh = lvl == 0 ? 21 : lvl == 1 ? 10 : 0;
    const uint32_t bm = lvl == 2 ? 0x3ffu : 0x7ffu;
    for_row(x, V, [&](int, float raw) {
      const float v = raw * inv_t;
      const uint32_t key = fkey(v);
      if ((key & mask) == prefix && key >= floor_key)
        atomicAdd(&sm.u.s.h.q[(key >> sh) & bm], MASS ? fixed_mass(v - M) : 1ull);
    });
    __syncthreads();
    uint64_t above;
    int bin = find_crossing<uint64_t>(sm.u.s.h.q, NBINS, remaining, &above, sm.u.s.scan.q, sm);
    if (bin < 0) {  // target beyond total (rounding): take the lowest populated bin
      bin = 0;
      above -= sm.u.s.h.q[0];
    }
    remaining -= above;
    prefix |= ((uint32_t)bin) << sh;
    mask |= bm << sh;
    __syncthreads();
  }
  return prefix;
}
}  // namespace

__global__ void __launch_bounds__(NT) sample_kernel(
    float* __restrict__ logits, int V, const float* __restrict__ temperature,
    const int32_t* __restrict__ top_k, const float* __restrict__ top_p,
    const float* __restrict__ rep_penalty, const int32_t* __restrict__ history, int hist_len,
    const int64_t* __restrict__ seeds, const int64_t* __restrict__ steps,
    int32_t* __restrict__ out_tok, float* __restrict__ out_logprob) {
  __shared__ Smem sm;

  const int row = blockIdx.x, t = threadIdx.x;
  float* x = logits + (int64_t)row * V;
  const float pen = rep_penalty ? rep_penalty[row] : 1.f;

  if (pen != 1.f && history != nullptr) {
    for (int i = t; i < 8192; i += NT) sm.u.bitmap[i] = 0;
    __syncthreads();
    const int32_t* hs = history + (int64_t)row * hist_len;
    for (int i = t; i < hist_len; i += NT) {
      const int tok = hs[i];
      if (tok >= 0 && tok < V) atomicOr(&sm.u.bitmap[tok >> 5], 1u << (tok & 31));
    }
    __syncthreads();
    for (int i = t; i < V; i += NT)
      if (sm.u.bitmap[i >> 5] & (1u << (i & 31))) {
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
  am = block_argmax(am, sm.ared);
  const float M = am.v;
  const float Z = block_sum(m_thr == -INFINITY ? 0.f : z * __expf(m_thr - M), sm.red);
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
    if (!fast_select<false>(x, V, inv_t, M, 0u, (float)k, sm, &thr, &kept_mass)) {
      thr = radix_select<false>(x, V, inv_t, M, 0u, (float)k, sm);
      float km = 0.f;
      for_row(x, V, [&](int, float raw) {
        const float v = raw * inv_t;
        if (fkey(v) >= thr) km += __expf(v - M);
      });
      kept_mass = block_sum(km, sm.red);
    }
  }
  if (p < 1.f) {
    uint32_t tp;
    float unused;
    if (!fast_select<true>(x, V, inv_t, M, thr, p * kept_mass, sm, &tp, &unused))
      tp = radix_select<true>(x, V, inv_t, M, thr, p * kept_mass, sm);
    thr = tp > thr ? tp : thr;
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
  best = block_argmax(best, sm.ared);
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
