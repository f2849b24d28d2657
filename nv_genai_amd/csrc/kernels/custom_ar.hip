// Custom all-reduce over IPC-mapped peer memory (xGMI), for latency-bound tensor-parallel
// decode messages (Llama-3-70B TP=8 does 160 all-reduces of
// 16 KiB x batch per generated token). The MI355X analogue of TRT-LLM's
// `enable_custom_all_reduce` (experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:36).
//
// Why not RCCL for these: a ring all-reduce moves every byte through W-1 serial hops, each
// on ONE of the 7 xGMI links, and pays per-hop launch/protocol latency. Here every rank
// reads its peers' buffers directly, so all 7 links are busy at once and a call costs two
// (one-shot) or three (two-shot) cross-GPU flag round trips plus the data time.
//
// Memory: each rank owns one uncached allocation (hipDeviceMallocUncached) holding a
// Signal block followed by two staging buffers (double-buffered by call parity). The
// allocation is exported with hipIpcGetMemHandle and opened by every peer. Stores to
// uncached memory go to HBM, so a peer's read over xGMI never meets a stale cache line.
//
// Algorithms (same deterministic fp32 sum in rank order 0..W-1 on every rank, so all
// ranks get bit-identical results — unlike ring reductions):
//   one-shot : copy input -> own staging; barrier; out[i] = sum_r staging_r[i]
//   two-shot : copy input -> own staging; barrier; reduce own 1/W chunk from all ranks,
//              write it back in place; barrier; gather every chunk from its owner
// Barriers are per block (block b only waits for block b of every peer) because block b
// touches exactly the same element set on every rank (same grid, same mapping).
//
// Safety: every wait is bounded by a wall-clock timeout; on expiry the kernel records a
// sticky error in its own Signal and every later call returns at once, so a lost peer can
// never hang the GPU. The host checks `error()` after its start-up self-test.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "custom_ar.h"

namespace nga {

namespace {

constexpr int kThreads = 512;

struct Signal {
  uint32_t start[kArMaxBlocks][kArMaxRanks];
  uint32_t mid[kArMaxBlocks][kArMaxRanks];
  uint32_t calls;  // completed calls; read by every block at start, bumped by the last block
  uint32_t done;   // blocks finished in the current call
  uint32_t error;  // sticky: != 0 = a barrier timed out (code of the first barrier that did)
  uint32_t pad[29];
};
static_assert(sizeof(Signal) % 128 == 0, "Signal must keep the staging buffers 128-B aligned");

struct ArArgs {
  const uint8_t* base[kArMaxRanks];  // each rank's allocation (Signal, then 2 staging buffers)
  const void* in;
  void* out;
  int64_t nvec;     // number of 16-B packets
  int64_t cap;      // bytes per staging buffer
  uint64_t timeout; // wall-clock ticks
  int rank;
  int world;
  int is_bf16;
};

__device__ __forceinline__ Signal* sig_of(const ArArgs& a, int r) {
  return reinterpret_cast<Signal*>(const_cast<uint8_t*>(a.base[r]));
}

__device__ __forceinline__ uint4* stage_of(const ArArgs& a, int r, uint32_t parity) {
  return reinterpret_cast<uint4*>(const_cast<uint8_t*>(a.base[r]) + sizeof(Signal) + parity * a.cap);
}

// Per-block cross-rank barrier on `slot` (start or mid). Every thread first publishes its
// own stores system-wide; thread r < world then raises our flag in peer r's Signal and
// waits for peer r's flag in ours. Returns false on timeout.
__device__ bool block_barrier(const ArArgs& a, size_t slot_off, uint32_t flag) {
  __threadfence_system();
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    uint32_t* remote = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(sig_of(a, t)) + slot_off) +
                       blockIdx.x * kArMaxRanks + a.rank;
    __hip_atomic_store(remote, flag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* local = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(sig_of(a, a.rank)) + slot_off) +
                      blockIdx.x * kArMaxRanks + t;
    const uint64_t t0 = wall_clock64();
    int n = 0;
    while ((int32_t)(__hip_atomic_load(local, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - flag) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if ((++n & 255) == 0 && (uint64_t)(wall_clock64() - t0) > a.timeout) {
        ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  return ok != 0;
}

__device__ __forceinline__ void acc_packet(float (&acc)[8], uint4 v, int is_bf16) {
  if (is_bf16) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[2 * j] += __uint_as_float(w[j] << 16);
      acc[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    acc[0] += __uint_as_float(v.x);
    acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z);
    acc[3] += __uint_as_float(v.w);
  }
}

__device__ __forceinline__ uint4 pack_packet(const float (&acc)[8], int is_bf16) {
  uint4 r;
  if (is_bf16) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)f2bf(acc[2 * j]) | ((uint32_t)f2bf(acc[2 * j + 1]) << 16);
    r = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    r = make_uint4(__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]),
                   __float_as_uint(acc[3]));
  }
  return r;
}

__device__ __forceinline__ uint4 reduce_at(const ArArgs& a, uint32_t parity, int64_t i) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < a.world; ++r) acc_packet(acc, stage_of(a, r, parity)[i], a.is_bf16);
  return pack_packet(acc, a.is_bf16);
}

// Common prologue: this call's flag (completed calls + 1; wraps harmlessly, every flag
// comparison is wrap-aware). Returns false when an earlier call poisoned the object.
__device__ __forceinline__ bool begin_call(const ArArgs& a, uint32_t& flag) {
  Signal* me = sig_of(a, a.rank);
  __shared__ uint32_t f, bad;
  if (threadIdx.x == 0) {
    bad = __hip_atomic_load(&me->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    f = __hip_atomic_load(&me->calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  }
  __syncthreads();
  flag = f;
  return bad == 0u;
}

// timeout codes (CustomAllReduce::error)
constexpr uint32_t kErrOneShot = 1, kErrTwoShotStart = 2, kErrTwoShotMid = 3, kErrAddNorm = 4, kErrGather = 5;

__device__ __forceinline__ void end_call(const ArArgs& a, uint32_t flag, uint32_t err) {
  Signal* me = sig_of(a, a.rank);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (err) {
      uint32_t zero = 0u;   // keep the first code
      __hip_atomic_compare_exchange_strong(&me->error, &zero, err, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t d = __hip_atomic_fetch_add(&me->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1) {
      __hip_atomic_store(&me->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&me->calls, flag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(kThreads) void ar_one_shot(ArArgs a) {
  uint32_t flag;
  if (!begin_call(a, flag)) return;
  const uint32_t par = flag & 1u;
  const uint4* in = reinterpret_cast<const uint4*>(a.in);
  uint4* mine = stage_of(a, a.rank, par);
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < a.nvec; i += stride) mine[i] = in[i];
  bool ok = block_barrier(a, offsetof(Signal, start), flag);
  if (ok) {
    uint4* out = reinterpret_cast<uint4*>(a.out);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < a.nvec; i += stride)
      out[i] = reduce_at(a, par, i);
  }
  end_call(a, flag, ok ? 0u : kErrOneShot);
}

__global__ __launch_bounds__(kThreads) void ar_two_shot(ArArgs a) {
  uint32_t flag;
  if (!begin_call(a, flag)) return;
  const uint32_t par = flag & 1u;
  const uint4* in = reinterpret_cast<const uint4*>(a.in);
  uint4* mine = stage_of(a, a.rank, par);
  const int64_t chunk = (a.nvec + a.world - 1) / a.world;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  // A: whole input -> own staging, block b writing sub-range b of every chunk
  for (int j = 0; j < a.world; ++j)
    for (int64_t i = i0; i < chunk; i += stride) {
      const int64_t e = j * chunk + i;
      if (e < a.nvec) mine[e] = in[e];
    }
  bool ok = block_barrier(a, offsetof(Signal, start), flag);
  uint32_t err = ok ? 0u : kErrTwoShotStart;
  if (ok) {
    // B: reduce my chunk (sub-range b) from every rank, in place into my staging
    for (int64_t i = i0; i < chunk; i += stride) {
      const int64_t e = a.rank * chunk + i;
      if (e < a.nvec) mine[e] = reduce_at(a, par, e);
    }
    ok = block_barrier(a, offsetof(Signal, mid), flag);
    if (!ok) err = kErrTwoShotMid;
  }
  if (ok) {
    // C: gather chunk r (sub-range b) from its owner r
    uint4* out = reinterpret_cast<uint4*>(a.out);
    for (int r = 0; r < a.world; ++r) {
      const uint4* src = stage_of(a, r, par);
      for (int64_t i = i0; i < chunk; i += stride) {
        const int64_t e = r * chunk + i;
        if (e < a.nvec) out[e] = src[e];
      }
    }
  }
  end_call(a, flag, err);
}

// Fused TP epilogue: resid += all_reduce(in); out = rmsnorm(resid) * w  (one-shot, bf16).
// The row-parallel GEMM output is summed over the ranks, added to the residual stream and
// normalised for the next GEMM in one pass: the sum never round-trips through HBM and the
// separate add+RMSNorm launch disappears. Rounding matches the unfused path (sum -> bf16,
// resid + sum -> bf16, norm of the stored residual). Block b owns rows b, b + G, ...
constexpr int kNormMaxVec = 4;  // packets per thread: H <= 4 * 512 * 8 = 16384

__global__ __launch_bounds__(kThreads) void ar_add_rmsnorm(ArArgs a, uint16_t* __restrict__ resid,
                                                           const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ out, int rows, int H,
                                                           float eps) {
  uint32_t flag;
  if (!begin_call(a, flag)) return;
  const uint32_t par = flag & 1u;
  const int hv = H / 8;
  const uint4* in = reinterpret_cast<const uint4*>(a.in);
  uint4* mine = stage_of(a, a.rank, par);
  for (int row = blockIdx.x; row < rows; row += gridDim.x)
    for (int p = threadIdx.x; p < hv; p += kThreads) mine[(int64_t)row * hv + p] = in[(int64_t)row * hv + p];
  bool ok = block_barrier(a, offsetof(Signal, start), flag);
  __shared__ float red[kThreads / 64];
  if (ok) {
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
      float x[kNormMaxVec][8];
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < kNormMaxVec; ++j) {
        const int p = threadIdx.x + j * kThreads;
        if (p < hv) {
          const int64_t e = (int64_t)row * hv + p;
          float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          for (int r = 0; r < a.world; ++r) acc_packet(acc, stage_of(a, r, par)[e], 1);
          u16x8 rv = load8(resid + e * 8);
          u16x8 sv;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float o = bf2f(f2bf(acc[i]));          // the all-reduced value, as bf16
            sv[i] = f2bf(bf2f(rv[i]) + o);
            x[j][i] = bf2f(sv[i]);
            ss += x[j][i] * x[j][i];
          }
          store8(resid + e * 8, sv);
        }
      }
      ss = block_sum(ss, red);
      const float rs = rsqrtf(ss / (float)H + eps);
#pragma unroll
      for (int j = 0; j < kNormMaxVec; ++j) {
        const int p = threadIdx.x + j * kThreads;
        if (p < hv) {
          u16x8 wv = load8(w + p * 8);
          u16x8 ov;
#pragma unroll
          for (int i = 0; i < 8; ++i) ov[i] = f2bf(x[j][i] * rs * bf2f(wv[i]));
          store8(out + ((int64_t)row * hv + p) * 8, ov);
        }
      }
      __syncthreads();  // red[] is reused by the next row
    }
  }
  end_call(a, flag, ok ? 0u : kErrAddNorm);
}

// All-gather along the last dim: out[row][r * cols + c] = in_r[row][c] for every rank r (the
// vocab-parallel LM head's logits, CC4). Every rank copies its shard into its own staging
// buffer; after the per-block barrier each block copies the same input packets it staged
// from every rank's staging buffer into the right column block of `out` (block b touches the
// same packet set on every rank, so the per-block barrier suffices, as in the one-shot).
__global__ __launch_bounds__(kThreads) void ag_last_dim(ArArgs a, int64_t rows, int64_t cpk) {
  uint32_t flag;
  if (!begin_call(a, flag)) return;
  const uint32_t par = flag & 1u;
  const uint4* in = reinterpret_cast<const uint4*>(a.in);
  uint4* mine = stage_of(a, a.rank, par);
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  for (int64_t i = i0; i < a.nvec; i += stride) mine[i] = in[i];
  bool ok = block_barrier(a, offsetof(Signal, start), flag);
  if (ok) {
    uint4* out = reinterpret_cast<uint4*>(a.out);
    for (int r = 0; r < a.world; ++r) {
      const uint4* src = stage_of(a, r, par);
      for (int64_t i = i0; i < a.nvec; i += stride) {
        const int64_t row = i / cpk, c = i - row * cpk;
        out[(row * a.world + r) * cpk + c] = src[i];
      }
    }
  }
  end_call(a, flag, ok ? 0u : kErrGather);
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

size_t CustomAllReduce::alloc_bytes(int64_t cap) { return sizeof(Signal) + 2 * (size_t)cap; }

CustomAllReduce::CustomAllReduce(int rank, int world, int64_t cap_bytes, double timeout_s)
    : rank_(rank), world_(world), cap_(cap_bytes) {
  if (world < 1 || world > kArMaxRanks || rank < 0 || rank >= world)
    throw std::runtime_error("custom all-reduce: 1 <= world <= 8 and 0 <= rank < world");
  if (cap_bytes <= 0 || cap_bytes % 128 != 0)
    throw std::runtime_error("custom all-reduce: capacity must be a positive multiple of 128 B");
  check(hipGetDevice(&device_), "hipGetDevice");
  int khz = 0;
  check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_), "wall clock rate");
  timeout_ticks_ = (uint64_t)(timeout_s * 1e3 * (khz > 0 ? khz : 100000));
  check(hipExtMallocWithFlags(&mine_, alloc_bytes(cap_bytes), hipDeviceMallocUncached), "hipExtMallocWithFlags");
  check(hipMemset(mine_, 0, sizeof(Signal)), "hipMemset");
  check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  for (int r = 0; r < kArMaxRanks; ++r) peers_[r] = nullptr;
  peers_[rank_] = mine_;
}

CustomAllReduce::~CustomAllReduce() {
  for (int r = 0; r < world_; ++r)
    if (r != rank_ && peers_[r]) (void)hipIpcCloseMemHandle(peers_[r]);
  if (mine_) (void)hipFree(mine_);
}

std::string CustomAllReduce::handle() const {
  hipIpcMemHandle_t h;
  check(hipIpcGetMemHandle(&h, mine_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void CustomAllReduce::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("custom all-reduce: need one handle per rank");
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("custom all-reduce: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    peers_[r] = p;
  }
  opened_ = true;
}

int CustomAllReduce::grid_for(int64_t nvec, bool two_shot) const {
  const int64_t work = two_shot ? (nvec + world_ - 1) / world_ : nvec;
  int64_t g = (work + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > max_blocks_) g = max_blocks_;
  return (int)g;
}

void CustomAllReduce::run(const void* in, void* out, int64_t bytes, bool is_bf16, int algo,
                          hipStream_t stream) {
  if (!opened_) throw std::runtime_error("custom all-reduce: open() the peer handles first");
  if (bytes <= 0 || bytes % 16 != 0 || bytes > cap_)
    throw std::runtime_error("custom all-reduce: size must be a positive multiple of 16 B within capacity");
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15)
    throw std::runtime_error("custom all-reduce: buffers must be 16-B aligned");
  ArArgs a;
  for (int r = 0; r < kArMaxRanks; ++r) a.base[r] = static_cast<const uint8_t*>(r < world_ ? peers_[r] : nullptr);
  a.in = in;
  a.out = out;
  a.nvec = bytes / 16;
  a.cap = cap_;
  a.timeout = timeout_ticks_;
  a.rank = rank_;
  a.world = world_;
  a.is_bf16 = is_bf16 ? 1 : 0;
  const bool two = algo == 2 || (algo == 0 && bytes > two_shot_threshold_ && world_ > 2);
  const int g = grid_for(a.nvec, two);
  if (two)
    hipLaunchKernelGGL(ar_two_shot, dim3(g), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(ar_one_shot, dim3(g), dim3(kThreads), 0, stream, a);
}

void CustomAllReduce::run_add_rmsnorm(const void* in, uint16_t* resid, const uint16_t* w, uint16_t* out,
                                      int rows, int H, float eps, hipStream_t stream) {
  if (!opened_) throw std::runtime_error("custom all-reduce: open() the peer handles first");
  const int64_t bytes = (int64_t)rows * H * 2;
  if (rows <= 0 || H % 8 != 0 || H > kNormMaxVec * kThreads * 8 || bytes > cap_)
    throw std::runtime_error("custom all-reduce + rmsnorm: rows > 0, H % 8 == 0, H <= 16384, within capacity");
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(resid) | reinterpret_cast<uintptr_t>(w) |
       reinterpret_cast<uintptr_t>(out)) & 15)
    throw std::runtime_error("custom all-reduce + rmsnorm: buffers must be 16-B aligned");
  ArArgs a;
  for (int r = 0; r < kArMaxRanks; ++r) a.base[r] = static_cast<const uint8_t*>(r < world_ ? peers_[r] : nullptr);
  a.in = in;
  a.out = out;
  a.nvec = bytes / 16;
  a.cap = cap_;
  a.timeout = timeout_ticks_;
  a.rank = rank_;
  a.world = world_;
  a.is_bf16 = 1;
  const int g = rows < max_blocks_ ? rows : max_blocks_;
  hipLaunchKernelGGL(ar_add_rmsnorm, dim3(g), dim3(kThreads), 0, stream, a, resid, w, out, rows, H, eps);
}

void CustomAllReduce::run_gather(const void* in, void* out, int64_t rows, int64_t row_bytes, hipStream_t stream) {
  if (!opened_) throw std::runtime_error("custom all-reduce: open() the peer handles first");
  const int64_t bytes = rows * row_bytes;
  if (rows <= 0 || row_bytes <= 0 || row_bytes % 16 != 0 || bytes > cap_)
    throw std::runtime_error("custom all-gather: rows > 0, row bytes a multiple of 16, shard within capacity");
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15)
    throw std::runtime_error("custom all-gather: buffers must be 16-B aligned");
  ArArgs a;
  for (int r = 0; r < kArMaxRanks; ++r) a.base[r] = static_cast<const uint8_t*>(r < world_ ? peers_[r] : nullptr);
  a.in = in;
  a.out = out;
  a.nvec = bytes / 16;
  a.cap = cap_;
  a.timeout = timeout_ticks_;
  a.rank = rank_;
  a.world = world_;
  a.is_bf16 = 0;
  const int g = grid_for(a.nvec, false);
  hipLaunchKernelGGL(ag_last_dim, dim3(g), dim3(kThreads), 0, stream, a, rows, row_bytes / 16);
}

int CustomAllReduce::error() const {
  uint32_t e = 0;
  check(hipMemcpy(&e, static_cast<uint8_t*>(mine_) + offsetof(Signal, error), sizeof(e), hipMemcpyDeviceToHost),
        "hipMemcpy");
  return (int)e;
}

}  // namespace nga
