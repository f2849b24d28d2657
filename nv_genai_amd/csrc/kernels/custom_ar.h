// Host API of the IPC custom all-reduce (custom_ar.hip). No PyTorch types here: the
// binding layer hands in raw device pointers and the current HIP stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace nga {

constexpr int kArMaxRanks = 8;
constexpr int kArMaxBlocks = 80;

class CustomAllReduce {
 public:
  // Allocates this rank's Signal block + 2 staging buffers of `cap_bytes` (uncached HBM).
  CustomAllReduce(int rank, int world, int64_t cap_bytes, double timeout_s);
  ~CustomAllReduce();
  CustomAllReduce(const CustomAllReduce&) = delete;
  CustomAllReduce& operator=(const CustomAllReduce&) = delete;

  // IPC handle (raw bytes) of this rank's allocation, to be exchanged with the peers.
  std::string handle() const;
  // Map every peer's allocation (handles indexed by rank; our own entry is ignored).
  void open(const std::vector<std::string>& handles);
  // out = sum over ranks of in (bf16 or fp32, `bytes` a multiple of 16). algo: 0 = pick by
  // size, 1 = one-shot, 2 = two-shot. Capture-safe: no allocation, no host sync.
  void run(const void* in, void* out, int64_t bytes, bool is_bf16, int algo, hipStream_t stream);
  // resid += sum over ranks of in; out = rmsnorm(resid) * w (bf16 [rows, H], one-shot).
  void run_add_rmsnorm(const void* in, uint16_t* resid, const uint16_t* w, uint16_t* out, int rows, int H,
                       float eps, hipStream_t stream);
  // out[row][r * row_bytes ...] = rank r's in[row] (all-gather along the last dim; `in` is
  // [rows, row_bytes] bytes, `out` [rows, world * row_bytes]; row_bytes % 16 == 0).
  void run_gather(const void* in, void* out, int64_t rows, int64_t row_bytes, hipStream_t stream);
  // Sticky barrier-timeout code (synchronous read; call outside graph capture): 0 = every
  // call met its peers in time, else which barrier first timed out (1 one-shot, 2 / 3
  // two-shot start / mid, 4 all-reduce + RMSNorm, 5 all-gather).
  int error() const;
  // Cap on workgroups per call (default kArMaxBlocks). Ranks that SHARE one device (the
  // one-GPU rehearsals) must keep every rank's spinning blocks co-resident at once, so they
  // lower it; on a node with one GPU per rank the default stands.
  void set_max_blocks(int b) { max_blocks_ = b < 1 ? 1 : (b > kArMaxBlocks ? kArMaxBlocks : b); }
  int max_blocks() const { return max_blocks_; }

  int64_t capacity() const { return cap_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  void set_two_shot_threshold(int64_t b) { two_shot_threshold_ = b; }
  static size_t alloc_bytes(int64_t cap);

 private:
  int grid_for(int64_t nvec, bool two_shot) const;
  int rank_, world_, device_ = 0;
  int64_t cap_;
  int64_t two_shot_threshold_ = 512 * 1024;
  int max_blocks_ = kArMaxBlocks;
  uint64_t timeout_ticks_ = 0;
  void* mine_ = nullptr;
  void* peers_[kArMaxRanks];
  bool opened_ = false;
};

}  // namespace nga
