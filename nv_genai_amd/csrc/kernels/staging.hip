// Step-input upload in one piece: the engine packs every host buffer a step needs (token ids,
// positions, KV slots, cu_seqlens, contexts, block tables, sampling parameters, the pipelined
// id gather, the step graph's work list) contiguously into a pinned staging buffer, copies it
// to the device with ONE hipMemcpyAsync, and this kernel scatters the segments to the fixed
// device buffers the step (and its captured hipGraph) reads. Before, every buffer was its own
// copy: ~18 blit dispatches of ~4.5 us each per step on the compute stream, each issued by a
// separate host API call (profiles/r6_busy: copyBuffer -> copyBuffer gaps were the largest idle
// source in the timed window's kernel trace).
//
// Grid: (segments, SPLIT) workgroups of 256 threads; workgroup (s, j) copies the 16-B packets
// j, j + SPLIT, ... (x 256 lanes) of segment s, then the 4-B tail words (every segment is
// a whole number of 4-B elements; offsets and destinations are 16-B aligned).
#include "common.h"
#include "kernels.h"

namespace nga {

namespace {
constexpr int kSplit = 8;
}

__global__ void __launch_bounds__(256) scatter_segments_kernel(const uint8_t* __restrict__ src, SegmentTable t) {
  const int s = blockIdx.x;
  if (s >= t.n) return;
  const uint8_t* a = src + t.off[s];
  uint8_t* d = reinterpret_cast<uint8_t*>(t.dst[s]);
  const int64_t nb = t.bytes[s];
  const int64_t nv = nb / 16;
  const int64_t step = (int64_t)kSplit * 256;
  for (int64_t i = (int64_t)blockIdx.y * 256 + threadIdx.x; i < nv; i += step)
    reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(a)[i];
  if (blockIdx.y == 0) {
    const int64_t w0 = nv * 4, nw = nb / 4;
    for (int64_t w = w0 + threadIdx.x; w < nw; w += 256)
      reinterpret_cast<uint32_t*>(d)[w] = reinterpret_cast<const uint32_t*>(a)[w];
  }
}

void launch_scatter_segments(const uint8_t* src, const SegmentTable& t, hipStream_t stream) {
  if (t.n <= 0) return;
  scatter_segments_kernel<<<dim3(t.n, kSplit), 256, 0, stream>>>(src, t);
}

}  // namespace nga
