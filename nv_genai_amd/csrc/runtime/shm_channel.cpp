// Shared-memory step channel: the driver of a model-parallel replica publishes each step's
// layout to the follower ranks on the same node without touching the GPU.
//
// Why not a collective: broadcasting the step over RCCL stages the host payload through the
// driver's current HIP stream (an H2D copy queued BEHIND the step still in flight), so the
// driver's host blocks until the GPU drains and a follower cannot launch step k + 1 before
// step k finishes — the TP engine could not pipeline its steps. Over gloo it is a TCP round
// trip per step. Here a step is a memcpy into a ring slot of a POSIX shared-memory segment
// and a release store; followers spin (then yield, then sleep) on the slot's sequence word.
//
// Layout: Header | nslots x Slot. Message s (1, 2, ...) goes to slot s % nslots. The writer
// waits until every reader has consumed message s - nslots (their per-reader `done` words),
// writes length + payload, then publishes slot.seq = s (release). A reader waiting for s
// acquires slot.seq == s, copies the payload out, then stores done[r] = s (release).
// `closed` (set by either side) makes every wait return at once — no rank can hang on a peer
// that went away; waits are also bounded by the caller's timeout.
//
// Lifetime: the creator makes the segment; readers attach by name; once every reader has
// attached the creator unlinks the name (`unlink()`), so a crash never leaves /dev/shm
// entries behind — the mapping lives until the last process unmaps it.
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

constexpr uint64_t kMagic = 0x6e67615f73746570ull;   // "nga_step"
constexpr int kMaxReaders = 64;

struct alignas(64) Header {
  uint64_t magic;
  uint64_t nslots;
  uint64_t slot_bytes;
  uint64_t nreaders;
  alignas(64) std::atomic<uint32_t> closed;
  alignas(64) std::atomic<uint32_t> attached;
  alignas(64) std::atomic<uint64_t> done[kMaxReaders];   // last message each reader consumed
};

struct alignas(64) SlotHead {
  std::atomic<uint64_t> seq;
  uint64_t len;
};

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

// spin -> yield -> short sleeps; returns false when `stop()` or the deadline says so
template <typename Ready, typename Stop>
bool wait_until(Ready ready, Stop stop, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (uint64_t i = 0;; ++i) {
    if (ready()) return true;
    if (stop()) return false;
    if (i < 4096) {
      cpu_relax();
      continue;
    }
    if (i < 8192) {
      sched_yield();
      continue;
    }
    if ((i & 63) == 0 && timeout_s >= 0 &&
        std::chrono::duration<double>(clk::now() - t0).count() > timeout_s)
      return false;
    timespec ts{0, i < 16384 ? 20000 : 200000};   // 20 us, then 200 us while idle
    nanosleep(&ts, nullptr);
  }
}

class ShmChannel {
 public:
  // create = true: make the segment (the writer); otherwise attach as reader `reader`
  ShmChannel(const std::string& name, bool create, int64_t nslots, int64_t slot_bytes, int64_t nreaders,
             int64_t reader)
      : name_(name), creator_(create), reader_(reader) {
    if (name.empty() || name[0] != '/') throw std::runtime_error("shm channel: name must start with '/'");
    int fd;
    if (create) {
      if (nslots < 2 || slot_bytes < 64 || nreaders < 1 || nreaders > kMaxReaders)
        throw std::runtime_error("shm channel: nslots >= 2, slot_bytes >= 64, 1 <= readers <= 64");
      slot_stride_ = (sizeof(SlotHead) + (size_t)slot_bytes + 63) / 64 * 64;
      bytes_ = sizeof(Header) + (size_t)nslots * slot_stride_;
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm channel: shm_open(create) failed for " + name);
      if (ftruncate(fd, (off_t)bytes_) != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("shm channel: ftruncate failed");
      }
    } else {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm channel: shm_open(attach) failed for " + name);
      struct stat st;
      if (fstat(fd, &st) != 0) {
        close(fd);
        throw std::runtime_error("shm channel: fstat failed");
      }
      bytes_ = (size_t)st.st_size;
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      if (create) shm_unlink(name.c_str());
      throw std::runtime_error("shm channel: mmap failed");
    }
    base_ = static_cast<uint8_t*>(p);
    hdr_ = reinterpret_cast<Header*>(base_);
    if (create) {
      std::memset(base_, 0, bytes_);
      new (hdr_) Header();
      hdr_->nslots = (uint64_t)nslots;
      hdr_->slot_bytes = (uint64_t)slot_bytes;
      hdr_->nreaders = (uint64_t)nreaders;
      std::atomic_thread_fence(std::memory_order_release);
      reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
    } else {
      if (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic)
        throw std::runtime_error("shm channel: not an initialised channel segment");
      if (reader < 0 || (uint64_t)reader >= hdr_->nreaders) throw std::runtime_error("shm channel: reader index out of range");
      slot_stride_ = (sizeof(SlotHead) + hdr_->slot_bytes + 63) / 64 * 64;
      hdr_->attached.fetch_add(1, std::memory_order_acq_rel);
    }
  }

  ~ShmChannel() {
    if (creator_ && !unlinked_) shm_unlink(name_.c_str());
    if (base_) munmap(base_, bytes_);
  }

  int64_t slot_bytes() const { return (int64_t)hdr_->slot_bytes; }
  int64_t attached() const { return hdr_->attached.load(std::memory_order_acquire); }
  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  void close_channel() { hdr_->closed.store(1, std::memory_order_release); }

  // Remove the name (every reader attached); the segment lives on in the mappings.
  void unlink() {
    if (creator_ && !unlinked_) {
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  // Publish one message; false on timeout or a closed channel.
  bool write(py::buffer buf, double timeout_s) {
    if (!creator_) throw std::runtime_error("shm channel: only the creator writes");
    py::buffer_info bi = buf.request();
    if (!bi.strides.empty() && bi.strides.back() != bi.itemsize)
      throw std::runtime_error("shm channel: the message must be a contiguous buffer");
    const size_t len = (size_t)bi.size * (size_t)bi.itemsize;
    if (len > hdr_->slot_bytes) throw std::runtime_error("shm channel: message exceeds the slot size");
    const uint64_t s = ++wseq_;
    const uint64_t nr = hdr_->nreaders;
    const uint64_t need = s > hdr_->nslots ? s - hdr_->nslots : 0;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = wait_until(
          [&] {
            for (uint64_t r = 0; r < nr; ++r)
              if (hdr_->done[r].load(std::memory_order_acquire) < need) return false;
            return true;
          },
          [&] { return closed(); }, timeout_s);
    }
    if (!ok) {
      --wseq_;
      return false;
    }
    SlotHead* sh = slot(s);
    sh->len = len;
    std::memcpy(reinterpret_cast<uint8_t*>(sh) + sizeof(SlotHead), bi.ptr, len);
    sh->seq.store(s, std::memory_order_release);
    return true;
  }

  // Wait for the next message and copy it into `out` (a writable buffer at least as large);
  // returns its length, -1 on timeout, -2 when the channel was closed.
  int64_t read(py::buffer out, double timeout_s) {
    if (creator_) throw std::runtime_error("shm channel: the creator does not read");
    py::buffer_info bi = out.request(true);
    const size_t cap = (size_t)bi.size * (size_t)bi.itemsize;
    const uint64_t s = rseq_ + 1;
    SlotHead* sh = slot(s);
    bool ok;
    {
      py::gil_scoped_release nogil;
      auto ready = [&] { return sh->seq.load(std::memory_order_acquire) == s; };
      // a message published just before the close is still delivered
      ok = wait_until(ready, [&] { return closed() && !ready(); }, timeout_s);
    }
    if (!ok) return closed() ? -2 : -1;
    const size_t len = sh->len;
    if (len > cap) throw std::runtime_error("shm channel: receive buffer too small");
    std::memcpy(bi.ptr, reinterpret_cast<const uint8_t*>(sh) + sizeof(SlotHead), len);
    rseq_ = s;
    hdr_->done[reader_].store(s, std::memory_order_release);
    return (int64_t)len;
  }

 private:
  SlotHead* slot(uint64_t s) { return reinterpret_cast<SlotHead*>(base_ + sizeof(Header) + (s % hdr_->nslots) * slot_stride_); }

  std::string name_;
  bool creator_;
  int64_t reader_;
  bool unlinked_ = false;
  uint8_t* base_ = nullptr;
  Header* hdr_ = nullptr;
  size_t bytes_ = 0, slot_stride_ = 0;
  uint64_t wseq_ = 0, rseq_ = 0;
};

}  // namespace

void register_shm(py::module_& m) {
  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<const std::string&, bool, int64_t, int64_t, int64_t, int64_t>(), py::arg("name"),
           py::arg("create"), py::arg("nslots") = 4, py::arg("slot_bytes") = 1 << 20, py::arg("nreaders") = 1,
           py::arg("reader") = 0)
      .def("write", &ShmChannel::write, py::arg("buf"), py::arg("timeout_s") = -1.0)
      .def("read", &ShmChannel::read, py::arg("out"), py::arg("timeout_s") = -1.0)
      .def("unlink", &ShmChannel::unlink)
      .def("close", &ShmChannel::close_channel)
      .def("closed", &ShmChannel::closed)
      .def("attached", &ShmChannel::attached)
      .def("slot_bytes", &ShmChannel::slot_bytes);
}
