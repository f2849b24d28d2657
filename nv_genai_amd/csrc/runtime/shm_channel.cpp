// Shared-memory step channel: the driver of a model-parallel replica publishes each step's
// layout to the follower ranks on the same node without touching the GPU.
//
// Why not a collective: broadcasting the step over RCCL stages the host payload through the
// driver's current HIP stream (an H2D copy queued BEHIND the step still in flight), so the
// driver's host blocks until the GPU drains and a follower cannot launch step k + 1 before
// step k finishes — the TP engine could not pipeline its steps. Over gloo it is a TCP round
// trip per step. Here a step is a memcpy into a ring slot of a POSIX shared-memory segment
// and a release store.
//
// Layout: Header | nslots x Slot. Message s (1, 2, ...) goes to slot s % nslots. The writer
// waits until every reader has consumed message s - nslots (their per-reader `done` words),
// writes length + payload, then publishes slot.seq = s (release). A reader waiting for s
// acquires slot.seq == s, copies the payload out, then stores done[r] = s (release).
//
// Waiting: spin (pause) for a few microseconds — the pipelined engine publishes step k + 1
// while the followers still launch step k, so a follower usually finds its message at once —
// then yield briefly, then sleep on a futex: readers on `pub_gen`, which the writer bumps
// after every publish and wakes only when someone sleeps (`sleepers`, a Dekker pair of
// seq_cst operations so a publish can never slip between a reader's check and its sleep);
// the writer (ring full) likewise on `done_gen`. Wake-up is a syscall away, not the next tick
// of a sleep loop (round 5's 200 us sleeps), and an idle replica costs no CPU.
//
// Liveness, not deadlines: every participant runs a heartbeat thread (C++, no GIL) that
// stamps its word in the header every 100 ms. A wait ends with "peer dead" once the peer it
// waits on (the writer, for a reader; any attached reader, for the writer) has not stamped
// for `liveness_s`, so an idle replica waits for its next step indefinitely while a crashed
// driver is noticed within seconds. `closed` (set by either side) makes every wait return at
// once, and a caller may still pass a hard timeout.
//
// Lifetime: the creator makes the segment; readers attach by name; once every reader has
// attached the creator unlinks the name (`unlink()`), so a crash never leaves /dev/shm
// entries behind — the mapping lives until the last process unmaps it.
#include <fcntl.h>
#include <linux/futex.h>
#include <pybind11/pybind11.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

constexpr uint64_t kMagic = 0x6e67615f73746570ull;   // "nga_step"
constexpr int kMaxReaders = 64;
constexpr int64_t kBeatNs = 100'000'000;             // heartbeat period

// wait outcomes (also the Python return codes)
constexpr int kOk = 1, kTimeout = -1, kClosed = -2, kPeerDead = -3;

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1'000'000'000 + ts.tv_nsec;
}

struct alignas(64) Header {
  uint64_t magic;
  uint64_t nslots;
  uint64_t slot_bytes;
  uint64_t nreaders;
  alignas(64) std::atomic<uint32_t> closed;
  alignas(64) std::atomic<uint32_t> attached;
  alignas(64) std::atomic<uint32_t> pub_gen;      // futex word: bumped after every publish / close
  std::atomic<uint32_t> sleepers;                 // readers inside a futex wait on pub_gen
  alignas(64) std::atomic<uint32_t> done_gen;     // futex word: bumped after every consume / close
  std::atomic<uint32_t> writer_sleeping;
  alignas(64) std::atomic<int64_t> beat[kMaxReaders + 1];   // [0] writer, [1 + r] reader r; 0 = never
  alignas(64) std::atomic<uint64_t> done[kMaxReaders];      // last message each reader consumed
};

struct alignas(64) SlotHead {
  std::atomic<uint64_t> seq;
  uint64_t len;
  int64_t pub_ns;    // writer's clock at publish: the reader's wake-up latency
};

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

// shared (not PRIVATE) futex ops: the word lives in a MAP_SHARED segment of several processes
inline void futex_wait(std::atomic<uint32_t>* w, uint32_t expect, int64_t ns) {
  timespec ts{(time_t)(ns / 1'000'000'000), (long)(ns % 1'000'000'000)};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expect, &ts, nullptr, 0);
}
inline void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

struct WaitStats {
  uint64_t spins = 0, yields = 0, sleeps = 0;
};

// spin -> yield -> futex sleep on `gen` (registering in `sleepers`); returns kOk, kClosed,
// kPeerDead (from `dead()`) or kTimeout (timeout_s >= 0 elapsed)
template <typename Ready, typename Closed, typename Dead>
int wait_until(Ready ready, Closed closed, Dead dead, std::atomic<uint32_t>* gen, std::atomic<uint32_t>* sleepers,
               double timeout_s, WaitStats& st) {
  for (int i = 0; i < 8192; ++i) {   // ~20-60 us
    if (ready()) { ++st.spins; return kOk; }
    if (closed()) return kClosed;
    cpu_relax();
  }
  for (int i = 0; i < 64; ++i) {
    if (ready()) { ++st.yields; return kOk; }
    if (closed()) return kClosed;
    sched_yield();
  }
  const int64_t t0 = now_ns();
  const int64_t limit = timeout_s >= 0 ? (int64_t)(timeout_s * 1e9) : INT64_MAX;
  for (;;) {
    sleepers->fetch_add(1, std::memory_order_seq_cst);
    const uint32_t g = gen->load(std::memory_order_seq_cst);
    if (ready()) {
      sleepers->fetch_sub(1, std::memory_order_seq_cst);
      ++st.sleeps;
      return kOk;
    }
    if (!closed()) futex_wait(gen, g, 20'000'000);   // 20 ms slices: liveness / deadline checks
    sleepers->fetch_sub(1, std::memory_order_seq_cst);
    if (ready()) { ++st.sleeps; return kOk; }
    if (closed()) return kClosed;
    if (dead()) return kPeerDead;
    if (now_ns() - t0 > limit) return kTimeout;
  }
}

class ShmChannel {
 public:
  // create = true: make the segment (the writer); otherwise attach as reader `reader`
  ShmChannel(const std::string& name, bool create, int64_t nslots, int64_t slot_bytes, int64_t nreaders,
             int64_t reader, double liveness_s)
      : name_(name), creator_(create), reader_(reader), liveness_ns_((int64_t)(liveness_s * 1e9)) {
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
      hdr_->beat[0].store(now_ns(), std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
      beat_idx_ = 0;
    } else {
      if (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic)
        throw std::runtime_error("shm channel: not an initialised channel segment");
      if (reader < 0 || (uint64_t)reader >= hdr_->nreaders) throw std::runtime_error("shm channel: reader index out of range");
      slot_stride_ = (sizeof(SlotHead) + hdr_->slot_bytes + 63) / 64 * 64;
      beat_idx_ = 1 + (int)reader;
      hdr_->beat[beat_idx_].store(now_ns(), std::memory_order_release);
      hdr_->attached.fetch_add(1, std::memory_order_acq_rel);
    }
    owner_pid_ = getpid();
    beat_ = new Beat();
    beat_->th = std::thread([this] { beat_loop(); });
  }

  ~ShmChannel() {
    if (getpid() != owner_pid_) {
      // a copy inherited across fork(): the heartbeat thread and the name belong to the parent;
      // leave both alone. The heartbeat state is leaked on purpose: its thread does not exist
      // here (destroying a joinable std::thread would terminate the process).
      if (base_) munmap(base_, bytes_);
      return;
    }
    stop_beating();
    delete beat_;
    if (creator_ && !unlinked_) shm_unlink(name_.c_str());
    if (base_) munmap(base_, bytes_);
  }

  int64_t slot_bytes() const { return (int64_t)hdr_->slot_bytes; }
  int64_t attached() const { return hdr_->attached.load(std::memory_order_acquire); }
  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  void close_channel() {
    hdr_->closed.store(1, std::memory_order_seq_cst);
    hdr_->pub_gen.fetch_add(1, std::memory_order_seq_cst);
    hdr_->done_gen.fetch_add(1, std::memory_order_seq_cst);
    futex_wake_all(&hdr_->pub_gen);
    futex_wake_all(&hdr_->done_gen);
  }

  // Remove the name (every reader attached); the segment lives on in the mappings.
  void unlink() {
    if (creator_ && !unlinked_) {
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  // Stop this participant's heartbeat (tests: a peer that hangs without exiting).
  void stop_beating() {
    if (getpid() != owner_pid_ || beat_ == nullptr) return;   // no heartbeat thread in a forked copy
    if (beat_->stop.exchange(1) != 0) return;
    futex_wake_all(&beat_->stop);
    if (beat_->th.joinable()) beat_->th.join();
  }

  // Publish one message: 1, or -1 timeout, -2 closed, -3 a reader died.
  int write(py::buffer buf, double timeout_s) {
    if (!creator_) throw std::runtime_error("shm channel: only the creator writes");
    py::buffer_info bi = buf.request();
    if (!bi.strides.empty() && bi.strides.back() != bi.itemsize)
      throw std::runtime_error("shm channel: the message must be a contiguous buffer");
    const size_t len = (size_t)bi.size * (size_t)bi.itemsize;
    if (len > hdr_->slot_bytes) throw std::runtime_error("shm channel: message exceeds the slot size");
    const uint64_t s = wseq_ + 1;
    const uint64_t nr = hdr_->nreaders;
    const uint64_t need = s > hdr_->nslots ? s - hdr_->nslots : 0;
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = wait_until(
          [&] {
            for (uint64_t r = 0; r < nr; ++r)
              if (hdr_->done[r].load(std::memory_order_acquire) < need) return false;
            return true;
          },
          [&] { return closed(); },
          [&] {
            for (uint64_t r = 0; r < nr; ++r)
              if (hdr_->done[r].load(std::memory_order_acquire) < need && stale(1 + (int)r)) return true;
            return false;
          },
          &hdr_->done_gen, &hdr_->writer_sleeping, timeout_s, wstats_);
    }
    if (rc != kOk) return rc;
    wseq_ = s;
    SlotHead* sh = slot(s);
    sh->len = len;
    std::memcpy(reinterpret_cast<uint8_t*>(sh) + sizeof(SlotHead), bi.ptr, len);
    sh->pub_ns = now_ns();
    sh->seq.store(s, std::memory_order_release);
    hdr_->pub_gen.fetch_add(1, std::memory_order_seq_cst);
    if (hdr_->sleepers.load(std::memory_order_seq_cst) != 0) futex_wake_all(&hdr_->pub_gen);
    return kOk;
  }

  // Wait for the next message and copy it into `out` (a writable buffer at least as large);
  // returns its length, or -1 timeout, -2 closed by a peer, -3 the writer died.
  int64_t read(py::buffer out, double timeout_s) {
    if (creator_) throw std::runtime_error("shm channel: the creator does not read");
    py::buffer_info bi = out.request(true);
    const size_t cap = (size_t)bi.size * (size_t)bi.itemsize;
    const uint64_t s = rseq_ + 1;
    SlotHead* sh = slot(s);
    const int64_t t_wait = now_ns();
    int rc;
    {
      py::gil_scoped_release nogil;
      auto ready = [&] { return sh->seq.load(std::memory_order_acquire) == s; };
      // a message published just before the close is still delivered
      rc = wait_until(ready, [&] { return closed() && !ready(); }, [&] { return stale(0); }, &hdr_->pub_gen,
                      &hdr_->sleepers, timeout_s, rstats_);
    }
    if (rc != kOk) return rc;
    const size_t len = sh->len;
    if (len > cap) throw std::runtime_error("shm channel: receive buffer too small");
    std::memcpy(bi.ptr, reinterpret_cast<const uint8_t*>(sh) + sizeof(SlotHead), len);
    const int64_t t_got = now_ns();
    const int64_t lat = t_got - sh->pub_ns;
    // wake-up latency: from the later of (message published, reader started waiting) to
    // receipt; the plain publish -> receipt latency also counts time the reader spent busy
    // with the previous step, when the message was already there
    const int64_t wake = t_got - std::max(sh->pub_ns, t_wait);
    rseq_ = s;
    hdr_->done[reader_].store(s, std::memory_order_release);
    hdr_->done_gen.fetch_add(1, std::memory_order_seq_cst);
    if (hdr_->writer_sleeping.load(std::memory_order_seq_cst) != 0) futex_wake_all(&hdr_->done_gen);
    if (lat_.size() < kLatCap) {
      lat_.push_back(lat);
      wake_.push_back(wake);
    } else {
      lat_[lat_n_ % kLatCap] = lat;
      wake_[lat_n_ % kLatCap] = wake;
    }
    ++lat_n_;
    return (int64_t)len;
  }

  // Receive side, over the last messages: publish -> receipt latency (lat_*), wake-up latency
  // (wake_*: from the later of publish and the start of the wait), and how each wait ended
  // (spinning, yielding or after a futex sleep).
  py::dict stats() const {
    py::dict d;
    const WaitStats& w = creator_ ? wstats_ : rstats_;
    d["spins"] = w.spins;
    d["yields"] = w.yields;
    d["sleeps"] = w.sleeps;
    d["messages"] = creator_ ? wseq_ : rseq_;
    if (!creator_ && !lat_.empty()) {
      for (int which = 0; which < 2; ++which) {
        std::vector<int64_t> v(which ? wake_ : lat_);
        std::sort(v.begin(), v.end());
        auto pct = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5))] / 1e3; };
        const std::string k = which ? "wake" : "lat";
        d[(k + "_p50_us").c_str()] = pct(0.5);
        d[(k + "_p99_us").c_str()] = pct(0.99);
        d[(k + "_max_us").c_str()] = v.back() / 1e3;
      }
      d["lat_n"] = (uint64_t)lat_.size();
    }
    return d;
  }

 private:
  static constexpr size_t kLatCap = 1 << 16;

  SlotHead* slot(uint64_t s) { return reinterpret_cast<SlotHead*>(base_ + sizeof(Header) + (s % hdr_->nslots) * slot_stride_); }

  // participant `i` has stamped before and not within liveness_s
  bool stale(int i) const {
    if (liveness_ns_ <= 0) return false;
    const int64_t b = hdr_->beat[i].load(std::memory_order_acquire);
    return b != 0 && now_ns() - b > liveness_ns_;
  }

  // stamp every kBeatNs until stop_beating() sets the stop word (a futex: it wakes the sleep)
  void beat_loop() {
    while (beat_->stop.load(std::memory_order_acquire) == 0) {
      hdr_->beat[beat_idx_].store(now_ns(), std::memory_order_release);
      futex_wait(&beat_->stop, 0, kBeatNs);
    }
  }

  struct Beat {   // heartbeat thread and its stop word (heap: a forked copy must not destroy it)
    std::atomic<uint32_t> stop{0};
    std::thread th;
  };

  std::string name_;
  bool creator_;
  int64_t reader_;
  int64_t liveness_ns_;
  int beat_idx_ = 0;
  bool unlinked_ = false;
  uint8_t* base_ = nullptr;
  Header* hdr_ = nullptr;
  size_t bytes_ = 0, slot_stride_ = 0;
  uint64_t wseq_ = 0, rseq_ = 0;
  WaitStats wstats_, rstats_;
  std::vector<int64_t> lat_, wake_;
  uint64_t lat_n_ = 0;
  Beat* beat_ = nullptr;
  pid_t owner_pid_ = 0;
};

}  // namespace

void register_shm(py::module_& m) {
  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<const std::string&, bool, int64_t, int64_t, int64_t, int64_t, double>(), py::arg("name"),
           py::arg("create"), py::arg("nslots") = 4, py::arg("slot_bytes") = 1 << 20, py::arg("nreaders") = 1,
           py::arg("reader") = 0, py::arg("liveness_s") = 30.0)
      .def("write", &ShmChannel::write, py::arg("buf"), py::arg("timeout_s") = -1.0)
      .def("read", &ShmChannel::read, py::arg("out"), py::arg("timeout_s") = -1.0)
      .def("unlink", &ShmChannel::unlink)
      .def("close", &ShmChannel::close_channel)
      .def("closed", &ShmChannel::closed)
      .def("attached", &ShmChannel::attached)
      .def("slot_bytes", &ShmChannel::slot_bytes)
      .def("stop_beating", &ShmChannel::stop_beating)
      .def("stats", &ShmChannel::stats);
}
