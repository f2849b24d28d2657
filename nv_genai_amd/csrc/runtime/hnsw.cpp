// HNSW graph index (host side) — the Milvus ``index_type: HNSW`` (M, efConstruction) of the
// reference's streaming-ingest collections
// (experimental/streaming_ingest_rag/morpheus_examples/streaming_ingest_rag/vdb_upload/kafka_config.yaml:112-122;
// SURVEY.md §2.B N4). On MI355X the batched, throughput path is the in-HBM flat / IVF scan
// (csrc/kernels/vector_search.hip); a proximity graph is the low-latency path for single queries
// on the host (no kernel launch, no PCIe round trip) and for collections configured as HNSW.
//
// Layout: vectors in one contiguous float32 array (row = internal node id); level-0 neighbour
// lists in one flat int32 array of capacity 2M per node (the hot layer: contiguous, no
// pointer chasing), upper-level lists per node in a small vector of arrays of capacity M.
// Insertion follows Malkov & Yashunin (greedy descent, ef-construction beam per layer, the
// diversity heuristic for neighbour selection and for shrinking overfull lists). Deletion
// marks a tombstone: deleted nodes still route the search but are never returned.
// Concurrency: a shared mutex — searches run in parallel (GIL released, batched queries are
// split over threads), adds take it exclusively; inside an add the batch is linked by worker
// threads with striped per-node locks on the link lists (vectors, levels and storage are laid
// out for the whole batch first, so nothing reallocates while the graph grows).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <mutex>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <queue>
#include <random>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

enum class Metric { L2, IP, COSINE };

Metric parse_metric(const std::string& m) {
  if (m == "l2" || m == "L2") return Metric::L2;
  if (m == "ip" || m == "IP") return Metric::IP;
  if (m == "cosine" || m == "COSINE") return Metric::COSINE;
  throw std::invalid_argument("metric must be l2, ip or cosine");
}

inline float dot(const float* a, const float* b, int d) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = 0;
  for (; i + 4 <= d; i += 4) {
    s0 += a[i] * b[i];
    s1 += a[i + 1] * b[i + 1];
    s2 += a[i + 2] * b[i + 2];
    s3 += a[i + 3] * b[i + 3];
  }
  for (; i < d; ++i) s0 += a[i] * b[i];
  return (s0 + s1) + (s2 + s3);
}

inline float l2sq(const float* a, const float* b, int d) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = 0;
  for (; i + 4 <= d; i += 4) {
    float e0 = a[i] - b[i], e1 = a[i + 1] - b[i + 1], e2 = a[i + 2] - b[i + 2], e3 = a[i + 3] - b[i + 3];
    s0 += e0 * e0;
    s1 += e1 * e1;
    s2 += e2 * e2;
    s3 += e3 * e3;
  }
  for (; i < d; ++i) {
    float e = a[i] - b[i];
    s0 += e * e;
  }
  return (s0 + s1) + (s2 + s3);
}

using Cand = std::pair<float, int32_t>;  // (distance, node); smaller distance = closer
constexpr int kMaxLinks = 2 * 512 + 1;   // level-0 capacity 2M for M up to 512

class HNSW {
 public:
  HNSW(int dim, const std::string& metric, int M, int ef_construction, int ef_search, uint64_t seed)
      : d_(dim), metric_(parse_metric(metric)), M_(std::min(512, std::max(2, M))),
        M0_(2 * std::min(512, std::max(2, M))),
        efc_(std::max(ef_construction, M)), ef_(std::max(1, ef_search)), rng_(seed),
        ml_(1.0 / std::log(double(std::max(2, M)))) {
    if (dim <= 0) throw std::invalid_argument("dim must be positive");
  }

  int64_t size() const { return (int64_t)ext_.size() - n_deleted_; }
  int dim() const { return d_; }
  int max_level() const { return max_level_; }
  void set_ef(int ef) { ef_ = std::max(1, ef); }
  int ef() const { return ef_; }

  void add(py::array_t<float, py::array::c_style | py::array::forcecast> vecs,
           py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids, int threads) {
    auto v = vecs.unchecked<2>();
    auto id = ids.unchecked<1>();
    if (v.shape(1) != d_) throw std::invalid_argument("vector dim mismatch");
    if (v.shape(0) != id.shape(0)) throw std::invalid_argument("vecs / ids length mismatch");
    const int64_t n = v.shape(0);
    py::gil_scoped_release nogil;
    std::unique_lock<std::shared_mutex> lk(mu_);
    // 1. sequential: ids, levels and storage for the whole batch (nothing reallocates while
    //    the batch is being linked)
    for (int64_t r = 0; r < n; ++r) {
      if (int_.count(id(r))) {
        for (int64_t u = 0; u < r; ++u) int_.erase(id(u));   // leave the index unchanged
        throw std::invalid_argument("duplicate id " + std::to_string(id(r)));
      }
      int_[id(r)] = (int32_t)(ext_.size() + r);
    }
    const int32_t first = (int32_t)ext_.size();
    std::uniform_real_distribution<double> U(std::numeric_limits<double>::min(), 1.0);
    data_.resize(data_.size() + (size_t)n * d_);
    l0_.resize(l0_.size() + (size_t)n * (M0_ + 1), 0);
    for (int64_t r = 0; r < n; ++r) {
      const int32_t me = first + (int32_t)r;
      float* x = &data_[(size_t)me * d_];
      for (int j = 0; j < d_; ++j) x[j] = v(r, j);
      normalise(x);
      const int lvl = std::min(32, (int)std::floor(-std::log(U(rng_)) * ml_));
      ext_.push_back(id(r));
      deleted_.push_back(0);
      level_.push_back(lvl);
      up_.emplace_back(lvl);
      for (int l = 1; l <= lvl; ++l) up_[me][l - 1].assign(M_ + 1, 0);
    }
    // 2. link: the first node of an empty graph becomes the entry point, then the batch is
    //    inserted by ``threads`` workers (per-node striped locks guard the link lists)
    int32_t start = first;
    if (entry_ < 0 && n > 0) {
      entry_ = first;
      max_level_ = level_[first];
      start = first + 1;
    }
    const int32_t end = first + (int32_t)n;
    const int T = std::max(1, std::min<int>(threads, (int)((end - start + 63) / 64)));
    if (T == 1) {
      for (int32_t me = start; me < end; ++me) link(me);
    } else {
      std::atomic<int32_t> next(start);
      std::vector<std::thread> pool;
      for (int t = 0; t < T; ++t)
        pool.emplace_back([&] {
          for (int32_t me = next.fetch_add(1); me < end; me = next.fetch_add(1)) link(me);
        });
      for (auto& th : pool) th.join();
    }
  }

  int64_t remove(const std::vector<int64_t>& ids) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    int64_t k = 0;
    for (int64_t e : ids) {
      auto it = int_.find(e);
      if (it == int_.end() || deleted_[it->second]) continue;
      deleted_[it->second] = 1;
      int_.erase(it);
      ++n_deleted_;
      ++k;
    }
    return k;
  }

  // -> (scores [q, k], ids [q, k]); scores: -squared L2, or the inner product (cosine: of the
  // normalised vectors); missing results are (-inf, -1)
  py::tuple search(py::array_t<float, py::array::c_style | py::array::forcecast> qs, int k, int ef, int threads) {
    auto q = qs.unchecked<2>();
    if (q.shape(1) != d_) throw std::invalid_argument("query dim mismatch");
    const int64_t nq = q.shape(0);
    k = std::max(k, 0);
    std::vector<py::ssize_t> shape{(py::ssize_t)nq, (py::ssize_t)k};
    py::array_t<float> scores(shape);
    py::array_t<int64_t> out(shape);
    float* S = scores.mutable_data();
    int64_t* I = out.mutable_data();
    const float* Q = qs.data();
    const int efq = std::max(ef > 0 ? ef : ef_, k);
    {
      py::gil_scoped_release nogil;
      std::shared_lock<std::shared_mutex> lk(mu_);
      auto work = [&](int64_t b, int64_t e) {
        std::vector<float> qb(d_);
        for (int64_t i = b; i < e; ++i) search_one(Q + i * d_, k, efq, qb.data(), S + i * k, I + i * k);
      };
      int T = std::max(1, std::min<int>(threads, (int)((nq + 7) / 8)));
      if (T == 1) {
        work(0, nq);
      } else {
        std::vector<std::thread> pool;
        int64_t per = (nq + T - 1) / T;
        for (int t = 0; t < T; ++t) {
          int64_t b = t * per, e = std::min(nq, b + per);
          if (b < e) pool.emplace_back(work, b, e);
        }
        for (auto& th : pool) th.join();
      }
    }
    return py::make_tuple(scores, out);
  }

  void save(const std::string& path) const {
    std::shared_lock<std::shared_mutex> lk(mu_);
    std::ofstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot write " + path);
    const char magic[8] = {'N', 'G', 'A', 'H', 'N', 'S', 'W', '1'};
    f.write(magic, 8);
    int32_t hdr[7] = {d_, (int32_t)metric_, M_, efc_, ef_, entry_, max_level_};
    f.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
    int64_t n = (int64_t)ext_.size();
    f.write(reinterpret_cast<const char*>(&n), sizeof(n));
    f.write(reinterpret_cast<const char*>(data_.data()), sizeof(float) * data_.size());
    f.write(reinterpret_cast<const char*>(ext_.data()), sizeof(int64_t) * ext_.size());
    f.write(reinterpret_cast<const char*>(deleted_.data()), deleted_.size());
    f.write(reinterpret_cast<const char*>(level_.data()), sizeof(int32_t) * level_.size());
    f.write(reinterpret_cast<const char*>(l0_.data()), sizeof(int32_t) * l0_.size());
    for (int64_t i = 0; i < n; ++i)
      for (int l = 1; l <= level_[i]; ++l)
        f.write(reinterpret_cast<const char*>(up_[i][l - 1].data()), sizeof(int32_t) * (M_ + 1));
    if (!f) throw std::runtime_error("short write to " + path);
  }

  static std::unique_ptr<HNSW> load(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot read " + path);
    char magic[8];
    f.read(magic, 8);
    if (std::string(magic, 8) != "NGAHNSW1") throw std::runtime_error("not an HNSW index file: " + path);
    int32_t hdr[7];
    f.read(reinterpret_cast<char*>(hdr), sizeof(hdr));
    const char* names[3] = {"l2", "ip", "cosine"};
    if (hdr[1] < 0 || hdr[1] > 2) throw std::runtime_error("corrupt HNSW header");
    auto hp = std::make_unique<HNSW>(hdr[0], names[hdr[1]], hdr[2], hdr[3], hdr[4], 0);
    HNSW& h = *hp;
    h.entry_ = hdr[5];
    h.max_level_ = hdr[6];
    int64_t n = 0;
    f.read(reinterpret_cast<char*>(&n), sizeof(n));
    if (n < 0 || n > (int64_t(1) << 34)) throw std::runtime_error("corrupt HNSW size");
    h.data_.resize((size_t)n * h.d_);
    h.ext_.resize(n);
    h.deleted_.resize(n);
    h.level_.resize(n);
    h.l0_.resize((size_t)n * (h.M0_ + 1));
    f.read(reinterpret_cast<char*>(h.data_.data()), sizeof(float) * h.data_.size());
    f.read(reinterpret_cast<char*>(h.ext_.data()), sizeof(int64_t) * n);
    f.read(reinterpret_cast<char*>(h.deleted_.data()), n);
    f.read(reinterpret_cast<char*>(h.level_.data()), sizeof(int32_t) * n);
    f.read(reinterpret_cast<char*>(h.l0_.data()), sizeof(int32_t) * h.l0_.size());
    h.up_.resize(n);
    for (int64_t i = 0; i < n; ++i) {
      if (h.level_[i] < 0 || h.level_[i] > 64) throw std::runtime_error("corrupt HNSW level");
      h.up_[i].resize(h.level_[i]);
      for (int l = 1; l <= h.level_[i]; ++l) {
        h.up_[i][l - 1].resize(h.M_ + 1);
        f.read(reinterpret_cast<char*>(h.up_[i][l - 1].data()), sizeof(int32_t) * (h.M_ + 1));
      }
    }
    if (!f) throw std::runtime_error("truncated HNSW index file: " + path);
    h.validate(path);
    for (int64_t i = 0; i < n; ++i) {
      if (h.deleted_[i]) ++h.n_deleted_;
      else h.int_[h.ext_[i]] = (int32_t)i;
    }
    return hp;
  }

 private:
  // a loaded graph is trusted by search (no bounds checks on the hot path): every list count
  // must fit its capacity, every neighbour id must name a node, and the entry point must be a
  // node whose level is the graph's top level
  void validate(const std::string& path) const {
    const int64_t n = (int64_t)ext_.size();
    auto bad = [&](const char* what) { throw std::runtime_error(std::string("corrupt HNSW graph (") + what + "): " + path); };
    if (entry_ < -1 || entry_ >= n) bad("entry point");
    if (entry_ < 0 ? (max_level_ != -1 || n != 0) : (max_level_ < 0 || max_level_ != level_[entry_])) bad("top level");
    if (M0_ + 1 > kMaxLinks || M_ + 1 > kMaxLinks) bad("link capacity");
    for (int64_t i = 0; i < n; ++i) {
      if (deleted_[i] > 1) bad("tombstone flag");
      for (int l = 0; l <= level_[i]; ++l) {
        const int32_t* ln = links((int32_t)i, l);
        const int cap = l == 0 ? M0_ : M_;
        if (ln[0] < 0 || ln[0] > cap) bad("link count");
        for (int j = 1; j <= ln[0]; ++j)
          if (ln[j] < 0 || ln[j] >= n) bad("neighbour id");
      }
    }
  }

  // visit marks of one search / link: a tag per node, bumped per layer search so the array
  // is cleared only when the tag wraps. Buffers are owned by the index and reused across
  // calls and threads (a fresh 2 x N array per thread per call dominated batched queries).
  struct Visit {
    std::vector<uint32_t> seen;
    uint32_t tag = 0;
  };
  struct VisitLease {
    const HNSW* h;
    std::unique_ptr<Visit> v;
    ~VisitLease() { h->release_visit(std::move(v)); }
  };
  VisitLease lease_visit() const {
    std::unique_ptr<Visit> v;
    {
      std::lock_guard<std::mutex> g(visit_mu_);
      if (!visit_pool_.empty()) {
        v = std::move(visit_pool_.back());
        visit_pool_.pop_back();
      }
    }
    if (!v) v = std::make_unique<Visit>();
    if (v->seen.size() < ext_.size()) {
      v->seen.assign(ext_.size() + ext_.size() / 2 + 1024, 0);
      v->tag = 0;
    }
    return VisitLease{this, std::move(v)};
  }
  void release_visit(std::unique_ptr<Visit> v) const {
    if (!v) return;
    std::lock_guard<std::mutex> g(visit_mu_);
    visit_pool_.push_back(std::move(v));
  }

  // neighbour list of node i at level l: [count, n_0, n_1, ...]
  int32_t* links(int32_t i, int l) {
    return l == 0 ? &l0_[(size_t)i * (M0_ + 1)] : up_[i][l - 1].data();
  }
  const int32_t* links(int32_t i, int l) const {
    return l == 0 ? &l0_[(size_t)i * (M0_ + 1)] : up_[i][l - 1].data();
  }
  const float* vec(int32_t i) const { return &data_[(size_t)i * d_]; }

  float dist(const float* a, const float* b) const {
    return metric_ == Metric::L2 ? l2sq(a, b, d_) : -dot(a, b, d_);
  }

  void normalise(float* v) const {
    if (metric_ != Metric::COSINE) return;
    float n = std::sqrt(dot(v, v, d_));
    if (n > 0.f)
      for (int j = 0; j < d_; ++j) v[j] /= n;
  }

  // beam search of one layer from ``ep``; returns up to ef closest (max-heap order undone)
  // copy of node i's level-l list (under its stripe lock while the graph is being linked)
  template <bool LOCK>
  int read_links(int32_t i, int l, int32_t* out) const {
    if (LOCK) {
      std::lock_guard<std::mutex> g(stripe(i));
      const int32_t* ln = links(i, l);
      std::memcpy(out, ln + 1, sizeof(int32_t) * ln[0]);
      return ln[0];
    }
    const int32_t* ln = links(i, l);
    std::memcpy(out, ln + 1, sizeof(int32_t) * ln[0]);
    return ln[0];
  }

  template <bool LOCK = false>
  std::vector<Cand> search_layer(const float* q, int32_t ep, int ef, int l, std::vector<uint32_t>& seen,
                                 uint32_t& tag) const {
    if (++tag == 0) {  // wrapped: reset the visit marks
      std::fill(seen.begin(), seen.end(), 0);
      tag = 1;
    }
    std::priority_queue<Cand, std::vector<Cand>, std::greater<Cand>> cand;  // min-heap
    std::priority_queue<Cand> best;                                          // max-heap
    float d0 = dist(q, vec(ep));
    cand.emplace(d0, ep);
    best.emplace(d0, ep);
    seen[ep] = tag;
    while (!cand.empty()) {
      Cand c = cand.top();
      if (c.first > best.top().first && (int)best.size() >= ef) break;
      cand.pop();
      int32_t nb[kMaxLinks];
      const int cnt = read_links<LOCK>(c.second, l, nb);
      for (int j = 0; j < cnt; ++j) {
        int32_t u = nb[j];
        if (seen[u] == tag) continue;
        seen[u] = tag;
        float du = dist(q, vec(u));
        if ((int)best.size() < ef || du < best.top().first) {
          cand.emplace(du, u);
          best.emplace(du, u);
          if ((int)best.size() > ef) best.pop();
        }
      }
    }
    std::vector<Cand> out;
    out.reserve(best.size());
    while (!best.empty()) {
      out.push_back(best.top());
      best.pop();
    }
    std::reverse(out.begin(), out.end());
    return out;
  }

  // Malkov & Yashunin's heuristic: keep a candidate only if it is closer to the base than to
  // every neighbour already kept (spreads the links over directions); sorted input
  std::vector<int32_t> select(const std::vector<Cand>& sorted, int m) const {
    std::vector<int32_t> keep;
    for (const Cand& c : sorted) {
      if ((int)keep.size() >= m) break;
      bool good = true;
      for (int32_t k : keep)
        if (dist(vec(c.second), vec(k)) < c.first) {
          good = false;
          break;
        }
      if (good) keep.push_back(c.second);
    }
    return keep;
  }

  void connect(int32_t a, int32_t b, int l) {
    std::lock_guard<std::mutex> g(stripe(a));
    int32_t* ln = links(a, l);
    const int cap = l == 0 ? M0_ : M_;
    if (ln[0] < cap) {
      ln[++ln[0]] = b;
      return;
    }
    std::vector<Cand> cs;
    cs.reserve(cap + 1);
    const float* va = vec(a);
    for (int j = 1; j <= ln[0]; ++j) cs.emplace_back(dist(va, vec(ln[j])), ln[j]);
    cs.emplace_back(dist(va, vec(b)), b);
    std::sort(cs.begin(), cs.end());
    std::vector<int32_t> keep = select(cs, cap);
    ln[0] = (int32_t)keep.size();
    for (size_t j = 0; j < keep.size(); ++j) ln[j + 1] = keep[j];
  }

  // graph insertion of node ``me`` (vector, level and storage already in place); safe to run
  // for several nodes at once
  void link(int32_t me) {
    const int lvl = level_[me];
    int32_t ep;
    int top;
    {
      std::lock_guard<std::mutex> g(entry_mu_);
      ep = entry_;
      top = max_level_;
    }
    VisitLease vis = lease_visit();
    std::vector<uint32_t>& seen = vis.v->seen;
    uint32_t& tag = vis.v->tag;
    const float* q = vec(me);
    int32_t nb[kMaxLinks];
    for (int l = top; l > lvl; --l) {  // greedy descent
      bool moved = true;
      float de = dist(q, vec(ep));
      while (moved) {
        moved = false;
        const int cnt = read_links<true>(ep, l, nb);
        for (int j = 0; j < cnt; ++j) {
          float du = dist(q, vec(nb[j]));
          if (du < de) {
            de = du;
            ep = nb[j];
            moved = true;
          }
        }
      }
    }
    for (int l = std::min(lvl, top); l >= 0; --l) {
      std::vector<Cand> w = search_layer<true>(q, ep, efc_, l, seen, tag);
      std::vector<int32_t> sel = select(w, l == 0 ? M0_ : M_);
      {
        std::lock_guard<std::mutex> g(stripe(me));
        int32_t* ln = links(me, l);
        ln[0] = (int32_t)sel.size();
        for (size_t j = 0; j < sel.size(); ++j) ln[j + 1] = sel[j];
      }
      for (int32_t u : sel) connect(u, me, l);
      ep = w.front().second;
    }
    if (lvl > top) {
      std::lock_guard<std::mutex> g(entry_mu_);
      if (lvl > max_level_) {
        max_level_ = lvl;
        entry_ = me;
      }
    }
  }

  void search_one(const float* q0, int k, int ef, float* qb, float* S, int64_t* I) const {
    for (int j = 0; j < k; ++j) {
      S[j] = -std::numeric_limits<float>::infinity();
      I[j] = -1;
    }
    if (entry_ < 0 || k == 0) return;
    std::memcpy(qb, q0, sizeof(float) * d_);
    normalise(qb);
    int32_t ep = entry_;
    float de = dist(qb, vec(ep));
    for (int l = max_level_; l > 0; --l) {
      bool moved = true;
      while (moved) {
        moved = false;
        const int32_t* ln = links(ep, l);
        for (int j = 1; j <= ln[0]; ++j) {
          float du = dist(qb, vec(ln[j]));
          if (du < de) {
            de = du;
            ep = ln[j];
            moved = true;
          }
        }
      }
    }
    // visit marks leased from the index's pool (searches run concurrently)
    VisitLease vis = lease_visit();
    std::vector<uint32_t>& seen = vis.v->seen;
    uint32_t& tag = vis.v->tag;
    // tombstones still route; widen the beam by the deleted share so k live results survive
    int efd = ef + (int)std::min<int64_t>(n_deleted_, ef);
    std::vector<Cand> w = search_layer(qb, ep, efd, 0, seen, tag);
    int j = 0;
    for (const Cand& c : w) {
      if (j >= k) break;
      if (deleted_[c.second]) continue;
      S[j] = -c.first;  // -L2^2, or the dot product (cosine: of the normalised vectors)
      I[j] = ext_[c.second];
      ++j;
    }
  }

  int d_;
  Metric metric_;
  int M_, M0_, efc_, ef_;
  std::mt19937_64 rng_;
  double ml_;
  int32_t entry_ = -1;
  int max_level_ = -1;
  std::vector<float> data_;
  std::vector<int64_t> ext_;
  std::vector<uint8_t> deleted_;
  std::vector<int32_t> level_;
  std::vector<int32_t> l0_;
  std::vector<std::vector<std::vector<int32_t>>> up_;
  std::unordered_map<int64_t, int32_t> int_;
  int64_t n_deleted_ = 0;
  mutable std::shared_mutex mu_;                 // searches shared, adds exclusive
  std::mutex entry_mu_;                          // entry point / top level during a batch link
  mutable std::array<std::mutex, 4096> stripes_; // link-list locks, striped by node id
  mutable std::mutex visit_mu_;                  // guards visit_pool_
  mutable std::vector<std::unique_ptr<Visit>> visit_pool_;
  std::mutex& stripe(int32_t i) const { return stripes_[(uint32_t)i & 4095u]; }
};

}  // namespace

void register_hnsw(py::module_& m) {
  py::class_<HNSW>(m, "HNSW")
      .def(py::init<int, const std::string&, int, int, int, uint64_t>(), py::arg("dim"),
           py::arg("metric") = "l2", py::arg("M") = 16, py::arg("ef_construction") = 200,
           py::arg("ef_search") = 64, py::arg("seed") = 100)
      .def("add", &HNSW::add, py::arg("vecs"), py::arg("ids"), py::arg("threads") = 1)
      .def("remove", &HNSW::remove)
      .def("search", &HNSW::search, py::arg("queries"), py::arg("k"), py::arg("ef") = 0,
           py::arg("threads") = 1)
      .def("save", &HNSW::save, py::call_guard<py::gil_scoped_release>())
      .def_static("load", &HNSW::load)
      .def_property("ef", &HNSW::ef, &HNSW::set_ef)
      .def_property_readonly("dim", &HNSW::dim)
      .def_property_readonly("max_level", &HNSW::max_level)
      .def("__len__", &HNSW::size);
}
