// External id -> slab row map of the flat vector index (index/flat.py), with tombstoning.
//
// The in-HBM index keeps vectors in one slab and deletes by a -inf row bias; the host needs
// id -> row for deletes / re-adds and the live count. A Python dict fed per id was the
// ingestion bottleneck (a 1M-chunk /documents ingest spent seconds in dict updates and a
// device sync per deleted row); here every operation is one call over a numpy batch:
//
//   add(ids, first_row)      -> rows that the new ids displace (re-added ids: the caller
//                               tombstones those rows on the device in one scatter)
//   add_range(start, stride, n, first_row)   synthetic / striped ids, no array at all
//   remove(ids)              -> rows of the ids that were live (-1 for unknown ids dropped)
//   rows(ids)                -> row per id (-1 if absent)
//   rebuild(ids, live)       after compaction / load: rows are the array positions
//
// Open addressing (linear probing, power-of-two table, backward-shift deletion) keyed by
// the id; no per-entry allocation.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

class IdMap {
 public:
  IdMap() { resize(1024); }

  int64_t size() const { return n_; }
  int64_t max_id() const { return n_ ? max_id_ : -1; }

  py::array_t<int64_t> add(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids, int64_t first_row) {
    auto a = ids.unchecked<1>();
    const int64_t m = a.shape(0);
    reserve(n_ + m);
    std::vector<int64_t> displaced;
    for (int64_t j = 0; j < m; ++j) {
      const int64_t old = put(a(j), first_row + j);
      if (old >= 0) displaced.push_back(old);
    }
    return to_array(displaced);
  }

  // all or nothing: a collision anywhere in the range leaves the map untouched
  void add_range(int64_t start, int64_t stride, int64_t n, int64_t first_row) {
    if (n < 0) throw std::invalid_argument("add_range: negative count");
    for (int64_t j = 0; j < n; ++j) {
      if (find(start + stride * j) >= 0) throw std::invalid_argument("add_range: id already present");
    }
    reserve(n_ + n);
    for (int64_t j = 0; j < n; ++j) put(start + stride * j, first_row + j);
  }

  py::array_t<int64_t> remove(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids) {
    auto a = ids.unchecked<1>();
    std::vector<int64_t> rows;
    rows.reserve(a.shape(0));
    for (int64_t j = 0; j < a.shape(0); ++j) {
      const int64_t r = erase(a(j));
      if (r >= 0) rows.push_back(r);
    }
    return to_array(rows);
  }

  py::array_t<int64_t> rows(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids) const {
    auto a = ids.unchecked<1>();
    py::array_t<int64_t> out(a.shape(0));
    auto o = out.mutable_unchecked<1>();
    for (int64_t j = 0; j < a.shape(0); ++j) o(j) = find(a(j));
    return out;
  }

  // rows are array positions; only positions with live != 0 are mapped
  void rebuild(py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
               py::array_t<uint8_t, py::array::c_style | py::array::forcecast> live) {
    auto a = ids.unchecked<1>();
    auto l = live.unchecked<1>();
    if (l.shape(0) != a.shape(0)) throw std::invalid_argument("rebuild: ids and live differ in length");
    clear();
    reserve(a.shape(0));
    for (int64_t j = 0; j < a.shape(0); ++j)
      if (l(j)) put(a(j), j);
  }

  void clear() {
    std::fill(keys_.begin(), keys_.end(), kEmpty);
    n_ = 0;
    max_id_ = -1;
  }

 private:
  static constexpr int64_t kEmpty = INT64_MIN;

  static uint64_t hash(int64_t k) {
    uint64_t z = (uint64_t)k + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }

  void resize(size_t cap) {
    std::vector<int64_t> ok = std::move(keys_), ov = std::move(vals_);
    keys_.assign(cap, kEmpty);
    vals_.assign(cap, -1);
    mask_ = cap - 1;
    n_ = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] != kEmpty) put(ok[i], ov[i]);
  }

  void reserve(int64_t n) {
    size_t cap = keys_.size();
    while ((int64_t)(cap * 7 / 10) < n) cap *= 2;
    if (cap != keys_.size()) resize(cap);
  }

  // insert or overwrite; returns the previous row (-1 if new)
  int64_t put(int64_t k, int64_t v) {
    if (k == kEmpty) throw std::invalid_argument("IdMap: id INT64_MIN is reserved");
    if ((int64_t)((keys_.size() * 7) / 10) <= n_) resize(keys_.size() * 2);
    size_t i = hash(k) & mask_;
    while (keys_[i] != kEmpty) {
      if (keys_[i] == k) {
        const int64_t old = vals_[i];
        vals_[i] = v;
        return old;
      }
      i = (i + 1) & mask_;
    }
    keys_[i] = k;
    vals_[i] = v;
    ++n_;
    if (k > max_id_ || n_ == 1) max_id_ = k;
    return -1;
  }

  int64_t find(int64_t k) const {
    size_t i = hash(k) & mask_;
    while (keys_[i] != kEmpty) {
      if (keys_[i] == k) return vals_[i];
      i = (i + 1) & mask_;
    }
    return -1;
  }

  // backward-shift deletion keeps probe chains intact without tombstones
  int64_t erase(int64_t k) {
    size_t i = hash(k) & mask_;
    while (keys_[i] != kEmpty && keys_[i] != k) i = (i + 1) & mask_;
    if (keys_[i] == kEmpty) return -1;
    const int64_t v = vals_[i];
    size_t j = i;
    for (;;) {
      j = (j + 1) & mask_;
      if (keys_[j] == kEmpty) break;
      const size_t h = hash(keys_[j]) & mask_;
      // move keys_[j] back to i when its home slot h is not in (i, j] (cyclically)
      const bool in_range = i <= j ? (i < h && h <= j) : (i < h || h <= j);
      if (!in_range) {
        keys_[i] = keys_[j];
        vals_[i] = vals_[j];
        i = j;
      }
    }
    keys_[i] = kEmpty;
    vals_[i] = -1;
    --n_;
    // max_id_ stays an upper bound after deletes (the index only uses it to pick fresh ids)
    return v;
  }

  static py::array_t<int64_t> to_array(const std::vector<int64_t>& v) {
    py::array_t<int64_t> out((py::ssize_t)v.size());
    std::copy(v.begin(), v.end(), out.mutable_data());
    return out;
  }

  std::vector<int64_t> keys_, vals_;
  size_t mask_ = 0;
  int64_t n_ = 0;
  int64_t max_id_ = -1;
};

}  // namespace

void register_idmap(py::module_& m) {
  py::class_<IdMap>(m, "IdMap")
      .def(py::init<>())
      .def("__len__", &IdMap::size)
      .def("max_id", &IdMap::max_id)
      .def("add", &IdMap::add, py::arg("ids"), py::arg("first_row"))
      .def("add_range", &IdMap::add_range, py::arg("start"), py::arg("stride"), py::arg("n"), py::arg("first_row"))
      .def("remove", &IdMap::remove, py::arg("ids"))
      .def("rows", &IdMap::rows, py::arg("ids"))
      .def("rebuild", &IdMap::rebuild, py::arg("ids"), py::arg("live"))
      .def("clear", &IdMap::clear);
}
