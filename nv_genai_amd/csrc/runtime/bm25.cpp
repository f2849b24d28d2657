// Okapi-BM25 keyword index (N5 in SURVEY.md §2.B): the sparse half of the NeMo Retriever
// `hybrid` / `ranked_hybrid` pipelines (Elasticsearch BM25, sparse top-k 100 —
// experimental/fm-asr-streaming-rag/deploy/docker-compose-nemo-retriever.yaml:39-66) and of
// the knowledge-graph example's dense+sparse RRF search (knowledge_graph_rag/vectorstore/
// search.py:51-87). Host-side C++: an inverted index with per-term postings, lazy deletes,
// and a bounded heap for top-k.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <queue>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace {

std::vector<std::string> tokenize(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c >= 0x80) {
      cur.push_back((char)std::tolower(c));
    } else if (!cur.empty()) {
      out.push_back(cur);
      cur.clear();
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

class BM25Index {
 public:
  BM25Index(double k1, double b) : k1_(k1), b_(b) {}

  void add(int64_t doc, const std::string& text) {
    if (len_.count(doc)) remove(doc);
    auto toks = tokenize(text);
    std::unordered_map<std::string, int> tf;
    for (auto& t : toks) tf[t]++;
    for (auto& kv : tf) {
      auto& plist = post_[kv.first];
      plist.push_back({doc, kv.second});
      df_[kv.first]++;
    }
    len_[doc] = (int)toks.size();
    terms_[doc].reserve(tf.size());
    for (auto& kv : tf) terms_[doc].push_back(kv.first);
    total_len_ += (int64_t)toks.size();
  }

  void remove(int64_t doc) {
    auto it = len_.find(doc);
    if (it == len_.end()) return;
    total_len_ -= it->second;
    for (auto& t : terms_[doc]) {
      auto& plist = post_[t];
      plist.erase(std::remove_if(plist.begin(), plist.end(),
                                 [&](const Posting& p) { return p.doc == doc; }),
                  plist.end());
      if (--df_[t] <= 0) {
        df_.erase(t);
        post_.erase(t);
      }
    }
    terms_.erase(doc);
    len_.erase(it);
  }

  std::vector<std::pair<int64_t, double>> search(const std::string& q, int k) const {
    std::vector<std::pair<int64_t, double>> res;
    const double N = (double)len_.size();
    if (N == 0 || k <= 0) return res;
    const double avgdl = (double)total_len_ / N;
    std::unordered_map<int64_t, double> acc;
    std::unordered_set<std::string> seen;
    for (auto& t : tokenize(q)) {
      if (!seen.insert(t).second) continue;
      auto it = post_.find(t);
      if (it == post_.end()) continue;
      const double n = (double)it->second.size();
      const double idf = std::log(1.0 + (N - n + 0.5) / (n + 0.5));
      for (const auto& p : it->second) {
        const double dl = (double)len_.at(p.doc);
        const double tf = (double)p.tf;
        acc[p.doc] += idf * tf * (k1_ + 1.0) / (tf + k1_ * (1.0 - b_ + b_ * dl / avgdl));
      }
    }
    using E = std::pair<double, int64_t>;
    std::priority_queue<E, std::vector<E>, std::greater<E>> heap;
    for (auto& kv : acc) {
      if ((int)heap.size() < k) {
        heap.push({kv.second, kv.first});
      } else if (kv.second > heap.top().first) {
        heap.pop();
        heap.push({kv.second, kv.first});
      }
    }
    while (!heap.empty()) {
      res.push_back({heap.top().second, heap.top().first});
      heap.pop();
    }
    std::reverse(res.begin(), res.end());
    return res;
  }

  size_t size() const { return len_.size(); }

 private:
  struct Posting {
    int64_t doc;
    int tf;
  };
  double k1_, b_;
  std::unordered_map<std::string, std::vector<Posting>> post_;
  std::unordered_map<std::string, int> df_;
  std::unordered_map<int64_t, int> len_;
  std::unordered_map<int64_t, std::vector<std::string>> terms_;
  int64_t total_len_ = 0;
};

}  // namespace

void register_bm25(py::module_& m) {
  py::class_<BM25Index>(m, "BM25Index")
      .def(py::init<double, double>(), py::arg("k1") = 1.2, py::arg("b") = 0.75)
      .def("add", &BM25Index::add)
      .def("remove", &BM25Index::remove)
      .def("search", &BM25Index::search, py::call_guard<py::gil_scoped_release>())
      .def("__len__", &BM25Index::size);
  m.def("bm25_tokenize", &tokenize);
}
