// Text chunking for ingestion (N11 in SURVEY.md §2.B):
//  * token windows with overlap (SentenceTransformersTokenTextSplitter semantics: windows of
//    tokens_per_chunk tokens advancing by tokens_per_chunk - overlap —
//    RetrievalAugmentedGeneration/common/utils.py:321-331);
//  * recursive character splitting (separator hierarchy "\n\n", "\n", " ", "" with chunk
//    size / overlap in characters — the 1000/100 splitter of
//    examples/multimodal_rag/vectorstore/vectorstore_updater.py:49-59).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <string>
#include <vector>

namespace py = pybind11;

namespace {

std::vector<std::pair<int, int>> token_windows(int n_tokens, int chunk, int overlap) {
  std::vector<std::pair<int, int>> out;
  if (chunk <= 0) return out;
  if (overlap >= chunk) overlap = chunk - 1;
  const int step = chunk - overlap;
  for (int s = 0; s < n_tokens; s += step) {
    const int e = std::min(n_tokens, s + chunk);
    out.push_back({s, e});
    if (e == n_tokens) break;
  }
  return out;
}

void split_rec(const std::string& text, const std::vector<std::string>& seps, size_t sep_i,
               std::vector<std::string>& pieces, size_t chunk) {
  if (text.size() <= chunk) {
    if (!text.empty()) pieces.push_back(text);
    return;
  }
  if (sep_i >= seps.size() || seps[sep_i].empty()) {
    for (size_t i = 0; i < text.size(); i += chunk) pieces.push_back(text.substr(i, chunk));
    return;
  }
  const std::string& sep = seps[sep_i];
  size_t start = 0;
  while (start <= text.size()) {
    size_t p = text.find(sep, start);
    std::string part = text.substr(start, p == std::string::npos ? std::string::npos : p - start);
    if (p != std::string::npos) part += sep;  // keep the separator with the left piece
    if (!part.empty()) {
      if (part.size() > chunk)
        split_rec(part, seps, sep_i + 1, pieces, chunk);
      else
        pieces.push_back(part);
    }
    if (p == std::string::npos) break;
    start = p + sep.size();
  }
}

// Greedy merge of pieces into chunks of <= chunk chars with ~overlap chars carried over.
std::vector<std::string> char_split(const std::string& text, int chunk, int overlap,
                                    std::vector<std::string> seps) {
  if (seps.empty()) seps = {"\n\n", "\n", " ", ""};
  std::vector<std::string> pieces;
  split_rec(text, seps, 0, pieces, (size_t)chunk);
  std::vector<std::string> out;
  std::vector<std::string> cur;
  size_t cur_len = 0;
  auto flush = [&]() {
    std::string s;
    for (auto& p : cur) s += p;
    // strip
    size_t a = s.find_first_not_of(" \n\t\r"), b = s.find_last_not_of(" \n\t\r");
    if (a != std::string::npos) out.push_back(s.substr(a, b - a + 1));
  };
  for (auto& p : pieces) {
    if (cur_len + p.size() > (size_t)chunk && !cur.empty()) {
      flush();
      while (!cur.empty() && (cur_len > (size_t)overlap || cur_len + p.size() > (size_t)chunk)) {
        cur_len -= cur.front().size();
        cur.erase(cur.begin());
      }
    }
    cur.push_back(p);
    cur_len += p.size();
  }
  if (!cur.empty()) flush();
  return out;
}

}  // namespace

void register_text(py::module_& m) {
  m.def("token_windows", &token_windows, py::arg("n_tokens"), py::arg("chunk"),
        py::arg("overlap"));
  m.def("char_split", &char_split, py::arg("text"), py::arg("chunk_size"), py::arg("overlap"),
        py::arg("separators") = std::vector<std::string>{});
}
