// JSON-constrained decoding (SURVEY.md §2.G "structured LLM output + repair": the reference
// repairs model JSON after the fact — experimental/fm-asr-streaming-rag/chain-server/
// utils.py:41-95, query_decomposition_rag/chains.py:162,367-369; the engine here makes the
// output valid by construction, OpenAI ``response_format={"type": "json_object"}``).
//
// A byte-level pushdown automaton over JSON text. For a sequence's state the grammar fills an
// allowed-token mask over the tokenizer vocabulary: a token is allowed iff every byte of its
// text is accepted from the current state (tokens are walked on a copy of the state, which
// is a fixed-size POD so the copy is a memcpy). Stop tokens are allowed exactly when the
// top-level object is complete. The engine applies the mask to the logits (-inf) before the
// sampling kernel, so temperature / top-k / top-p keep their meaning on the allowed set.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

enum Mode : uint8_t {
  VALUE, ARR_FIRST, OBJ_FIRST, OBJ_KEY, COLON, AFTER, STRING, ESC, UNI, NUMBER, LITERAL, DONE
};
enum Num : uint8_t { N_SIGN, N_ZERO, N_INT, N_FRAC0, N_FRAC, N_EXP0, N_EXPS, N_EXP };
constexpr int kMaxDepth = 48;
constexpr int kMaxWs = 3;  // consecutive whitespace bytes: no endless-blank generations
const char* kLit[3] = {"true", "false", "null"};

struct JsonState {
  char stack[kMaxDepth];
  int8_t depth = 0;
  uint8_t mode = VALUE;
  uint8_t sub = 0;   // number substate / literal index / unicode digit count
  uint8_t lit = 0;
  uint8_t ws = 0;
  bool key = false;
  bool object_only = true;

  bool done() const { return mode == DONE; }

  static bool is_ws(unsigned c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r'; }
  static bool is_hex(unsigned c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
  }

  bool blank(unsigned c) {
    if (!is_ws(c)) {
      ws = 0;
      return false;
    }
    return ++ws <= kMaxWs;
  }

  bool begin_value(unsigned c) {
    if (depth == 0 && object_only && c != '{') return false;
    switch (c) {
      case '{':
        if (depth >= kMaxDepth) return false;
        stack[depth++] = '{';
        mode = OBJ_FIRST;
        return true;
      case '[':
        if (depth >= kMaxDepth) return false;
        stack[depth++] = '[';
        mode = ARR_FIRST;
        return true;
      case '"':
        mode = STRING;
        key = false;
        return true;
      case '-':
        mode = NUMBER;
        sub = N_SIGN;
        return true;
      case 't': case 'f': case 'n':
        mode = LITERAL;
        lit = c == 't' ? 0 : (c == 'f' ? 1 : 2);
        sub = 1;
        return true;
      default:
        if (c >= '0' && c <= '9') {
          mode = NUMBER;
          sub = c == '0' ? N_ZERO : N_INT;
          return true;
        }
        return false;
    }
  }

  void end_value() { mode = depth == 0 ? DONE : AFTER; }

  bool feed(unsigned c) {
    switch (mode) {
      case DONE:
        return false;
      case VALUE:
        if (is_ws(c)) return blank(c);
        ws = 0;
        return begin_value(c);
      case ARR_FIRST:
        if (is_ws(c)) return blank(c);
        ws = 0;
        if (c == ']') {
          --depth;
          end_value();
          return true;
        }
        return begin_value(c);
      case OBJ_FIRST:
      case OBJ_KEY:
        if (is_ws(c)) return blank(c);
        ws = 0;
        if (c == '"') {
          mode = STRING;
          key = true;
          return true;
        }
        if (c == '}' && mode == OBJ_FIRST) {
          --depth;
          end_value();
          return true;
        }
        return false;
      case COLON:
        if (is_ws(c)) return blank(c);
        ws = 0;
        if (c != ':') return false;
        mode = VALUE;
        return true;
      case AFTER: {
        if (is_ws(c)) return blank(c);
        ws = 0;
        const char top = stack[depth - 1];
        if (c == ',') {
          mode = top == '{' ? OBJ_KEY : VALUE;
          return true;
        }
        if ((top == '{' && c == '}') || (top == '[' && c == ']')) {
          --depth;
          end_value();
          return true;
        }
        return false;
      }
      case STRING:
        if (c == '"') {
          if (key) mode = COLON;
          else end_value();
          return true;
        }
        if (c == '\\') {
          mode = ESC;
          return true;
        }
        return c >= 0x20;  // raw control characters are not allowed in JSON strings
      case ESC:
        if (c == 'u') {
          mode = UNI;
          sub = 0;
          return true;
        }
        if (std::strchr("\"\\/bfnrt", (int)c) && c) {
          mode = STRING;
          return true;
        }
        return false;
      case UNI:
        if (!is_hex(c)) return false;
        if (++sub == 4) mode = STRING;
        return true;
      case LITERAL:
        if ((unsigned char)kLit[lit][sub] != c) return false;
        if (kLit[lit][++sub] == 0) end_value();
        return true;
      case NUMBER: {
        const bool digit = c >= '0' && c <= '9';
        switch (sub) {
          case N_SIGN:
            if (!digit) return false;
            sub = c == '0' ? N_ZERO : N_INT;
            return true;
          case N_ZERO:
          case N_INT:
            if (digit && sub == N_INT) return true;
            if (c == '.') { sub = N_FRAC0; return true; }
            if (c == 'e' || c == 'E') { sub = N_EXP0; return true; }
            break;  // terminator
          case N_FRAC0:
            if (!digit) return false;
            sub = N_FRAC;
            return true;
          case N_FRAC:
            if (digit) return true;
            if (c == 'e' || c == 'E') { sub = N_EXP0; return true; }
            break;
          case N_EXP0:
            if (c == '+' || c == '-') { sub = N_EXPS; return true; }
            if (!digit) return false;
            sub = N_EXP;
            return true;
          case N_EXPS:
            if (!digit) return false;
            sub = N_EXP;
            return true;
          case N_EXP:
            if (digit) return true;
            break;
        }
        // the number ended at a byte of the enclosing structure: re-read it there
        if (depth == 0) return false;
        mode = AFTER;
        return feed(c);
      }
    }
    return false;
  }

  bool feed_bytes(const std::string& b) {
    for (unsigned char c : b)
      if (!feed(c)) return false;
    return true;
  }
};

class JsonGrammar {
 public:
  JsonGrammar(const std::vector<py::bytes>& token_bytes, const std::vector<int>& stop_ids)
      : stop_(stop_ids) {
    toks_.reserve(token_bytes.size());
    for (const auto& b : token_bytes) toks_.emplace_back(std::string(b));
  }
  int vocab() const { return (int)toks_.size(); }

  // mask[i] = 1 iff token i (mod the tokenizer size, as the detokenizer folds model ids) may
  // follow `st`; covers the full model vocabulary given by mask's length
  int fill_mask(const JsonState& st, py::array_t<uint8_t> mask) const {
    auto m = mask.mutable_unchecked<1>();
    const int V = (int)m.shape(0), n = (int)toks_.size();
    std::vector<uint8_t> base(n, 0);
    int allowed = 0;
    if (!st.done()) {
      for (int i = 0; i < n; ++i) {
        const std::string& b = toks_[i];
        if (b.empty()) continue;
        JsonState s = st;
        if (s.feed_bytes(b)) {
          base[i] = 1;
          ++allowed;
        }
      }
    }
    for (int i = 0; i < V; ++i) m(i) = base[i % n];
    if (st.done() || allowed == 0)
      for (int s : stop_) if (s >= 0 && s < V) m(s) = 1;
    if (!st.done())
      for (int s : stop_) if (s >= 0 && s < V && allowed) m(s) = 0;
    return allowed;
  }

  bool advance(JsonState& st, int tok) const {
    for (int s : stop_) if (s == tok) return st.done();
    return st.feed_bytes(toks_[tok % (int)toks_.size()]);
  }

 private:
  std::vector<std::string> toks_;
  std::vector<int> stop_;
};

}  // namespace

void register_json(py::module_& m) {
  py::class_<JsonState>(m, "JsonState")
      .def(py::init([](bool object_only) {
             JsonState s;
             s.object_only = object_only;
             return s;
           }),
           py::arg("object_only") = true)
      .def("feed", [](JsonState& s, const std::string& text) { return s.feed_bytes(text); })
      .def("copy", [](const JsonState& s) { return s; })
      .def_property_readonly("done", &JsonState::done)
      .def_property_readonly("depth", [](const JsonState& s) { return (int)s.depth; });
  py::class_<JsonGrammar>(m, "JsonGrammar")
      .def(py::init<const std::vector<py::bytes>&, const std::vector<int>&>(),
           py::arg("token_bytes"), py::arg("stop_ids"))
      .def("fill_mask", &JsonGrammar::fill_mask)
      .def("advance", &JsonGrammar::advance)
      .def_property_readonly("vocab", &JsonGrammar::vocab);
}
