// Native serving runtime: paged-KV block manager with prefix caching and the
// continuous-batching scheduler of the LLM engine (the part of TensorRT-LLM's batch manager
// the reference relies on through NIM: paged KV, inflight batching, max_batch/max_input/
// max_output envelopes — SURVEY.md §2.B N1, mistral-7b.yaml:28-39).
//
// Python owns the model and the GPU; this object owns sequence state and KV-block
// accounting, and fills caller-provided int32 buffers (pinned host memory) with the step
// layout (input ids, positions, slot mapping, cu_seqlens, context lengths, block tables)
// so one host->device copy per buffer is all the engine does per step.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <deque>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t block_hash(uint64_t prev, const int32_t* toks, int n) {
  uint64_t h = mix64(prev ^ 0x5bd1e995ull);
  for (int i = 0; i < n; ++i) h = mix64(h ^ (uint64_t)(uint32_t)toks[i]);
  return h | 1ull;  // never 0 (0 = "no hash")
}

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool prefix_caching)
      : nb_(num_blocks), bs_(block_size), prefix_(prefix_caching), ref_(num_blocks, 0),
        hash_(num_blocks, 0), lru_pos_(num_blocks) {
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
  }
  int block_size() const { return bs_; }
  int num_blocks() const { return nb_; }
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }
  int num_used() const { return nb_ - num_free(); }

  int alloc() {
    int b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else if (!lru_.empty()) {
      b = lru_.front();
      lru_.pop_front();
      cached_.erase(hash_[b]);
      hash_[b] = 0;
    } else {
      return -1;
    }
    ref_[b] = 1;
    return b;
  }
  void release(int b) {
    if (b < 0 || b >= nb_ || ref_[b] <= 0) throw std::runtime_error("release of a free block");
    if (--ref_[b] == 0) {
      if (hash_[b] != 0) {
        lru_.push_back(b);
        lru_pos_[b] = std::prev(lru_.end());
      } else {
        free_.push_back(b);
      }
    }
  }
  // Add a reference to a block another sequence already holds (copy-on-fork sharing).
  void share(int b) {
    if (b < 0 || b >= nb_ || ref_[b] <= 0) throw std::runtime_error("share of a free block");
    ref_[b] += 1;
  }
  // Look up a full block by content hash; on hit the block is referenced.
  int lookup(uint64_t h) {
    if (!prefix_) return -1;
    auto it = cached_.find(h);
    if (it == cached_.end()) return -1;
    const int b = it->second;
    if (ref_[b] == 0) lru_.erase(lru_pos_[b]);
    ref_[b] += 1;
    ++hits_;
    return b;
  }
  void register_full(int b, uint64_t h) {
    if (b < 0 || b >= nb_ || ref_[b] <= 0) throw std::runtime_error("register_full of a free block");
    if (!prefix_ || hash_[b] != 0) return;
    if (cached_.count(h)) return;  // identical content already cached in another block
    hash_[b] = h;
    cached_[h] = b;
  }
  int64_t hits() const { return hits_; }
  void reset_prefix_cache() {
    for (int b : lru_) {
      cached_.erase(hash_[b]);
      hash_[b] = 0;
      free_.push_back(b);
    }
    lru_.clear();
  }

 private:
  int nb_, bs_;
  bool prefix_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<int> free_;
  std::list<int> lru_;  // ref==0 blocks that still hold reusable (hashed) content
  std::vector<std::list<int>::iterator> lru_pos_;
  std::unordered_map<uint64_t, int> cached_;
  int64_t hits_ = 0;
};

enum Status { WAITING = 0, RUNNING = 1, FINISHED = 2 };

struct Seq {
  int64_t id;
  std::vector<int32_t> toks;  // prompt + generated
  int prompt_len;
  int max_new;
  int computed = 0;            // tokens whose KV is in the cache
  int cached_prefix = 0;       // tokens served from the prefix cache at admission
  std::vector<int32_t> blocks;
  std::vector<uint64_t> hashes;  // hash of each full block
  int status = WAITING;
  int64_t arrival;
  int preemptions = 0;
  int64_t enq_step = 0;  // scheduler step at which it (re)entered the waiting queue
};

class Scheduler {
 public:
  Scheduler(int num_blocks, int block_size, int max_num_seqs, int max_batched_tokens,
            int max_model_len, bool prefix_caching)
      : bm_(num_blocks, block_size, prefix_caching), bs_(block_size), max_seqs_(max_num_seqs),
        max_tokens_(max_batched_tokens), max_len_(max_model_len) {}

  void add(int64_t id, const std::vector<int32_t>& prompt, int max_new) {
    if (seqs_.count(id)) throw std::runtime_error("duplicate sequence id");
    if (prompt.empty()) throw std::runtime_error("empty prompt");
    if ((int)prompt.size() + max_new > max_len_)
      throw std::runtime_error("prompt + max_tokens exceeds max_model_len");
    Seq s;
    s.id = id;
    s.toks = prompt;
    s.prompt_len = (int)prompt.size();
    s.max_new = max_new;
    s.arrival = clock_++;
    s.enq_step = step_;
    seqs_.emplace(id, std::move(s));
    waiting_.push_back(id);
  }

  // Mixed steps (SARATHI-style piggybacking): when > 0, a step that has decode-ready
  // sequences also carries up to this many prefill tokens, so the decode rows ride along the
  // prefill GEMMs instead of re-reading every weight in a separate skinny decode step.
  void set_mixed_prefill_tokens(int n) { mixed_tokens_ = std::max(0, n); }
  // Round the token count of prefill/mixed steps down to a multiple of `a` by shortening the
  // last prefill chunks (the remainder runs next step): the projection GEMMs then always see
  // M in a small set of tile-aligned sizes, which the per-shape GEMM table covers.
  void set_token_alignment(int a) { align_ = std::max(1, a); }
  // Accumulate prefill work for mixed steps: while decodes are running, a mixed step is only
  // formed once at least `min_tokens` prompt tokens are pending or the oldest waiting request
  // has waited `max_wait_steps` scheduler steps — larger mixed GEMMs run closer to the MFMA
  // roofline than one small prefill per step, at a bounded cost in time-to-first-token.
  void set_mixed_min_tokens(int min_tokens, int max_wait_steps) {
    mixed_min_ = std::max(0, min_tokens);
    mixed_wait_ = std::max(0, max_wait_steps);
  }
  int last_num_decode() const { return last_nd_; }

  // Fill the step buffers. Returns (kind, num_seqs, num_tokens); kind 0 idle, 1 prefill,
  // 2 decode, 3 mixed (rows [0, last_num_decode()) decode one token each, the rest prefill).
  // seq_ids[i], cu_q[i..i+1], ctx[i], sample[i] (1 = produce a token), block_tables[i][:] per seq.
  py::tuple schedule(py::array_t<int32_t> input_ids, py::array_t<int32_t> positions,
                     py::array_t<int32_t> slots, py::array_t<int32_t> cu_q,
                     py::array_t<int32_t> ctx, py::array_t<int32_t> block_tables,
                     py::array_t<int64_t> seq_ids, py::array_t<int32_t> sample) {
    Bufs B{input_ids.mutable_unchecked<1>(), positions.mutable_unchecked<1>(),
           slots.mutable_unchecked<1>(), cu_q.mutable_unchecked<1>(), ctx.mutable_unchecked<1>(),
           block_tables.mutable_unchecked<2>(), seq_ids.mutable_unchecked<1>(),
           sample.mutable_unchecked<1>()};
    const int cap_tokens = std::min<int>((int)B.ids.shape(0), max_tokens_);
    const int cap_seqs = std::min<int>((int)B.sid.shape(0), max_seqs_);
    last_nd_ = 0;

    ++step_;
    if (mixed_tokens_ > 0) {
      std::vector<int64_t> dec = decode_ready();
      if (!dec.empty() && !prefill_ready()) {
        std::vector<int64_t> ok = prepare_decode(dec, cap_seqs);
        const std::vector<int> ones(ok.size(), 1);
        B.cq(0) = 0;
        const int t = fill_rows(B, ok, ones, 0, 0);
        return py::make_tuple(ok.empty() ? 0 : 2, (int)ok.size(), t);
      }
      if (!dec.empty()) {
        std::vector<int64_t> ok = prepare_decode(dec, cap_seqs);
        std::vector<int64_t> chosen;
        std::vector<int> qlen;
        // a large prefill backlog (a burst of arrivals) is worked off in full-size chunks:
        // capping it at mixed_tokens_ would stretch it over many decode-dominated steps
        const int budget = pending_prefill_tokens() >= 4LL * mixed_tokens_ ? cap_tokens - (int)ok.size()
                                                                           : mixed_tokens_;
        pick_prefill(std::min(cap_tokens - (int)ok.size(), budget), cap_seqs - (int)ok.size(),
                     chosen, qlen);
        align_tokens((int)ok.size(), chosen, qlen);
        const std::vector<int> ones(ok.size(), 1);
        B.cq(0) = 0;
        int t = fill_rows(B, ok, ones, 0, 0);
        if (chosen.empty()) return py::make_tuple(ok.empty() ? 0 : 2, (int)ok.size(), t);
        last_nd_ = (int)ok.size();
        t = fill_rows(B, chosen, qlen, (int)ok.size(), t);
        return py::make_tuple(ok.empty() ? 1 : 3, (int)(ok.size() + chosen.size()), t);
      }
    }

    // ---- prefill: continue partially prefilled seqs, then admit waiting ones (FCFS)
    std::vector<int64_t> chosen;
    std::vector<int> qlen;
    pick_prefill(cap_tokens, cap_seqs, chosen, qlen);
    align_tokens(0, chosen, qlen);
    if (!chosen.empty()) {
      B.cq(0) = 0;
      const int t = fill_rows(B, chosen, qlen, 0, 0);
      return py::make_tuple(1, (int)chosen.size(), t);
    }

    // ---- decode: every running seq with all tokens but the last computed
    std::vector<int64_t> dec = decode_ready();
    if (dec.empty()) return py::make_tuple(0, 0, 0);
    std::vector<int64_t> ok = prepare_decode(dec, cap_seqs);
    const std::vector<int> ones(ok.size(), 1);
    B.cq(0) = 0;
    const int t = fill_rows(B, ok, ones, 0, 0);
    return py::make_tuple(ok.empty() ? 0 : 2, (int)ok.size(), t);
  }

  void append_token(int64_t id, int32_t tok) {
    Seq& s = seqs_.at(id);
    s.toks.push_back(tok);
  }

  void append_tokens(py::array_t<int64_t> ids, py::array_t<int32_t> toks, int n) {
    auto a = ids.unchecked<1>();
    auto b = toks.unchecked<1>();
    for (int i = 0; i < n; ++i) append_token(a(i), b(i));
  }

  // Pipelined decode: the token a sequence will sample in the in-flight step is not known
  // yet; a placeholder (-1) lets the next step be scheduled now (its input id is gathered
  // on the GPU from the previous step's output) and is replaced once the step completes.
  void append_placeholders(const std::vector<int64_t>& ids) {
    for (int64_t id : ids) seqs_.at(id).toks.push_back(-1);
  }

  void set_last_token(int64_t id, int32_t tok) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;  // finished / aborted meanwhile
    Seq& s = it->second;
    if (s.toks.empty() || s.toks.back() != -1) throw std::runtime_error("no placeholder to fill");
    s.toks.back() = tok;
  }

  bool has_placeholder(int64_t id) const {
    auto it = seqs_.find(id);
    return it != seqs_.end() && !it->second.toks.empty() && it->second.toks.back() == -1;
  }

  void drop_placeholder(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;
    Seq& s = it->second;
    if (!s.toks.empty() && s.toks.back() == -1) {
      s.toks.pop_back();
      if (s.computed > (int)s.toks.size()) s.computed = (int)s.toks.size();
    }
  }

  // Beam search: clone a sequence. The child shares every full KV block of the parent
  // (reference-counted) and gets a fresh block for the partially filled last one; the caller
  // copies that block's KV on the GPU (returned as (src, dst), or (-1, -1) when the parent's
  // computed length is block-aligned). With no free block the child re-enters the waiting
  // queue and recomputes (prefix-cached blocks still hit), like a preempted sequence.
  py::tuple fork(int64_t pid, int64_t cid) {
    if (seqs_.count(cid)) throw std::runtime_error("duplicate sequence id");
    const Seq& p = seqs_.at(pid);
    Seq c;
    c.id = cid;
    c.toks = p.toks;
    c.prompt_len = p.prompt_len;
    c.max_new = p.max_new;
    c.arrival = p.arrival;
    c.enq_step = step_;
    int src = -1, dst = -1;
    const int full = p.computed / bs_;
    const bool partial = p.computed % bs_ != 0;
    // the child gets as many blocks as the parent holds: the full ones shared, a copy of the
    // partial one, and fresh blocks for the rest (a parent still prefilling already holds
    // the blocks of its whole prompt, and fill_rows indexes them)
    const int fresh = (int)p.blocks.size() - full;
    if (p.status == RUNNING && fresh <= bm_.num_free()) {
      for (int i = 0; i < full; ++i) {
        bm_.share(p.blocks[i]);
        c.blocks.push_back(p.blocks[i]);
      }
      if (partial) {
        src = p.blocks[full];
        dst = bm_.alloc();
        c.blocks.push_back(dst);
      }
      while (c.blocks.size() < p.blocks.size()) c.blocks.push_back(bm_.alloc());
      c.hashes.assign(p.hashes.begin(), p.hashes.begin() + std::min<size_t>(full, p.hashes.size()));
      c.computed = p.computed;
      c.cached_prefix = p.cached_prefix;
      c.status = RUNNING;
      running_.push_back(cid);
    } else {
      c.status = WAITING;
      waiting_.push_front(cid);
    }
    seqs_.emplace(cid, std::move(c));
    return py::make_tuple(src, dst);
  }

  void finish(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;
    Seq& s = it->second;
    for (int b : s.blocks) bm_.release(b);
    s.blocks.clear();
    if (s.status == RUNNING)
      running_.erase(std::find(running_.begin(), running_.end(), id));
    else if (s.status == WAITING) {
      auto w = std::find(waiting_.begin(), waiting_.end(), id);
      if (w != waiting_.end()) waiting_.erase(w);
    }
    seqs_.erase(it);
  }

  int num_generated(int64_t id) const {
    const Seq& s = seqs_.at(id);
    return (int)s.toks.size() - s.prompt_len;
  }
  std::vector<int32_t> tokens(int64_t id) const { return seqs_.at(id).toks; }
  int cached_prefix(int64_t id) const { return seqs_.at(id).cached_prefix; }
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  bool has_work() const { return !waiting_.empty() || !running_.empty(); }
  int free_blocks() const { return bm_.num_free(); }
  int used_blocks() const { return bm_.num_used(); }
  int total_blocks() const { return bm_.num_blocks(); }
  int64_t prefix_hits() const { return bm_.hits(); }
  int64_t preemptions() const { return preempt_count_; }
  void reset_prefix_cache() { bm_.reset_prefix_cache(); }

 private:
  struct Bufs {
    py::detail::unchecked_mutable_reference<int32_t, 1> ids, pos, sl, cq, cx;
    py::detail::unchecked_mutable_reference<int32_t, 2> bt;
    py::detail::unchecked_mutable_reference<int64_t, 1> sid;
    py::detail::unchecked_mutable_reference<int32_t, 1> smp;
  };

  // Prefill candidates: partially prefilled running seqs first, then FCFS admission.
  void pick_prefill(int budget, int cap_seqs, std::vector<int64_t>& chosen, std::vector<int>& qlen) {
    if (budget <= 0 || cap_seqs <= 0) return;
    for (int64_t id : running_) {
      Seq& s = seqs_.at(id);
      const int todo = (int)s.toks.size() - s.computed;
      if (todo > 1 || (todo == 1 && s.computed < s.prompt_len)) {
        if ((int)chosen.size() >= cap_seqs || budget <= 0) break;
        const int n = std::min(todo, budget);
        chosen.push_back(id);
        qlen.push_back(n);
        budget -= n;
      }
    }
    while (!waiting_.empty() && budget > 0 && (int)chosen.size() < cap_seqs &&
           (int)running_.size() < max_seqs_) {
      const int64_t id = waiting_.front();
      Seq& s = seqs_.at(id);
      if (!admit(s)) break;
      waiting_.pop_front();
      running_.push_back(id);
      s.status = RUNNING;
      const int todo = (int)s.toks.size() - s.computed;
      const int n = std::min(todo, budget);
      chosen.push_back(id);
      qlen.push_back(n);
      budget -= n;
    }
  }

  // Round the step's token count DOWN to a multiple of align_ by shortening the last prefill
  // chunk (the rest goes in the next step), so a graph bucket is not mostly padding — unless
  // that would leave the chunk's sequence a tail shorter than align_. Such a tail used to be fed
  // 256 - nd tokens a step (nd = 250 decode rows: a 40-token tail in 7 steps of 6 tokens, each
  // paying a prefill-attention pass, the prompt's first token 7 steps late; the headline ran
  // 55 % of its steps that way, profiles/r6_steps/); finishing it in one padded 512-token step
  // cost as much. Keeping the whole prompt in this step costs its padding to the next bucket
  // instead: headline +1.2 % (41.01 / 41.19 vs 40.79 / 40.46 QPS interleaved, p50 TTFT 161-170
  // vs 169-209 ms; profiles/r6_align/).
  void align_tokens(int nd, std::vector<int64_t>& chosen, std::vector<int>& qlen) {
    if (align_ <= 1 || chosen.empty()) return;
    int total = nd;
    for (int q : qlen) total += q;
    const int target = total - total % align_;
    if (target - nd < align_ || target == total) return;
    const Seq& last = seqs_.at(chosen.back());
    const int todo = (int)last.toks.size() - last.computed;   // its tokens left before this step
    if (total - target <= qlen.back() && todo - (qlen.back() - (total - target)) < align_) return;
    int cut = total - target;
    while (cut > 0 && !chosen.empty()) {
      const int take = std::min(cut, qlen.back());
      qlen.back() -= take;
      cut -= take;
      if (qlen.back() == 0) {
        chosen.pop_back();
        qlen.pop_back();
      }
    }
  }

  int64_t pending_prefill_tokens() const {
    int64_t pending = 0;
    for (int64_t id : running_) {
      const Seq& s = seqs_.at(id);
      if (s.computed < s.prompt_len) pending += (int)s.toks.size() - s.computed;
    }
    for (int64_t id : waiting_) {
      const Seq& s = seqs_.at(id);
      pending += (int)s.toks.size() - s.computed;
    }
    return pending;
  }

  // Enough prefill work pending (or waited long enough) to form a mixed step.
  bool prefill_ready() const {
    if (mixed_min_ <= 0) return true;
    int64_t pending = 0;
    int64_t oldest = -1;
    for (int64_t id : running_) {  // admitted, partially prefilled (chunk cut by the budget)
      const Seq& s = seqs_.at(id);
      if (s.computed < s.prompt_len) {
        pending += (int)s.toks.size() - s.computed;
        if (oldest < 0 || s.enq_step < oldest) oldest = s.enq_step;
      }
    }
    for (int64_t id : waiting_) {
      const Seq& s = seqs_.at(id);
      pending += (int)s.toks.size() - s.computed;
      if (oldest < 0 || s.enq_step < oldest) oldest = s.enq_step;
    }
    if (pending == 0) return false;
    if (pending >= mixed_min_) return true;
    return oldest >= 0 && step_ - oldest >= mixed_wait_;
  }

  std::vector<int64_t> decode_ready() {
    std::vector<int64_t> dec;
    for (int64_t id : running_) {
      Seq& s = seqs_.at(id);
      if ((int)s.toks.size() - s.computed == 1 && s.computed >= s.prompt_len) dec.push_back(id);
    }
    return dec;
  }

  // Give every decode seq whose next token starts a new block that block, preempting the
  // latest arrivals (recompute later) when the pool is exhausted.
  std::vector<int64_t> prepare_decode(std::vector<int64_t> dec, int cap_seqs) {
    std::sort(dec.begin(), dec.end(),
              [&](int64_t a, int64_t b) { return seqs_.at(a).arrival < seqs_.at(b).arrival; });
    std::vector<int64_t> ok;
    for (size_t i = 0; i < dec.size(); ++i) {
      Seq& s = seqs_.at(dec[i]);
      if (s.status != RUNNING) continue;
      const int p = s.computed;  // position of the token being computed now
      bool have = p / bs_ < (int)s.blocks.size();
      while (!have) {
        const int b = bm_.alloc();
        if (b >= 0) {
          s.blocks.push_back(b);
          have = true;
          break;
        }
        int64_t victim = -1;
        for (size_t j = dec.size(); j-- > i + 1;) {
          if (seqs_.at(dec[j]).status == RUNNING) {
            victim = dec[j];
            break;
          }
        }
        if (victim < 0) victim = s.id;
        preempt(victim);
        if (victim == s.id) break;
      }
      if (have && s.status == RUNNING) ok.push_back(s.id);
      if ((int)ok.size() >= cap_seqs) break;
    }
    return ok;
  }

  // Lay out rows [row0, row0 + ids.size()) starting at token t; returns the next token index.
  int fill_rows(Bufs& B, const std::vector<int64_t>& ids, const std::vector<int>& qlen, int row0, int t) {
    const int max_bt = (int)B.bt.shape(1);
    for (size_t i = 0; i < ids.size(); ++i) {
      Seq& s = seqs_.at(ids[i]);
      const int n = qlen[i];
      if ((s.computed + n + bs_ - 1) / bs_ > (int)s.blocks.size())
        throw std::runtime_error("scheduled tokens outside the sequence's KV blocks");
      for (int j = 0; j < n; ++j) {
        const int p = s.computed + j;
        B.ids(t) = s.toks[p];
        B.pos(t) = p;
        B.sl(t) = s.blocks[p / bs_] * bs_ + p % bs_;
        ++t;
      }
      s.computed += n;
      const int r = row0 + (int)i;
      B.cq(r + 1) = t;
      B.cx(r) = s.computed;
      B.sid(r) = s.id;
      B.smp(r) = s.computed == (int)s.toks.size() ? 1 : 0;
      fill_bt(B.bt, r, s, max_bt);
      register_full_blocks(s);
    }
    return t;
  }

  bool admit(Seq& s) {
    // prefix-cache lookup over full blocks, keeping >= 1 token to compute
    const int n = (int)s.toks.size();
    std::vector<int32_t> got;
    std::vector<uint64_t> hs;
    uint64_t prev = 0;
    const int max_cached_blocks = (n - 1) / bs_;
    for (int i = 0; i < max_cached_blocks; ++i) {
      const uint64_t h = block_hash(prev, s.toks.data() + i * bs_, bs_);
      const int b = bm_.lookup(h);
      if (b < 0) break;
      got.push_back(b);
      hs.push_back(h);
      prev = h;
    }
    const int need = (n + bs_ - 1) / bs_ - (int)got.size();
    // keep one spare block per running sequence for decode growth (watermark)
    if (need > bm_.num_free() - (int)running_.size() / 4) {
      for (int b : got) bm_.release(b);
      return false;
    }
    for (int i = 0; i < need; ++i) got.push_back(bm_.alloc());
    s.blocks = got;
    s.hashes = hs;
    s.computed = (int)hs.size() * bs_;
    s.cached_prefix = s.computed;
    return true;
  }

  void register_full_blocks(Seq& s) {
    const int full = s.computed / bs_;
    while ((int)s.hashes.size() < full) {
      const int i = (int)s.hashes.size();
      bool pending = false;
      for (int j = 0; j < bs_; ++j) pending |= s.toks[i * bs_ + j] < 0;
      if (pending) break;  // hash once the placeholder has its real token
      const uint64_t prev = i ? s.hashes[i - 1] : 0;
      const uint64_t h = block_hash(prev, s.toks.data() + i * bs_, bs_);
      s.hashes.push_back(h);
      bm_.register_full(s.blocks[i], h);
    }
  }

  void preempt(int64_t id) {
    Seq& s = seqs_.at(id);
    for (int b : s.blocks) bm_.release(b);
    s.blocks.clear();
    s.hashes.clear();
    s.computed = 0;
    s.status = WAITING;
    s.preemptions += 1;
    ++preempt_count_;
    running_.erase(std::find(running_.begin(), running_.end(), id));
    s.enq_step = step_ - mixed_wait_;  // a preempted sequence is due at once
    waiting_.push_front(id);
  }

  template <typename BT>
  void fill_bt(BT& bt, int row, const Seq& s, int max_bt) {
    if ((int)s.blocks.size() > max_bt) throw std::runtime_error("block table too narrow");
    for (int j = 0; j < (int)s.blocks.size(); ++j) bt(row, j) = s.blocks[j];
    for (int j = (int)s.blocks.size(); j < max_bt; ++j) bt(row, j) = 0;
  }

  BlockManager bm_;
  int bs_, max_seqs_, max_tokens_, max_len_;
  std::unordered_map<int64_t, Seq> seqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
  int64_t clock_ = 0;
  int64_t preempt_count_ = 0;
  int mixed_tokens_ = 0;
  int mixed_min_ = 0;
  int mixed_wait_ = 0;
  int64_t step_ = 0;
  int align_ = 1;
  int last_nd_ = 0;
};

}  // namespace

void register_bm25(py::module_& m);
void register_text(py::module_& m);
void register_json(py::module_& m);
void register_hnsw(py::module_& m);
void register_idmap(py::module_& m);
void register_shm(py::module_& m);

PYBIND11_MODULE(_rt, m) {
  m.doc() = "nv_genai_amd native host runtime";
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = true)
      .def("alloc", &BlockManager::alloc)
      .def("release", &BlockManager::release)
      .def("lookup", &BlockManager::lookup)
      .def("register_full", &BlockManager::register_full)
      .def("num_free", &BlockManager::num_free)
      .def("num_used", &BlockManager::num_used)
      .def_property_readonly("block_size", &BlockManager::block_size);
  m.def("block_hash", [](uint64_t prev, const std::vector<int32_t>& toks) {
    return block_hash(prev, toks.data(), (int)toks.size());
  });
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int, bool>(), py::arg("num_blocks"),
           py::arg("block_size"), py::arg("max_num_seqs"), py::arg("max_batched_tokens"),
           py::arg("max_model_len"), py::arg("prefix_caching") = true)
      .def("add", &Scheduler::add)
      .def("schedule", &Scheduler::schedule)
      .def("append_token", &Scheduler::append_token)
      .def("append_tokens", &Scheduler::append_tokens)
      .def("append_placeholders", &Scheduler::append_placeholders)
      .def("set_last_token", &Scheduler::set_last_token)
      .def("has_placeholder", &Scheduler::has_placeholder)
      .def("drop_placeholder", &Scheduler::drop_placeholder)
      .def("finish", &Scheduler::finish)
      .def("fork", &Scheduler::fork)
      .def("num_generated", &Scheduler::num_generated)
      .def("tokens", &Scheduler::tokens)
      .def("cached_prefix", &Scheduler::cached_prefix)
      .def("num_waiting", &Scheduler::num_waiting)
      .def("num_running", &Scheduler::num_running)
      .def("has_work", &Scheduler::has_work)
      .def("free_blocks", &Scheduler::free_blocks)
      .def("used_blocks", &Scheduler::used_blocks)
      .def("total_blocks", &Scheduler::total_blocks)
      .def("prefix_hits", &Scheduler::prefix_hits)
      .def("preemptions", &Scheduler::preemptions)
      .def("reset_prefix_cache", &Scheduler::reset_prefix_cache)
      .def("set_mixed_prefill_tokens", &Scheduler::set_mixed_prefill_tokens)
      .def("set_token_alignment", &Scheduler::set_token_alignment)
      .def("set_mixed_min_tokens", &Scheduler::set_mixed_min_tokens)
      .def("last_num_decode", &Scheduler::last_num_decode);
  register_bm25(m);
  register_text(m);
  register_json(m);
  register_hnsw(m);
  register_idmap(m);
  register_shm(m);
}
