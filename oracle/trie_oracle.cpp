// trie_oracle.cpp — C++ restatement of the reference's emqx_trie / emqx_router
// lookup, used as (1) the large-scale parity checker and (2) the timed CPU
// baseline ("kind": "port") in bench.py.
//
// TEST INFRASTRUCTURE ONLY: nothing in emqx_amd/ or libemqx_gpu_match.so links
// or calls this.  Parity pinning: see oracle/trie_ref.py's header (the Python
// restatement is pinned to the reference's known-answer tests; this file is
// cross-checked against it in tests/test_oracle_cpp.py).
//
// Faithful to the reference's data layout on purpose: the mnesia ordered_set
// `emqx_trie` (apps/emqx/src/emqx_trie.erl:45-51,61-71) becomes a hash map of
// whole-string keys {Prefix,0} / {Topic,1} with ref-counts, and match/1 is the
// same recursive DFS that builds a fresh prefix string per probe with join/2
// (:154-158) — match_compact/4 (:251-266) or match_no_compact/4 (:225-249).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

// A word is either a binary or one of the atoms '' '+' '#' (emqx_topic.erl:161-164).
struct Word {
  enum Kind : uint8_t { BIN, EMPTY, PLUS, HASH } kind;
  std::string bin;
};

std::vector<Word> words(const char* p, size_t len) {  // emqx_topic.erl:153-164
  std::vector<Word> out;
  size_t s = 0;
  for (size_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    size_t wl = i - s;
    Word w;
    if (wl == 0) w.kind = Word::EMPTY;
    else if (wl == 1 && p[s] == '+') w.kind = Word::PLUS;
    else if (wl == 1 && p[s] == '#') w.kind = Word::HASH;
    else {
      w.kind = Word::BIN;
      w.bin.assign(p + s, wl);
    }
    out.push_back(std::move(w));
    s = i + 1;
  }
  return out;
}

bool wildcard(const std::vector<Word>& ws) {  // emqx_topic.erl:53-62
  for (const auto& w : ws)
    if (w.kind == Word::PLUS || w.kind == Word::HASH) return true;
  return false;
}

const std::string& bin_of(const Word& w) {  // emqx_topic.erl:140-144
  static const std::string e, plus("+"), hash("#");
  switch (w.kind) {
    case Word::EMPTY: return e;
    case Word::PLUS: return plus;
    case Word::HASH: return hash;
    default: return w.bin;
  }
}

// A prefix is either the virtual root `empty` or a binary (emqx_trie.erl:154-158,201).
struct Prefix {
  bool root;
  std::string bin;
};

Prefix join(const Prefix& p, const Word& w) {  // emqx_trie.erl:154-158
  if (p.root) return Prefix{false, bin_of(w)};
  std::string s;
  s.reserve(p.bin.size() + 1 + bin_of(w).size());
  s += p.bin;
  s += '/';
  s += bin_of(w);
  return Prefix{false, std::move(s)};
}

std::string join_list(const std::vector<std::string>& ws) {  // emqx_topic.erl:184-195
  std::string s;
  for (size_t i = 0; i < ws.size(); ++i) {
    if (i) s += '/';
    s += ws[i];
  }
  return s;
}

struct Trie {
  bool compact = true;
  std::unordered_map<std::string, uint32_t> tab;  // key = tag byte ('0'|'1') + bytes

  static std::string key(char tag, const std::string& b) {
    std::string k;
    k.reserve(b.size() + 1);
    k += tag;
    k += b;
    return k;
  }

  std::vector<std::string> compact_segs(const std::vector<Word>& ws) const {  // :132-152
    std::vector<std::string> acc;
    if (!compact) {
      for (const auto& w : ws) acc.push_back(bin_of(w));
      return acc;
    }
    Prefix seg{true, {}};
    for (const auto& w : ws) {
      if (w.kind == Word::PLUS || w.kind == Word::HASH) {
        acc.push_back(join(seg, w).bin);
        seg = Prefix{true, {}};
      } else {
        seg = join(seg, w);
      }
    }
    if (!seg.root) acc.push_back(seg.bin);
    return acc;
  }

  std::vector<std::string> make_keys(const std::string& topic) const {  // :128-130,160-169
    std::vector<std::string> keys{key('1', topic)};
    auto segs = compact_segs(words(topic.data(), topic.size()));
    std::vector<std::string> cur;
    for (size_t i = 0; i + 1 < segs.size(); ++i) {
      cur.push_back(segs[i]);
      keys.push_back(key('0', join_list(cur)));
    }
    return keys;
  }

  bool insert(const std::string& topic) {  // :82-87
    if (tab.count(key('1', topic))) return false;
    for (auto& k : make_keys(topic)) ++tab[k];
    return true;
  }

  bool remove(const std::string& topic) {  // :91-96,180-188
    if (!tab.count(key('1', topic))) return false;
    for (auto& k : make_keys(topic)) {
      auto it = tab.find(k);
      if (it == tab.end()) continue;
      if (it->second > 1) --it->second;
      else tab.erase(it);
    }
    return true;
  }

  bool lookup(const std::string& k) const {
    auto it = tab.find(k);
    return it != tab.end() && it->second > 0;
  }
  void lookup_topic(const std::string& t, std::vector<std::string>& acc) const {  // :195-199
    if (lookup(key('1', t))) acc.push_back(t);
  }
  bool has_prefix(const Prefix& p) const {  // :201-206
    return p.root || lookup(key('0', p.bin));
  }
  void match_hash(const Prefix& p, std::vector<std::string>& acc) const {  // :268-270
    static const Word hash{Word::HASH, {}};
    lookup_topic(join(p, hash).bin, acc);
  }

  void match_compact(const std::vector<Word>& ws, size_t i, const Prefix& p, bool wc,
                     std::vector<std::string>& acc) const {  // :251-266
    if (i == ws.size()) {
      match_hash(p, acc);
      if (wc) lookup_topic(p.bin, acc);
      return;
    }
    match_hash(p, acc);
    match_compact(ws, i + 1, join(p, ws[i]), wc, acc);
    static const Word plus{Word::PLUS, {}};
    Prefix wp = join(p, plus);
    if (i + 1 == ws.size() || has_prefix(wp)) match_compact(ws, i + 1, wp, true, acc);
  }

  void match_no_compact(const std::vector<Word>& ws, size_t i, const Prefix& p, bool wc,
                        std::vector<std::string>& acc) const {  // :225-249
    if (i == ws.size()) {
      match_hash(p, acc);
      if (wc) lookup_topic(p.bin, acc);
      return;
    }
    if (!has_prefix(p)) return;
    match_hash(p, acc);
    static const Word plus{Word::PLUS, {}};
    match_no_compact(ws, i + 1, join(p, plus), true, acc);
    match_no_compact(ws, i + 1, join(p, ws[i]), wc, acc);
  }

  std::vector<std::string> match(const char* t, size_t len) const {  // :100-114,208-223
    std::vector<std::string> acc;
    auto ws = words(t, len);
    if (wildcard(ws)) return acc;
    size_t i0 = 0;
    Prefix p{true, {}};
    if (ws[0].kind == Word::BIN && ws[0].bin[0] == '$') {
      if (ws.size() == 1) lookup_topic(ws[0].bin, acc);
      p = Prefix{false, ws[0].bin};
      i0 = 1;
    }
    if (compact) match_compact(ws, i0, p, false, acc);
    else match_no_compact(ws, i0, p, false, acc);
    return acc;
  }
};

struct Oracle {
  Trie trie;
  int mode = 0;  // 0 = emqx_trie:match/1, 1 = emqx_router:match_routes/1 filter set
  std::unordered_map<std::string, uint32_t> ids;  // filter -> id (the route table keys)
  // every word-prefix of every filter up to (not including) a '#' word, '+'
  // spelled "+": the states an NFA over the filter set can be in (built on
  // first use by ot_visited_counts; SURVEY §8d's V_t)
  std::unordered_set<std::string> prefixes;
  bool prefixes_built = false;
};

// SURVEY §8d V_t, counted from string prefixes independently of the GPU
// table: per topic without a '+'/'#' word, the root plus every prefix P of
// length l = 1..D that is a prefix of some filter and matches the topic's
// first l words word by word ('+' any word; a '$' first word never under a
// root '+', emqx_trie.erl:208-215).  These are the states the kernels create
// (a literal or '+' child that exists); '#' children are emitted, not states.
void build_prefixes(Oracle* o) {
  if (o->prefixes_built) return;
  for (const auto& kv : o->ids) {
    auto ws = words(kv.first.data(), kv.first.size());
    std::string p;
    for (size_t i = 0; i < ws.size(); ++i) {
      if (ws[i].kind == Word::HASH) break;
      if (i) p += '/';
      p += bin_of(ws[i]);
      o->prefixes.insert(p);
    }
  }
  o->prefixes_built = true;
}

uint64_t visited_one(const Oracle* o, const char* t, size_t len) {
  auto ws = words(t, len);
  if (wildcard(ws)) return 0;
  const bool dollar = ws[0].kind == Word::BIN && ws[0].bin[0] == '$';
  uint64_t v = 1;   // the root
  std::vector<std::string> cur, nxt;
  for (size_t l = 0; l < ws.size(); ++l) {
    nxt.clear();
    auto step = [&](const std::string* s, const std::string& w) {
      std::string c = s ? *s + "/" + w : w;
      if (o->prefixes.count(c)) {
        ++v;
        nxt.push_back(std::move(c));
      }
    };
    if (l == 0) {
      step(nullptr, bin_of(ws[0]));
      if (!dollar) step(nullptr, "+");
    } else {
      for (const auto& s : cur) {
        step(&s, bin_of(ws[l]));
        step(&s, "+");
      }
    }
    cur.swap(nxt);
    if (cur.empty()) break;
  }
  return v;
}

}  // namespace

extern "C" {

void* ot_new(int compact, int mode) {
  Oracle* o = new Oracle();
  o->trie.compact = compact != 0;
  o->mode = mode;
  return o;
}

void ot_free(void* h) { delete (Oracle*)h; }

// Switch the match mode of a built oracle.  Only valid when the trie holds the
// same filters in both modes, i.e. every filter added is a wildcard filter
// (mode 1 keeps exact filters out of the trie, emqx_router.erl:118-123);
// returns -1 otherwise.  Saves building a large all-wildcard oracle twice.
int ot_set_mode(void* h, int mode) {
  Oracle* o = (Oracle*)h;
  if (o->trie.tab.size() && o->mode != mode) {
    for (const auto& kv : o->ids)
      if (!wildcard(words(kv.first.data(), kv.first.size()))) return -1;
  }
  o->mode = mode;
  return 0;
}

// Add filters (ids optional, default = running index).  In mode 1 only
// wildcard filters enter the trie (emqx_router.erl:118-123); every filter is a
// route-table key.
int ot_add(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n, const uint32_t* ids) {
  Oracle* o = (Oracle*)h;
  for (uint32_t i = 0; i < n; ++i) {
    std::string f((const char*)blob + off[i], off[i + 1] - off[i]);
    if (o->ids.count(f)) continue;
    uint32_t id = ids ? ids[i] : (uint32_t)o->ids.size();
    o->ids.emplace(f, id);
    o->prefixes_built = false;
    if (o->mode == 0 || wildcard(words(f.data(), f.size()))) o->trie.insert(f);
  }
  if (!o->prefixes_built) std::unordered_set<std::string>().swap(o->prefixes);   // rebuilt on next use
  return 0;
}

int ot_remove(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n) {
  Oracle* o = (Oracle*)h;
  for (uint32_t i = 0; i < n; ++i) {
    std::string f((const char*)blob + off[i], off[i + 1] - off[i]);
    auto it = o->ids.find(f);
    if (it == o->ids.end()) continue;
    o->ids.erase(it);
    o->trie.remove(f);
    o->prefixes_built = false;
  }
  if (!o->prefixes_built) std::unordered_set<std::string>().swap(o->prefixes);
  return 0;
}

static void match_one(const Oracle* o, const char* t, size_t len, std::vector<uint32_t>& out) {
  std::vector<std::string> m;
  if (!(o->mode == 1 && o->trie.tab.empty())) m = o->trie.match(t, len);  // match_trie/1 :137-141
  if (o->mode == 1) {                                                     // lookup_routes(Topic) :133
    auto it = o->ids.find(std::string(t, len));
    if (it != o->ids.end()) out.push_back(it->second);
  }
  for (auto& f : m) out.push_back(o->ids.at(f));
}

// Match n topics with `threads` workers (static partition).  Outputs a CSR of
// filter ids (rows in the walk's natural order).  Returns total ids.
uint64_t ot_match(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n, int threads,
                  uint64_t* row_out, uint32_t** ids_out) {
  const Oracle* o = (const Oracle*)h;
  if (threads < 1) threads = 1;
  std::vector<std::vector<uint32_t>> per(threads);
  std::vector<uint32_t> cnt(n, 0);
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) {
    th.emplace_back([&, k]() {
      uint32_t a = (uint32_t)((uint64_t)n * k / threads), b = (uint32_t)((uint64_t)n * (k + 1) / threads);
      std::vector<uint32_t> tmp;
      for (uint32_t i = a; i < b; ++i) {
        tmp.clear();
        match_one(o, (const char*)blob + off[i], off[i + 1] - off[i], tmp);
        cnt[i] = (uint32_t)tmp.size();
        per[k].insert(per[k].end(), tmp.begin(), tmp.end());
      }
    });
  }
  for (auto& t : th) t.join();
  uint64_t total = 0;
  if (row_out) {
    row_out[0] = 0;
    for (uint32_t i = 0; i < n; ++i) row_out[i + 1] = row_out[i] + cnt[i];
  }
  for (auto& v : per) total += v.size();
  if (ids_out) {
    uint32_t* ids = (uint32_t*)malloc(total * 4 + 4);
    uint64_t p = 0;
    for (auto& v : per) {
      memcpy(ids + p, v.data(), v.size() * 4);
      p += v.size();
    }
    *ids_out = ids;
  }
  return total;
}

// Timing variant: matches and returns only the total count (no id mapping) —
// the work the reference does per publish (binaries out, no ids).
uint64_t ot_match_count(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n, int threads) {
  const Oracle* o = (const Oracle*)h;
  if (threads < 1) threads = 1;
  std::vector<uint64_t> tot(threads, 0);
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) {
    th.emplace_back([&, k]() {
      uint32_t a = (uint32_t)((uint64_t)n * k / threads), b = (uint32_t)((uint64_t)n * (k + 1) / threads);
      uint64_t s = 0;
      for (uint32_t i = a; i < b; ++i) {
        const char* t = (const char*)blob + off[i];
        size_t len = off[i + 1] - off[i];
        std::vector<std::string> m;
        if (!(o->mode == 1 && o->trie.tab.empty())) m = o->trie.match(t, len);
        s += m.size();
        if (o->mode == 1 && o->ids.count(std::string(t, len))) ++s;
      }
      tot[k] = s;
    });
  }
  for (auto& t : th) t.join();
  uint64_t s = 0;
  for (auto v : tot) s += v;
  return s;
}

// Per-topic match counts for n topics (no ids): the whole-batch row totals a
// GPU result is checked against at full config size.
uint64_t ot_match_counts(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n, int threads,
                         uint32_t* counts) {
  const Oracle* o = (const Oracle*)h;
  if (threads < 1) threads = 1;
  std::vector<uint64_t> tot(threads, 0);
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) {
    th.emplace_back([&, k]() {
      uint32_t a = (uint32_t)((uint64_t)n * k / threads), b = (uint32_t)((uint64_t)n * (k + 1) / threads);
      uint64_t s = 0;
      std::vector<uint32_t> tmp;
      for (uint32_t i = a; i < b; ++i) {
        tmp.clear();
        match_one(o, (const char*)blob + off[i], off[i + 1] - off[i], tmp);
        counts[i] = (uint32_t)tmp.size();
        s += tmp.size();
      }
      tot[k] = s;
    });
  }
  for (auto& t : th) t.join();
  uint64_t s = 0;
  for (auto v : tot) s += v;
  return s;
}

// Per-topic match counts AND an order-independent checksum of each topic's
// filter-id set: the sum (mod 2^64) of a 64-bit mix of every id in the row —
// the same mix as tests/test_gpu_scale.py::row_checksums, so a whole batch's
// rows are compared as sets at full config size without moving the ids.  The
// sum is additive over disjoint filter shards, so a sharded
// oracle's rows are checked by summing the shards' checksums.
static inline uint64_t id_mix(uint32_t id) {
  uint64_t x = id;
  x ^= x >> 16;
  x *= 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  return x;
}

uint64_t ot_match_sums(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n, int threads,
                       uint32_t* counts, uint64_t* sums) {
  const Oracle* o = (const Oracle*)h;
  if (threads < 1) threads = 1;
  std::vector<uint64_t> tot(threads, 0);
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) {
    th.emplace_back([&, k]() {
      uint32_t a = (uint32_t)((uint64_t)n * k / threads), b = (uint32_t)((uint64_t)n * (k + 1) / threads);
      uint64_t s = 0;
      std::vector<uint32_t> tmp;
      for (uint32_t i = a; i < b; ++i) {
        tmp.clear();
        match_one(o, (const char*)blob + off[i], off[i + 1] - off[i], tmp);
        uint64_t c = 0;
        for (uint32_t id : tmp) c += id_mix(id);
        counts[i] = (uint32_t)tmp.size();
        sums[i] = c;
        s += tmp.size();
      }
      tot[k] = s;
    });
  }
  for (auto& t : th) t.join();
  uint64_t s = 0;
  for (auto v : tot) s += v;
  return s;
}

// Per-topic V_t (counts may be null) and their sum over n topics.
uint64_t ot_visited_counts(void* h, const uint8_t* blob, const uint32_t* off, uint32_t n, int threads,
                           uint64_t* counts) {
  Oracle* o = (Oracle*)h;
  build_prefixes(o);
  if (threads < 1) threads = 1;
  std::vector<uint64_t> tot(threads, 0);
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) {
    th.emplace_back([&, k]() {
      uint32_t a = (uint32_t)((uint64_t)n * k / threads), b = (uint32_t)((uint64_t)n * (k + 1) / threads);
      uint64_t s = 0;
      for (uint32_t i = a; i < b; ++i) {
        const uint64_t v = visited_one(o, (const char*)blob + off[i], off[i + 1] - off[i]);
        if (counts) counts[i] = v;
        s += v;
      }
      tot[k] = s;
    });
  }
  for (auto& t : th) t.join();
  uint64_t s = 0;
  for (auto v : tot) s += v;
  return s;
}

uint64_t ot_n_keys(void* h) { return ((Oracle*)h)->trie.tab.size(); }
void ot_free_ptr(void* p) { free(p); }

}  // extern "C"
