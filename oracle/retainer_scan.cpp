// retainer_scan.cpp — C++ restatement of the reference's retained lookup, the
// CPU baseline of the retained reverse match.
//
// TEST INFRASTRUCTURE ONLY: linked into oracle/liboracle_trie.so, used by
// tests/ and tools/bench_retained.py's CPU leg, never by the product path.
//
// emqx_retainer_mnesia:match_messages/1 (apps/emqx_retainer/src/
// emqx_retainer_mnesia.erl:200-204) runs mnesia:dirty_select over the
// `retained` set table with the match spec of make_match_spec/1 (:222-228):
// the key pattern of condition/1 (:215-220) is only partially bound, so ETS
// visits every record and tests the pattern and the expiry guard on each —
// restated here as that scan.  read_messages/1 (:187-198) is a key lookup.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

struct Rec {
  std::vector<std::string> words;   // topic2tokens/1 (:164-165)
  uint32_t id;
  uint64_t expiry;
};

struct Store {
  std::vector<Rec> recs;
  std::unordered_map<std::string, size_t> by_topic;
};

std::vector<std::string> split(std::string_view t) {
  std::vector<std::string> w;
  size_t s = 0;
  for (size_t i = 0; i <= t.size(); ++i)
    if (i == t.size() || t[i] == '/') {
      w.emplace_back(t.substr(s, i - s));
      s = i + 1;
    }
  return w;
}

// condition/1: '+' -> '_' (any word); a last '#' -> the first '#' removed and
// an improper '_' tail (any rest).  A '#' elsewhere stays a literal '#'.
struct Pattern {
  std::vector<std::string> head;
  std::vector<bool> any;
  bool tail = false;
};

Pattern condition(std::string_view f) {
  Pattern p;
  std::vector<std::string> w = split(f);
  if (!w.empty() && w.back() == "#") {
    p.tail = true;
    auto it = std::find(w.begin(), w.end(), std::string("#"));
    w.erase(it);
  }
  for (auto& x : w) {
    p.any.push_back(x == "+");
    p.head.push_back(x);
  }
  return p;
}

bool matches(const Pattern& p, const std::vector<std::string>& key) {
  if (p.tail ? key.size() < p.head.size() : key.size() != p.head.size()) return false;
  for (size_t i = 0; i < p.head.size(); ++i)
    if (!p.any[i] && p.head[i] != key[i]) return false;
  return true;
}

bool wildcard(std::string_view f) {
  for (auto& w : split(f))
    if (w == "+" || w == "#") return true;
  return false;
}

}  // namespace

extern "C" {

void* rs_new() { return new Store(); }
void rs_free(void* s) { delete (Store*)s; }

void rs_put(void* sp, const uint8_t* blob, const uint32_t* off, uint32_t n, const uint32_t* ids,
            const uint64_t* expiry) {
  Store* s = (Store*)sp;
  for (uint32_t i = 0; i < n; ++i) {
    std::string t((const char*)blob + off[i], off[i + 1] - off[i]);
    auto it = s->by_topic.find(t);
    if (it != s->by_topic.end()) {
      s->recs[it->second].id = ids[i];
      s->recs[it->second].expiry = expiry[i];
      continue;
    }
    s->by_topic.emplace(t, s->recs.size());
    s->recs.push_back(Rec{split(t), ids[i], expiry[i]});
  }
}

// Match n filters (mode 0 = match_messages, 1 = dispatch); counts[i] = number
// of records returned for filter i; returns the total.  `threads` workers
// split the filters.
uint64_t rs_match_count(void* sp, const uint8_t* blob, const uint32_t* off, uint32_t n, uint64_t now, int mode,
                        int threads, uint32_t* counts) {
  const Store* s = (const Store*)sp;
  std::atomic<uint32_t> next{0};
  std::atomic<uint64_t> total{0};
  auto work = [&]() {
    uint64_t mine = 0;
    for (;;) {
      const uint32_t i = next.fetch_add(1);
      if (i >= n) break;
      std::string_view f((const char*)blob + off[i], off[i + 1] - off[i]);
      uint32_t c = 0;
      if (mode == 1 && !wildcard(f)) {   // read_messages/1: key lookup, Et >= Now
        auto it = s->by_topic.find(std::string(f));
        if (it != s->by_topic.end()) {
          const Rec& r = s->recs[it->second];
          c = (r.expiry == 0 || r.expiry >= now) ? 1 : 0;
        }
      } else {                           // dirty_select: every record
        const Pattern p = condition(f);
        for (const Rec& r : s->recs)
          if (matches(p, r.words) && (r.expiry == 0 || r.expiry > now)) ++c;
      }
      if (counts) counts[i] = c;
      mine += c;
    }
    total += mine;
  };
  std::vector<std::thread> th;
  for (int k = 1; k < threads; ++k) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return total.load();
}

}  // extern "C"
