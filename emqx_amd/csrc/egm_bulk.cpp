// egm_bulk.cpp — HostTable::bulk_build: the whole table from n filters in
// parallel (egm_table_build), producing the same image as inserting the
// filters one by one (emqx_trie:insert/1, apps/emqx/src/emqx_trie.erl:82-87,
// first occurrence of a repeated filter wins) followed by relayout():
//
//   * word ids in order of first occurrence (filter order, then word order);
//   * nodes numbered breadth-first, a parent's children in the order the
//     filters first reach them (what relayout's BFS over creation-ordered
//     node ids gives);
//   * ref-counts, '+'/'#' children, '#' and terminal filter ids, literal-child
//     signatures and flags exactly as insert + relayout set them;
//   * the edge table at relayout's size, edges inserted in child order (a
//     bucket range per thread; the rare probe that runs past its range is
//     placed afterwards, so slot positions may differ from a sequential
//     insert near range ends — a valid image either way).
//
// At C4 (100M filters) the sequential insert loop took 256 s on the GPU box's
// host cores; this build is level-synchronous: per trie level
// one parallel sort of (parent, word, filter) triples groups the filters into
// children.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

#include <algorithm>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "egm_table.h"

namespace egm {

namespace {

// fn(lo, hi, t) over min(nt, n) contiguous parts of [0, n), part t on a thread
// of its own (the same n and nt always give the same parts).
template <class F>
void parallel_for(size_t n, unsigned nt, F fn) {
  if (n < nt) nt = (unsigned)n;
  if (nt <= 1) {
    fn((size_t)0, n, 0u);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) {
    const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
    th.emplace_back([=, &fn] { fn(lo, hi, t); });
  }
  for (auto& x : th) x.join();
}

// Parallel sort: chunks sorted in parallel, then merged pairwise in rounds.
template <class T>
void parallel_sort(std::vector<T>& v, unsigned nt) {
  const size_t n = v.size();
  if (nt <= 1 || n < (1u << 16)) {
    std::sort(v.begin(), v.end());
    return;
  }
  std::vector<size_t> b(nt + 1);
  for (unsigned t = 0; t <= nt; ++t) b[t] = n * t / nt;
  parallel_for(nt, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t t = lo; t < hi; ++t) std::sort(v.begin() + b[t], v.begin() + b[t + 1]);
  });
  std::vector<T> tmp(n);
  std::vector<T>* src = &v;
  std::vector<T>* dst = &tmp;
  for (size_t w = 1; w < nt; w <<= 1) {
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; t += 2 * w) {
      const size_t a = b[t], m = b[std::min<size_t>(t + w, nt)], e = b[std::min<size_t>(t + 2 * w, nt)];
      th.emplace_back([=] { std::merge(src->begin() + a, src->begin() + m, src->begin() + m, src->begin() + e,
                                       dst->begin() + a); });
    }
    for (auto& x : th) x.join();
    std::swap(src, dst);
  }
  if (src != &v) v.swap(*src);
}

// One filter at one trie level: the node it has reached (parent of the next
// one), the next level's token and the filter's rank (first-occurrence order).
struct Item {
  uint64_t key;   // parent << 32 | token
  uint32_t li;    // filter rank
  uint32_t pad;
  bool operator<(const Item& o) const { return key != o.key ? key < o.key : li < o.li; }
};

// Indices 0..n-1 whose key(i) (< R) is r, for every r, each list in index
// order: threads bin contiguous index chunks, range r is the chunks' bins
// concatenated.
template <class K>
std::vector<std::vector<uint32_t>> bin_by_range(size_t n, unsigned R, unsigned nt, K key) {
  std::vector<std::vector<std::vector<uint32_t>>> part(nt, std::vector<std::vector<uint32_t>>(R));
  parallel_for(n, nt, [&](size_t lo, size_t hi, unsigned t) {
    for (size_t i = lo; i < hi; ++i) {
      const uint32_t r = key(i);
      if (r < R) part[t][r].push_back((uint32_t)i);
    }
  });
  std::vector<std::vector<uint32_t>> out(R);
  parallel_for(R, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t r = lo; r < hi; ++r)
      for (unsigned t = 0; t < nt; ++t) {
        out[r].insert(out[r].end(), part[t][r].begin(), part[t][r].end());
        std::vector<uint32_t>().swap(part[t][r]);
      }
  });
  return out;
}


}  // namespace

unsigned build_threads() {
  const char* e = getenv("EGM_BUILD_THREADS");
  if (e && *e) return (unsigned)std::max(1, atoi(e));
  unsigned n = std::max(1u, std::thread::hardware_concurrency());
  // the cgroup CPU quota (a container may see 256 cores and be granted 16)
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[64] = {0};
    unsigned long long period = 0;
    if (fscanf(f, "%63s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period) {
      const unsigned long long quota = strtoull(q, nullptr, 10);
      n = std::min<unsigned>(n, (unsigned)std::max<unsigned long long>(1, (quota + period - 1) / period));
    }
    fclose(f);
  }
  return std::min(n, 64u);
}

namespace {
struct Phase {   // EGM_BULK_TRACE=1: time each phase on stderr
  bool on = getenv("EGM_BULK_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void operator()(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[egm bulk] %-22s %8.3f s\n", what, std::chrono::duration<double>(now - t).count());
    t = now;
  }
};
}  // namespace

int HostTable::bulk_build(const uint8_t* blob, const uint32_t* off, uint32_t n, const uint32_t* ids, unsigned nt) {
  Phase phase;
  clear();
  if (nt == 0) nt = build_threads();
  // ---- 1. dedup (first occurrence wins), ranks in input order ----
  std::vector<uint64_t> h(n);
  parallel_for(n, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t i = lo; i < hi; ++i) h[i] = word_hash(blob + off[i], off[i + 1] - off[i]);
  });
  std::vector<uint8_t> dup(n, 0);
  {
    std::vector<Item> byh(n);
    parallel_for(n, nt, [&](size_t lo, size_t hi, unsigned) {
      for (size_t i = lo; i < hi; ++i) byh[i] = Item{h[i], (uint32_t)i, 0};
    });
    parallel_sort(byh, nt);
    parallel_for(n, nt, [&](size_t lo, size_t hi, unsigned) {
      for (size_t k = lo; k < hi; ++k) {   // compare with every earlier entry of an equal-hash run
        if (k == 0 || byh[k - 1].key != byh[k].key) continue;
        const uint32_t i = byh[k].li, li = off[i + 1] - off[i];
        for (size_t j = k; j-- > 0 && byh[j].key == byh[k].key;) {
          const uint32_t p = byh[j].li;
          if (off[p + 1] - off[p] == li && memcmp(blob + off[p], blob + off[i], li) == 0) {
            dup[i] = 1;
            break;
          }
        }
      }
    });
  }
  phase("dedup");
  std::vector<uint32_t> uniq;
  uniq.reserve(n);
  for (uint32_t i = 0; i < n; ++i)
    if (!dup[i]) uniq.push_back(i);
  std::vector<uint8_t>().swap(dup);
  const uint32_t U = (uint32_t)uniq.size();
  // filter store, in rank order
  foff_.assign((size_t)U + 1, 0);
  for (uint32_t r = 0; r < U; ++r) foff_[r + 1] = foff_[r] + (off[uniq[r] + 1] - off[uniq[r]]);
  fblob_.resize(foff_[U]);
  ffid_.resize(U);
  falive_.assign(U, 1);
  uint32_t max_fid = 0;
  parallel_for(U, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t r = lo; r < hi; ++r) {
      const uint32_t i = uniq[r];
      memcpy(fblob_.data() + foff_[r], blob + off[i], off[i + 1] - off[i]);
      ffid_[r] = ids ? ids[i] : i;
    }
  });
  for (uint32_t r = 0; r < U; ++r) max_fid = std::max(max_fid, ffid_[r] + 1);
  n_filters_ = U;
  next_fid_ = U ? max_fid : 0;
  {
    std::vector<uint64_t> hb(U), hf(U);
    parallel_for(U, nt, [&](size_t lo, size_t hi, unsigned) {
      for (size_t r = lo; r < hi; ++r) {
        hb[r] = h[uniq[r]];
        hf[r] = mix64(ffid_[r]);
      }
    });
    std::vector<uint64_t>().swap(h);
    by_bytes_.bulk_build(hb, nt);
    by_fid_.bulk_build(hf, nt);
  }
  phase("filter store + maps");
  // ---- 2. tokens per filter word: word ids in first-occurrence order ----
  std::vector<uint64_t> tok_off((size_t)U + 1, 0);
  {
    std::vector<uint32_t> depth(U);
    parallel_for(U, nt, [&](size_t lo, size_t hi, unsigned) {
      for (size_t r = lo; r < hi; ++r) {
        const uint8_t* p = fblob_.data() + foff_[r];
        const uint64_t len = foff_[r + 1] - foff_[r];
        uint32_t d = 1;
        for (uint64_t k = 0; k < len; ++k) d += p[k] == '/';
        depth[r] = d;
      }
    });
    for (uint32_t r = 0; r < U; ++r) tok_off[r + 1] = tok_off[r] + depth[r];
  }
  std::vector<uint32_t> tok(tok_off[U]);
  {
    // per thread: its words in local first-occurrence order; tokens hold local
    // ids (tagged by thread) until the merged dictionary is known
    const unsigned T = (U < 4096) ? 1u : nt;
    std::vector<std::vector<std::string_view>> local(T);
    std::vector<std::vector<uint32_t>> to_global(T);
    parallel_for(U, T, [&](size_t lo, size_t hi, unsigned t) {
      std::unordered_map<std::string_view, uint32_t> seen;
      auto& lw = local[t];
      for (size_t r = lo; r < hi; ++r) {
        const uint8_t* p = fblob_.data() + foff_[r];
        const uint32_t len = (uint32_t)(foff_[r + 1] - foff_[r]);
        uint64_t o = tok_off[r];
        uint32_t s = 0;
        for (uint32_t i = 0; i <= len; ++i) {
          if (i < len && p[i] != '/') continue;
          const uint32_t wl = i - s;
          uint32_t v;
          if (wl == 1 && p[s] == '+') v = WID_PLUS;
          else if (wl == 1 && p[s] == '#') v = WID_HASH;
          else {
            std::string_view w((const char*)p + s, wl);
            auto it = seen.find(w);
            if (it == seen.end()) {
              it = seen.emplace(w, (uint32_t)lw.size()).first;
              lw.push_back(w);
            }
            v = it->second;
          }
          tok[o++] = v;
          s = i + 1;
        }
      }
    });
    size_t total = 0;
    for (auto& l : local) total += l.size();
    size_t cap = 64;
    while (cap < 2 * total) cap <<= 1;   // the size sequential dict_add growth ends at
    dict_rehash(cap);
    for (unsigned t = 0; t < T; ++t) {
      to_global[t].resize(local[t].size());
      for (size_t k = 0; k < local[t].size(); ++k)
        to_global[t][k] = dict_add((const uint8_t*)local[t][k].data(), (uint32_t)local[t][k].size());
    }
    parallel_for(U, T, [&](size_t lo, size_t hi, unsigned t) {
      const auto& g = to_global[t];
      for (uint64_t k = tok_off[lo]; k < tok_off[hi]; ++k)
        if (tok[k] < WID_MAX) tok[k] = g[tok[k]];
    });
  }
  phase("dictionary + tokens");
  // ---- 3. the trie, one level at a time ----
  // `act` holds the filters still descending, ordered by (node reached, rank);
  // a run of equal nodes is one parent.  A level's children are numbered
  // after the previous level's: by parent in parent order, siblings in the
  // order the filters (by rank) first reach them — relayout's BFS order.  The
  // runs are split over threads (a run larger than a thread's share is sorted
  // with all of them: the root's, the root '+' child's).
  std::vector<uint32_t> act(U), nxt;
  for (uint32_t r = 0; r < U; ++r) act[r] = r;
  std::vector<uint32_t> cur_node(U, 0);   // node filter r has reached
  std::vector<NodeRec> nn(1, NodeRec{NONE, NONE, NONE, 0});
  std::vector<uint32_t> npar(1, NONE), nvia(1, NONE), nref(1, U), nhc(1, NONE);
  {   // at most one node per filter word (+ the root): reserved address space, touched as used
    const size_t bound = (size_t)tok_off[U] + 1;
    nn.reserve(bound + bound / 8 + 1024);
    for (auto* v : {&npar, &nvia, &nref, &nhc}) v->reserve(bound + bound / 8 + 1024);
  }
  struct Child {   // one child of a run, local to its chunk
    uint32_t token, first, count, start;   // its first rank, its items [start, start + count) in the chunk
  };
  for (uint32_t level = 0; !act.empty(); ++level) {
    const size_t A = act.size();
    // run boundaries, then chunks of whole runs (about A / nt items each)
    std::vector<size_t> cb{0};
    for (unsigned t = 1; t < nt; ++t) {
      size_t k = std::max(cb.back(), A * t / nt);
      while (k < A && k > 0 && cur_node[act[k]] == cur_node[act[k - 1]]) ++k;
      if (k > cb.back() && k < A) cb.push_back(k);
    }
    cb.push_back(A);
    const size_t C = cb.size() - 1;
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> citems(C);   // (token << 32 | rank), kept sorted
    std::vector<std::vector<Child>> ckids(C);
    auto sort_chunk = [&](size_t c, unsigned inner) {
      auto& it = citems[c];
      auto& kids = ckids[c];
      it.resize(cb[c + 1] - cb[c]);
      for (size_t k = cb[c]; k < cb[c + 1]; ++k) {
        const uint32_t r = act[k];
        it[k - cb[c]] = {((uint64_t)tok[tok_off[r] + level] << 32) | r, cur_node[r]};
      }
      // sort each run by (token, rank); a chunk is whole runs
      size_t a = 0;
      while (a < it.size()) {
        size_t e = a + 1;
        while (e < it.size() && it[e].second == it[a].second) ++e;
        if (e - a > 1) {
          if (inner > 1) {
            std::vector<std::pair<uint64_t, uint32_t>> run(it.begin() + a, it.begin() + e);
            parallel_sort(run, inner);
            std::copy(run.begin(), run.end(), it.begin() + a);
          } else {
            std::sort(it.begin() + a, it.begin() + e);
          }
        }
        // children of this run, then in first-rank order
        const size_t k0 = kids.size();
        for (size_t k = a; k < e; ++k)
          if (k == a || (it[k].first >> 32) != (it[k - 1].first >> 32))
            kids.push_back(Child{(uint32_t)(it[k].first >> 32), (uint32_t)it[k].first, 0, (uint32_t)k});
        for (size_t g = k0; g < kids.size(); ++g)
          kids[g].count = (uint32_t)((g + 1 < kids.size() ? kids[g + 1].start : e) - kids[g].start);
        std::sort(kids.begin() + k0, kids.end(), [](const Child& x, const Child& y) { return x.first < y.first; });
        a = e;
      }
    };
    if (C == 1) sort_chunk(0, nt);
    else parallel_for(C, (unsigned)C, [&](size_t lo, size_t hi, unsigned) {
      for (size_t c = lo; c < hi; ++c) sort_chunk(c, 1);
    });
    // child ids: chunk bases by an exclusive scan of children per chunk
    std::vector<uint64_t> cbase(C + 1, nn.size());
    for (size_t c = 0; c < C; ++c) cbase[c + 1] = cbase[c] + ckids[c].size();
    if (cbase[C] >= (uint64_t)WID_MAX) return -1;
    const uint32_t N2 = (uint32_t)cbase[C];
    nn.resize(N2, NodeRec{NONE, NONE, NONE, 0});
    npar.resize(N2);
    nvia.resize(N2);
    nref.resize(N2);
    nhc.resize(N2, NONE);
    std::vector<uint64_t> nbase(C + 1, 0);   // next level's filters per chunk
    std::vector<std::vector<uint32_t>> cnext(C);
    parallel_for(C, (unsigned)std::min<size_t>(C, nt), [&](size_t lo, size_t hi, unsigned) {
      for (size_t c = lo; c < hi; ++c) {
        const auto& it = citems[c];
        auto& out = cnext[c];
        out.reserve(it.size());
        for (size_t g = 0; g < ckids[c].size(); ++g) {
          const Child& k = ckids[c][g];
          const uint32_t node = (uint32_t)(cbase[c] + g), p = it[k.start].second;
          npar[node] = p;
          nvia[node] = k.token;
          nref[node] = k.count;
          if (k.token == WID_PLUS) nn[p].plus_child = node;   // one '+' / '#' child per parent: no race
          else if (k.token == WID_HASH) nhc[p] = node;
          for (size_t q = k.start; q < (size_t)k.start + k.count; ++q) {   // ranks ascending
            const uint32_t r = (uint32_t)it[q].first;
            cur_node[r] = node;
            if (tok_off[r] + level + 1 == tok_off[r + 1]) {   // the filter ends here
              nn[node].term_fid = ffid_[r];
              if (k.token == WID_HASH) nn[p].hash_fid = ffid_[r];   // "P/#": P emits it
            } else {
              out.push_back(r);
            }
          }
        }
        std::vector<std::pair<uint64_t, uint32_t>>().swap(citems[c]);
      }
    });
    for (size_t c = 0; c < C; ++c) nbase[c + 1] = nbase[c] + cnext[c].size();
    nxt.resize(nbase[C]);
    parallel_for(C, (unsigned)std::min<size_t>(C, nt), [&](size_t lo, size_t hi, unsigned) {
      for (size_t c = lo; c < hi; ++c) std::copy(cnext[c].begin(), cnext[c].end(), nxt.begin() + nbase[c]);
    });
    act.swap(nxt);
    phase("  level");
  }
  std::vector<uint32_t>().swap(cur_node);
  std::vector<uint32_t>().swap(tok);
  const uint32_t N = (uint32_t)nn.size();
  nodes.swap(nn);
  hash_child.swap(nhc);
  parent_.swap(npar);
  via_.swap(nvia);
  ref_.swap(nref);
  lit_count_.assign(N, 0);
  sig_.assign(N, 0);
  edge_slot_.assign(N, NONE);
  free_nodes_.clear();
  n_live_nodes_ = N;
  uint64_t n_lit = 0;
  for (uint32_t c = 1; c < N; ++c)
    if (via_[c] < WID_MAX) {
      ++lit_count_[parent_[c]];
      sig_[parent_[c]] |= sig_bit(via_[c]);
      ++n_lit;
    }
  parallel_for(N, nt, [&](size_t lo, size_t hi, unsigned) {
    for (size_t c = lo; c < hi; ++c) nodes[c].flags = own_flags((uint32_t)c);
  });
  const size_t room = N + N / 8 + 1024;   // as relayout: churn appends without moving the arrays
  for (auto* v : {&hash_child, &parent_, &via_, &ref_, &lit_count_, &sig_, &edge_slot_}) v->reserve(room);
  nodes.reserve(room);
  phase("node records");
  // ---- 4. edge table at relayout's size, edges in child order ----
  size_t nb = 16;
  while (nb * EDGE_BUCKET < (size_t)n_lit * EDGE_SPREAD) nb <<= 1;
  edges.assign(nb * EDGE_BUCKET, EdgeSlot{NONE, 0, 0, 0, NONE, NONE, NONE, 0});
  n_edges_ = n_lit;
  n_edge_tombs_ = 0;
  {
    const uint32_t m = (uint32_t)(nb - 1);
    const unsigned T = (n_lit < 65536) ? 1u : nt;
    std::vector<std::vector<uint32_t>> spill(T);
    // bucket range [nb*t/T, nb*(t+1)/T) belongs to thread t; its children in order
    auto bins = bin_by_range(N, T, nt, [&](size_t c) -> uint32_t {
      if (c == 0 || via_[c] >= WID_MAX) return T;   // root, '+' and '#' children have no edge slot
      return (uint32_t)((uint64_t)edge_bucket(parent_[c], via_[c], m) * T / nb);
    });
    parallel_for(T, T, [&](size_t lo, size_t hi, unsigned) {
      for (size_t t = lo; t < hi; ++t) {
        const uint64_t b1 = (uint64_t)nb * (t + 1) / T;
        for (uint32_t c : bins[t]) {
          const uint32_t b = edge_bucket(parent_[c], via_[c], m);
          bool placed = false;
          for (uint64_t bb = b; bb < b1 && !placed; ++bb)
            for (int k = 0; k < EDGE_BUCKET; ++k) {
              EdgeSlot& s = edges[bb * EDGE_BUCKET + k];
              if (s.parent != NONE) continue;
              const NodeRec& r = nodes[c];
              s = EdgeSlot{parent_[c], via_[c], c, r.flags, r.plus_child, r.hash_fid, r.term_fid, plus_flags(c)};
              edge_slot_[c] = (uint32_t)(bb * EDGE_BUCKET + k);
              placed = true;
              break;
            }
          if (!placed) spill[t].push_back(c);
        }
      }
    });
    for (auto& sp : spill)
      for (uint32_t c : sp) {
        uint32_t b = edge_bucket(parent_[c], via_[c], m);
        for (bool placed = false; !placed; b = (b + 1) & m)
          for (int k = 0; k < EDGE_BUCKET; ++k) {
            EdgeSlot& s = edges[(size_t)b * EDGE_BUCKET + k];
            if (s.parent != NONE) continue;
            const NodeRec& r = nodes[c];
            s = EdgeSlot{parent_[c], via_[c], c, r.flags, r.plus_child, r.hash_fid, r.term_fid, plus_flags(c)};
            edge_slot_[c] = (uint32_t)((size_t)b * EDGE_BUCKET + k);
            placed = true;
            break;
          }
      }
  }
  phase("edge table");
  dirty_.clear();
  dirty_.nodes_full = dirty_.edges_full = dirty_.dict_full = dirty_.words_full = true;
  return 0;
}

// Open-addressing map built from n distinct keys in parallel: the payload of
// key i is i; a slot range per thread, the probes that run past a range
// placed afterwards (the linear-probing invariant holds: every slot between
// a key's home and its slot is full).
void IndexMap::bulk_build(const std::vector<uint64_t>& h, unsigned nt) {
  const size_t n = h.size();
  size_t cap = 16;
  while (cap < 4 * n) cap <<= 1;   // as insert(): grows to 4x at half load
  slots_.assign(cap, Slot{0, 0, 0});
  n_ = n;
  tombs_ = 0;
  const size_t m = cap - 1;
  const unsigned T = n < 65536 ? 1u : nt;
  std::vector<std::vector<uint32_t>> spill(T);
  auto bins = bin_by_range(n, T, nt, [&](size_t i) -> uint32_t { return (uint32_t)((h[i] & m) * T / cap); });
  parallel_for(T, T, [&](size_t lo, size_t hi, unsigned) {
    for (size_t t = lo; t < hi; ++t) {
      const size_t s1 = cap * (t + 1) / T;
      for (uint32_t i : bins[t]) {
        size_t j = h[i] & m;
        while (j < s1 && slots_[j].state == 1) ++j;
        if (j < s1) slots_[j] = Slot{h[i], i, 1};
        else spill[t].push_back(i);
      }
    }
  });
  for (auto& sp : spill)
    for (uint32_t i : sp) {
      size_t j = h[i] & m;
      while (slots_[j].state == 1) j = (j + 1) & m;
      slots_[j] = Slot{h[i], i, 1};
    }
}

}  // namespace egm
