// egm_table.cpp — host filter table (see egm_table.h).
#include "egm_table.h"

#include <string.h>

#include <algorithm>

namespace egm {

// ---------------------------------------------------------------- IndexMap --
static size_t pow2_at_least(size_t n) {
  size_t c = 16;
  while (c < n) c <<= 1;
  return c;
}

void IndexMap::reserve(size_t n) {
  if (slots_.size() < 2 * n) grow(2 * n);
}

void IndexMap::grow(size_t want) {
  std::vector<Slot> old;
  old.swap(slots_);
  slots_.assign(pow2_at_least(want), Slot{0, 0, 0});
  n_ = 0;
  tombs_ = 0;
  for (const Slot& s : old)
    if (s.state == 1) insert(s.h, s.v);
}

template <class Eq>
uint32_t IndexMap::find(uint64_t h, Eq eq) const {
  if (slots_.empty()) return NONE;
  size_t m = slots_.size() - 1, i = h & m;
  for (;;) {
    const Slot& s = slots_[i];
    if (s.state == 0) return NONE;
    if (s.state == 1 && s.h == h && eq(s.v)) return s.v;
    i = (i + 1) & m;
  }
}

void IndexMap::insert(uint64_t h, uint32_t v) {
  if ((n_ + tombs_ + 1) * 2 > slots_.size()) grow(std::max<size_t>(32, (n_ + 1) * 4));
  size_t m = slots_.size() - 1, i = h & m;
  while (slots_[i].state == 1) i = (i + 1) & m;
  if (slots_[i].state == 2) --tombs_;
  slots_[i] = Slot{h, v, 1};
  ++n_;
}

template <class Eq>
bool IndexMap::erase(uint64_t h, Eq eq) {
  if (slots_.empty()) return false;
  size_t m = slots_.size() - 1, i = h & m;
  for (;;) {
    Slot& s = slots_[i];
    if (s.state == 0) return false;
    if (s.state == 1 && s.h == h && eq(s.v)) {
      s.state = 2;
      --n_;
      ++tombs_;
      return true;
    }
    i = (i + 1) & m;
  }
}

// ---------------------------------------------------------------- DirtyLog --
static void append_or_full(std::vector<uint32_t>& v, bool& full, const std::vector<uint32_t>& o) {
  if (full) return;
  v.insert(v.end(), o.begin(), o.end());
}

void DirtyLog::merge(const DirtyLog& o) {
  nodes_full |= o.nodes_full;
  edges_full |= o.edges_full;
  dict_full |= o.dict_full;
  words_full |= o.words_full;
  append_or_full(nodes, nodes_full, o.nodes);
  append_or_full(edges, edges_full, o.edges);
  append_or_full(dict, dict_full, o.dict);
  if (nodes_full) std::vector<uint32_t>().swap(nodes);
  if (edges_full) std::vector<uint32_t>().swap(edges);
  if (dict_full) std::vector<uint32_t>().swap(dict);
}

void DirtyLog::clear() {
  std::vector<uint32_t>().swap(nodes);
  std::vector<uint32_t>().swap(edges);
  std::vector<uint32_t>().swap(dict);
  nodes_full = edges_full = dict_full = words_full = false;
}

// A log longer than a quarter of its array costs more to apply than a copy.
void HostTable::mark_node(uint32_t n) {
  if (dirty_.nodes_full) return;
  dirty_.nodes.push_back(n);
  if (dirty_.nodes.size() > nodes.size() / 4 + 4096) {
    dirty_.nodes_full = true;
    std::vector<uint32_t>().swap(dirty_.nodes);
  }
}

void HostTable::mark_edge(uint32_t s) {
  if (dirty_.edges_full) return;
  dirty_.edges.push_back(s);
  if (dirty_.edges.size() > edges.size() / 4 + 4096) {
    dirty_.edges_full = true;
    std::vector<uint32_t>().swap(dirty_.edges);
  }
}

DirtyLog HostTable::take_dirty() {
  DirtyLog d;
  std::swap(d, dirty_);
  return d;
}

// --------------------------------------------------------------- HostTable --
HostTable::HostTable() { clear(); }

void HostTable::clear() {
  dirty_.clear();
  dirty_.nodes_full = dirty_.edges_full = dirty_.dict_full = dirty_.words_full = true;
  nodes.clear();
  hash_child.clear();
  parent_.clear();
  via_.clear();
  ref_.clear();
  lit_count_.clear();
  sig_.clear();
  edge_slot_.clear();
  free_nodes_.clear();
  n_live_nodes_ = 0;
  edges.assign(16 * EDGE_BUCKET, EdgeSlot{NONE, 0, 0, 0, NONE, NONE, NONE, 0});
  n_edges_ = n_edge_tombs_ = 0;
  dict.assign(64, DictSlot{0, NONE, 0, {0}});
  dict_blob.clear();
  dict_off.assign(1, 0);
  n_dict_used_ = 0;
  fblob_.clear();
  foff_.assign(1, 0);
  ffid_.clear();
  falive_.clear();
  by_bytes_ = IndexMap();
  by_fid_ = IndexMap();
  n_filters_ = 0;
  next_fid_ = 0;
  new_node(NONE, NONE);  // root = node 0
}

uint32_t HostTable::new_node(uint32_t parent, uint32_t via) {
  uint32_t n;
  if (!free_nodes_.empty()) {
    n = free_nodes_.back();
    free_nodes_.pop_back();
  } else {
    n = (uint32_t)nodes.size();
    nodes.push_back({});
    hash_child.push_back(NONE);
    parent_.push_back(NONE);
    via_.push_back(NONE);
    ref_.push_back(0);
    lit_count_.push_back(0);
    sig_.push_back(0);
    edge_slot_.push_back(NONE);
  }
  nodes[n] = NodeRec{NONE, NONE, NONE, 0};
  hash_child[n] = NONE;
  parent_[n] = parent;
  via_[n] = via;
  ref_[n] = 0;
  lit_count_[n] = 0;
  sig_[n] = 0;
  edge_slot_[n] = NONE;
  ++n_live_nodes_;
  mark_node(n);
  return n;
}

void HostTable::free_node(uint32_t n) {
  nodes[n] = NodeRec{NONE, NONE, NONE, 0};
  hash_child[n] = NONE;
  parent_[n] = NONE;
  via_[n] = NONE;
  edge_slot_[n] = NONE;
  free_nodes_.push_back(n);
  --n_live_nodes_;
  mark_node(n);
}

uint32_t HostTable::own_flags(uint32_t n) const {
  const NodeRec& r = nodes[n];
  return (lit_count_[n] ? F_LIT | sig_[n] : 0u) | (r.plus_child != NONE ? F_PLUS : 0u) |
         (r.hash_fid != NONE ? F_HASH : 0u) | (r.term_fid != NONE ? F_TERM : 0u);
}

// Recompute n's flags and republish its record where a walker picks it up:
// the literal edge slot that reaches n carries a copy (the '+' child and the
// root are read from nodes[] itself).
void HostTable::update_flags(uint32_t n) {
  NodeRec& r = nodes[n];
  r.flags = own_flags(n);
  mark_node(n);
  // a '+' child's flags are also carried by the slot that reaches its parent
  const uint32_t par = parent_[n];
  if (par != NONE && via_[n] == WID_PLUS && parent_[par] != NONE && via_[par] < WID_MAX) {
    mark_edge(edge_slot_[par]);
    edges[edge_slot_[par]].child_pflags = r.flags;
  }
  if (par == NONE || via_[n] >= WID_MAX) return;
  mark_edge(edge_slot_[n]);
  EdgeSlot& s = edges[edge_slot_[n]];
  s.child_flags = r.flags;
  s.child_plus = r.plus_child;
  s.child_hash = r.hash_fid;
  s.child_term = r.term_fid;
  s.child_pflags = plus_flags(n);
}

uint32_t HostTable::plus_flags(uint32_t n) const {
  return nodes[n].plus_child != NONE ? nodes[nodes[n].plus_child].flags : 0u;
}

// ---- dictionary ----
uint32_t HostTable::dict_find(const uint8_t* p, uint32_t len) const {
  uint64_t h = word_hash(p, len);
  uint32_t m = dict_mask(), i = (uint32_t)(h & m);
  for (;;) {
    const DictSlot& s = dict[i];
    if (s.wid == NONE) return NONE;
    if (s.hash == h && s.len == len && memcmp(dict_blob.data() + dict_off[s.wid], p, len) == 0)
      return s.wid;
    i = (i + 1) & m;
  }
}

void HostTable::dict_rehash(size_t cap) {
  std::vector<DictSlot> old;
  old.swap(dict);
  dict.assign(cap, DictSlot{0, NONE, 0, {0}});
  dirty_.dict_full = true;
  std::vector<uint32_t>().swap(dirty_.dict);
  uint32_t m = (uint32_t)cap - 1;
  for (const DictSlot& s : old) {
    if (s.wid == NONE) continue;
    uint32_t i = (uint32_t)(s.hash & m);
    while (dict[i].wid != NONE) i = (i + 1) & m;
    dict[i] = s;
  }
}

uint32_t HostTable::dict_add(const uint8_t* p, uint32_t len) {
  uint32_t w = dict_find(p, len);
  if (w != NONE) return w;
  if ((size_t)(n_dict_used_ + 1) * 2 > dict.size()) dict_rehash(dict.size() * 2);
  w = (uint32_t)dict_off.size() - 1;
  dict_blob.insert(dict_blob.end(), p, p + len);
  dict_off.push_back(dict_blob.size());
  uint64_t h = word_hash(p, len);
  uint32_t m = dict_mask(), i = (uint32_t)(h & m);
  while (dict[i].wid != NONE) i = (i + 1) & m;
  DictSlot s{h, w, len, {0}};
  memcpy(s.inl, p, len < 16 ? len : 16);
  dict[i] = s;
  if (!dirty_.dict_full) dirty_.dict.push_back(i);
  ++n_dict_used_;
  return w;
}

// ---- edges ----
uint32_t HostTable::edge_find(uint32_t parent, uint32_t wid) const {
  uint32_t m = edge_mask(), b = edge_bucket(parent, wid, m);
  for (;;) {
    bool has_empty = false;
    for (int k = 0; k < EDGE_BUCKET; ++k) {
      const EdgeSlot& s = edges[(size_t)b * EDGE_BUCKET + k];
      if (s.parent == parent && s.wid == wid) return (uint32_t)(b * EDGE_BUCKET + k);
      if (s.parent == NONE) has_empty = true;
    }
    if (has_empty) return NONE;
    b = (b + 1) & m;
  }
}

uint32_t HostTable::edge_insert(uint32_t parent, uint32_t wid, uint32_t child, uint32_t cflags) {
  size_t nb = edges.size() / EDGE_BUCKET;
  if ((n_edges_ + n_edge_tombs_ + 1) * EDGE_SPREAD > nb * EDGE_BUCKET) {
    size_t want = nb;
    while ((n_edges_ + 1) * EDGE_SPREAD > want * EDGE_BUCKET / 2) want *= 2;  // rehash to <= half the max load
    edge_rehash(want);
  }
  uint32_t m = edge_mask(), b = edge_bucket(parent, wid, m);
  for (;;) {
    for (int k = 0; k < EDGE_BUCKET; ++k) {
      EdgeSlot& s = edges[(size_t)b * EDGE_BUCKET + k];
      if (s.parent == NONE || s.parent == TOMB) {
        if (s.parent == TOMB) --n_edge_tombs_;
        const NodeRec& r = nodes[child];
        s = EdgeSlot{parent, wid, child, cflags, r.plus_child, r.hash_fid, r.term_fid, plus_flags(child)};
        ++n_edges_;
        mark_edge((uint32_t)(b * EDGE_BUCKET + k));
        return (uint32_t)(b * EDGE_BUCKET + k);
      }
    }
    b = (b + 1) & m;
  }
}

void HostTable::edge_rehash(size_t n_buckets) {
  std::vector<EdgeSlot> old;
  old.swap(edges);
  edges.assign(n_buckets * EDGE_BUCKET, EdgeSlot{NONE, 0, 0, 0, NONE, NONE, NONE, 0});
  n_edges_ = n_edge_tombs_ = 0;
  dirty_.edges_full = true;
  std::vector<uint32_t>().swap(dirty_.edges);
  for (const EdgeSlot& s : old) {
    if (s.parent == NONE || s.parent == TOMB) continue;
    uint32_t slot = edge_insert(s.parent, s.wid, s.child, s.child_flags);
    edge_slot_[s.child] = slot;
  }
}

// ---- filters ----
uint32_t HostTable::find_local(const uint8_t* p, uint32_t len, uint64_t h) const {
  return by_bytes_.find(h, [&](uint32_t li) {
    uint64_t a = foff_[li], b = foff_[li + 1];
    return falive_[li] && b - a == len && memcmp(fblob_.data() + a, p, len) == 0;
  });
}

uint32_t HostTable::lookup(const uint8_t* p, uint32_t len) const {
  uint32_t li = find_local(p, len, word_hash(p, len));
  return li == NONE ? NONE : ffid_[li];
}

bool HostTable::id_in_use(uint32_t fid) const {
  return by_fid_.find(mix64(fid), [&](uint32_t x) { return falive_[x] && ffid_[x] == fid; }) != NONE;
}

const uint8_t* HostTable::filter_bytes(uint32_t fid, uint32_t* len) const {
  uint32_t li = by_fid_.find(mix64(fid), [&](uint32_t x) { return falive_[x] && ffid_[x] == fid; });
  if (li == NONE) return nullptr;
  *len = (uint32_t)(foff_[li + 1] - foff_[li]);
  return fblob_.data() + foff_[li];
}

int HostTable::insert(const uint8_t* p, uint32_t len, uint32_t fid, uint32_t* out_fid) {
  uint64_t h = word_hash(p, len);
  uint32_t li = find_local(p, len, h);
  if (li != NONE) {  // emqx_trie.erl:84-85 — already inserted
    if (out_fid) *out_fid = ffid_[li];
    return 1;
  }
  if (fid == NONE) fid = next_fid_;
  if (fid >= WID_MAX) return -1;
  if (by_fid_.find(mix64(fid), [&](uint32_t x) { return falive_[x] && ffid_[x] == fid; }) != NONE)
    return -2;  // id already used by another filter
  if (fid >= next_fid_) next_fid_ = fid + 1;

  // walk/create the path (one node per word; '+' and '#' are dedicated edges)
  uint32_t cur = 0;
  uint32_t start = 0;
  bool last_hash = false;
  for (uint32_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    const uint8_t* w = p + start;
    uint32_t wl = i - start;
    start = i + 1;
    uint32_t c;
    last_hash = false;
    if (wl == 1 && w[0] == '+') {
      c = nodes[cur].plus_child;
      if (c == NONE) {
        c = new_node(cur, WID_PLUS);
        nodes[cur].plus_child = c;
        update_flags(c);
        update_flags(cur);
      }
    } else if (wl == 1 && w[0] == '#') {
      c = hash_child[cur];
      if (c == NONE) {
        c = new_node(cur, WID_HASH);
        hash_child[cur] = c;
        mark_node(cur);
      }
      last_hash = true;
    } else {
      uint32_t wid = dict_add(w, wl);
      uint32_t s = edge_find(cur, wid);
      if (s == NONE) {
        c = new_node(cur, wid);
        s = edge_insert(cur, wid, c, 0);
        edge_slot_[c] = s;
        ++lit_count_[cur];
        sig_[cur] |= sig_bit(wid);
        update_flags(cur);
      } else {
        c = edges[s].child;
      }
    }
    ++ref_[c];
    cur = c;
  }
  ++ref_[0];
  nodes[cur].term_fid = fid;
  update_flags(cur);
  if (last_hash) {  // "P/#": the parent emits it at every level >= |P|
    uint32_t par = parent_[cur];
    nodes[par].hash_fid = fid;
    update_flags(par);
  }

  uint32_t nli = (uint32_t)ffid_.size();
  fblob_.insert(fblob_.end(), p, p + len);
  foff_.push_back(fblob_.size());
  ffid_.push_back(fid);
  falive_.push_back(1);
  by_bytes_.insert(h, nli);
  by_fid_.insert(mix64(fid), nli);
  ++n_filters_;
  if (out_fid) *out_fid = fid;
  return 0;
}

int HostTable::remove(const uint8_t* p, uint32_t len) {
  uint64_t h = word_hash(p, len);
  uint32_t li = find_local(p, len, h);
  if (li == NONE) return 1;  // emqx_trie.erl:93-95 — not present: ok
  uint32_t fid = ffid_[li];

  std::vector<uint32_t> path;
  uint32_t cur = 0, start = 0;
  for (uint32_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    const uint8_t* w = p + start;
    uint32_t wl = i - start;
    start = i + 1;
    if (wl == 1 && w[0] == '+') cur = nodes[cur].plus_child;
    else if (wl == 1 && w[0] == '#') cur = hash_child[cur];
    else cur = edges[edge_find(cur, dict_find(w, wl))].child;
    path.push_back(cur);
  }
  uint32_t term = path.back();
  nodes[term].term_fid = NONE;
  update_flags(term);
  if (via_[term] == WID_HASH) {
    nodes[parent_[term]].hash_fid = NONE;
    update_flags(parent_[term]);
  }
  for (size_t k = path.size(); k-- > 0;) {
    uint32_t n = path[k];
    if (--ref_[n] != 0) continue;
    uint32_t par = parent_[n];
    if (via_[n] == WID_PLUS) {
      nodes[par].plus_child = NONE;
    } else if (via_[n] == WID_HASH) {
      hash_child[par] = NONE;
    } else {
      edges[edge_slot_[n]].parent = TOMB;
      mark_edge(edge_slot_[n]);
      --n_edges_;
      ++n_edge_tombs_;
      --lit_count_[par];
    }
    free_node(n);
    update_flags(par);
  }
  --ref_[0];

  by_bytes_.erase(h, [&](uint32_t x) { return x == li; });
  by_fid_.erase(mix64(fid), [&](uint32_t x) { return x == li; });
  falive_[li] = 0;
  --n_filters_;
  return 0;
}

// Renumber live nodes breadth-first from the root so that every level is a
// contiguous id range (the hot upper levels then share cache lines), and
// rebuild the edge table at <= 25 % load.
void HostTable::relayout() {
  dirty_.nodes_full = dirty_.edges_full = true;   // every node id changes
  std::vector<uint32_t>().swap(dirty_.nodes);
  std::vector<uint32_t>().swap(dirty_.edges);
  const uint32_t N = (uint32_t)nodes.size();
  // children lists via counting sort by parent
  std::vector<uint32_t> cnt(N + 1, 0);
  for (uint32_t n = 1; n < N; ++n)
    if (parent_[n] != NONE) ++cnt[parent_[n] + 1];
  for (uint32_t i = 0; i < N; ++i) cnt[i + 1] += cnt[i];
  std::vector<uint32_t> kids(cnt[N]);
  {
    std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
    for (uint32_t n = 1; n < N; ++n)
      if (parent_[n] != NONE) kids[pos[parent_[n]]++] = n;
  }
  std::vector<uint32_t> order;
  order.reserve(n_live_nodes_);
  std::vector<uint32_t> newid(N, NONE);
  order.push_back(0);
  newid[0] = 0;
  for (size_t qi = 0; qi < order.size(); ++qi) {
    uint32_t n = order[qi];
    for (uint32_t k = cnt[n]; k < cnt[n + 1]; ++k) {
      uint32_t c = kids[k];
      newid[c] = (uint32_t)order.size();
      order.push_back(c);
    }
  }
  const uint32_t L = (uint32_t)order.size();
  std::vector<NodeRec> nn(L);
  std::vector<uint32_t> nhc(L), npar(L), nvia(L), nref(L), nlit(L);
  for (uint32_t i = 0; i < L; ++i) {
    uint32_t o = order[i];
    NodeRec r = nodes[o];
    if (r.plus_child != NONE) r.plus_child = newid[r.plus_child];
    nn[i] = r;
    nhc[i] = hash_child[o] == NONE ? NONE : newid[hash_child[o]];
    npar[i] = parent_[o] == NONE ? NONE : newid[parent_[o]];
    nvia[i] = via_[o];
    nref[i] = ref_[o];
    nlit[i] = lit_count_[o];
  }
  std::vector<uint32_t>().swap(sig_);
  sig_.assign(L, 0);
  nodes.swap(nn);
  hash_child.swap(nhc);
  parent_.swap(npar);
  via_.swap(nvia);
  ref_.swap(nref);
  lit_count_.swap(nlit);
  edge_slot_.assign(L, NONE);
  free_nodes_.clear();
  n_live_nodes_ = L;
  // room to grow: route churn after a rebuild appends nodes without moving
  // multi-GB vectors
  const size_t room = L + L / 8 + 1024;
  for (auto* v : {&hash_child, &parent_, &via_, &ref_, &lit_count_, &sig_, &edge_slot_}) v->reserve(room);
  nodes.reserve(room);

  size_t nb = 16;
  while (nb * EDGE_BUCKET < (size_t)n_edges_ * EDGE_SPREAD) nb <<= 1;  // slot load in (1/(2 SPREAD), 1/SPREAD]
  std::vector<EdgeSlot> old;
  old.swap(edges);
  edges.assign(nb * EDGE_BUCKET, EdgeSlot{NONE, 0, 0, 0, NONE, NONE, NONE, 0});
  n_edges_ = n_edge_tombs_ = 0;
  // insert in BFS order of the child so that bucket contents follow the levels
  std::vector<EdgeSlot> live;
  live.reserve(old.size());
  for (const EdgeSlot& s : old)
    if (s.parent != NONE && s.parent != TOMB) live.push_back(s);
  for (EdgeSlot& s : live) {
    s.parent = newid[s.parent];
    s.child = newid[s.child];
  }
  std::sort(live.begin(), live.end(), [](const EdgeSlot& a, const EdgeSlot& b) { return a.child < b.child; });
  // exact literal-child signatures, then every record and slot copy refreshed
  for (const EdgeSlot& s : live) sig_[s.parent] |= sig_bit(s.wid);
  for (uint32_t n = 0; n < L; ++n) nodes[n].flags = own_flags(n);
  for (const EdgeSlot& s : live)
    edge_slot_[s.child] = edge_insert(s.parent, s.wid, s.child, nodes[s.child].flags);
}

}  // namespace egm
