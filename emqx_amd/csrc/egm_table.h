// egm_table.h — host-side filter table: the mutable word-level trie that is
// uploaded to HBM as the NFA graph (egm_common.h layouts).
//
// Semantics mirror the reference's trie content operations:
//   insert/1  apps/emqx/src/emqx_trie.erl:82-87   (idempotent per filter)
//   delete/1  apps/emqx/src/emqx_trie.erl:91-96   (no-op when absent)
//   empty/0   apps/emqx/src/emqx_trie.erl:118
// The reference ref-counts prefix keys (:171-188); here every trie node counts
// the filters passing through it and is unlinked when the count reaches zero,
// which is the same invariant (a prefix exists iff some live filter has it).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "egm_common.h"

namespace egm {

// Open-addressing map from a 64-bit hash to a u32 payload; equality of the
// underlying keys is decided by a caller-supplied predicate.
class IndexMap {
 public:
  void reserve(size_t n);
  template <class Eq>
  uint32_t find(uint64_t h, Eq eq) const;
  void insert(uint64_t h, uint32_t v);           // caller guarantees absence
  // from n distinct keys at once (payload = key index), in parallel (egm_bulk.cpp)
  void bulk_build(const std::vector<uint64_t>& h, unsigned threads);
  template <class Eq>
  bool erase(uint64_t h, Eq eq);
  size_t size() const { return n_; }

 private:
  struct Slot { uint64_t h; uint32_t v; uint32_t state; };  // state 0 empty, 1 full, 2 tomb
  std::vector<Slot> slots_;
  size_t n_ = 0, tombs_ = 0;
  void grow(size_t want);
};

// Records of the device image written since the last take_dirty(): what an
// epoch commit has to patch into a device copy of the previous image instead
// of re-uploading it (the reference mutates its trie one
// key at a time inside mnesia transactions, emqx_trie.erl:171-188).
// Indices may repeat; *_full means the array was rebuilt (rehash, relayout,
// clear) and must be copied whole.  dict_blob/dict_off only ever grow between
// clears, so their tails are found from the sizes.
struct DirtyLog {
  std::vector<uint32_t> nodes;   // indices into nodes[] and hash_child[]
  std::vector<uint32_t> edges;   // edge slot indices
  std::vector<uint32_t> dict;    // dictionary slot indices
  bool nodes_full = false, edges_full = false, dict_full = false, words_full = false;
  void merge(const DirtyLog& o);
  void clear();
  bool empty() const {
    return nodes.empty() && edges.empty() && dict.empty() && !nodes_full && !edges_full && !dict_full &&
           !words_full;
  }
};

class HostTable {
 public:
  HostTable();

  // status: 0 inserted, 1 already present (out_fid = existing id), <0 error
  int insert(const uint8_t* p, uint32_t len, uint32_t fid, uint32_t* out_fid);
  // status: 0 removed, 1 absent
  int remove(const uint8_t* p, uint32_t len);
  // filter id for bytes, or NONE
  uint32_t lookup(const uint8_t* p, uint32_t len) const;
  // bytes of a filter id (nullptr if unknown)
  const uint8_t* filter_bytes(uint32_t fid, uint32_t* len) const;
  // whether a live filter holds this id
  bool id_in_use(uint32_t fid) const;

  void relayout();          // BFS renumbering of nodes + edge table rebuild
  void clear();
  // clear() + insert() of every filter + relayout(), in parallel (egm_bulk.cpp):
  // ids must be valid and unique, none NONE (validated by the caller).
  // threads 0 = build_threads().  0, or <0 when the table would be too large.
  int bulk_build(const uint8_t* blob, const uint32_t* off, uint32_t n, const uint32_t* ids, unsigned threads);

  uint64_t n_filters() const { return n_filters_; }
  uint32_t n_nodes_live() const { return n_live_nodes_; }
  uint32_t next_fid() const { return next_fid_; }

  // ---- device image (read by egm_capi.cpp at commit) ----
  std::vector<NodeRec> nodes;
  std::vector<uint32_t> hash_child;
  std::vector<EdgeSlot> edges;       // n_buckets * EDGE_BUCKET
  std::vector<DictSlot> dict;
  std::vector<uint8_t> dict_blob;    // all dictionary words back to back
  std::vector<uint64_t> dict_off;    // word id -> offset in dict_blob (n_words + 1)
  uint32_t edge_mask() const { return (uint32_t)(edges.size() / EDGE_BUCKET - 1); }
  uint32_t dict_mask() const { return (uint32_t)(dict.size() - 1); }
  uint32_t n_words() const { return (uint32_t)dict_off.size() - 1; }
  uint64_t n_edges() const { return n_edges_; }

  // exact lookup of a word (host mirror of the device tokeniser's probe)
  uint32_t dict_find(const uint8_t* p, uint32_t len) const;

  // changes since the previous call (see DirtyLog)
  DirtyLog take_dirty();
  // hand a taken log back (a commit that failed after taking it)
  void restore_dirty(const DirtyLog& d) { dirty_.merge(d); }
  const DirtyLog& dirty() const { return dirty_; }

 private:
  DirtyLog dirty_;
  void mark_node(uint32_t n);
  void mark_edge(uint32_t s);
  // host-only per-node bookkeeping
  std::vector<uint32_t> parent_, via_, ref_, lit_count_, edge_slot_, sig_;
  std::vector<uint32_t> free_nodes_;
  uint32_t n_live_nodes_ = 0;
  uint64_t n_edges_ = 0, n_edge_tombs_ = 0;

  // filters: local index -> bytes / fid / alive
  std::vector<uint8_t> fblob_;
  std::vector<uint64_t> foff_;
  std::vector<uint32_t> ffid_;
  std::vector<uint8_t> falive_;
  IndexMap by_bytes_, by_fid_;
  uint64_t n_filters_ = 0;
  uint32_t next_fid_ = 0;
  uint32_t n_dict_used_ = 0;

  uint32_t new_node(uint32_t parent, uint32_t via);
  void free_node(uint32_t n);
  void update_flags(uint32_t n);
  uint32_t own_flags(uint32_t n) const;
  uint32_t plus_flags(uint32_t n) const;   // flags of n's '+' child (0: none)
  uint32_t dict_add(const uint8_t* p, uint32_t len);
  void dict_rehash(size_t cap);
  uint32_t edge_find(uint32_t parent, uint32_t wid) const;
  uint32_t edge_insert(uint32_t parent, uint32_t wid, uint32_t child, uint32_t cflags);
  void edge_rehash(size_t n_buckets);
  uint32_t find_local(const uint8_t* p, uint32_t len, uint64_t h) const;
};

// worker threads for host-side table work: EGM_BUILD_THREADS, else the usable
// CPUs (affinity and cgroup quota), at most 64
unsigned build_threads();

}  // namespace egm
