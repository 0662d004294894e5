// egm_common.h — layouts and hash functions shared by the host table builder
// (egm_table.cpp, g++) and the gfx950 kernels (egm_kernels.hip, hipcc).
//
// The reference keeps the wildcard index as string keys {Prefix,0}/{Filter,1}
// in a mnesia ordered_set (apps/emqx/src/emqx_trie.erl:45-51,61-71) and probes
// it once per visited prefix (:192-206).  Here the same filter set is a
// word-level trie flattened into three HBM arrays:
//
//   nodes[]  16 B  {plus_child, hash_fid, term_fid, flags}
//   edges[]  64 B buckets of two 32 B slots {parent, word_id, child, flags,
//            child's plus_child, hash_fid, term_fid, flags of the child's '+' child}
//   dict[]   32 B slots {hash64, word_id, len, inline bytes[16]}  (+ blob for long words)
//
// A literal transition is one bucket read keyed by (node, word_id); word ids
// come from the dictionary with byte-exact verification, so a 64-bit hash
// collision can never create a false edge.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define EGM_HD __host__ __device__ __forceinline__
#else
#define EGM_HD inline
#endif

namespace egm {

constexpr uint32_t NONE = 0xFFFFFFFFu;        // empty id / "no child"
constexpr uint32_t TOMB = 0xFFFFFFFEu;        // deleted edge slot (parent field)

// word ids reserved for topic words that are not literal dictionary words
constexpr uint32_t WID_NONE = 0xFFFFFFFFu;    // literal word absent from every filter
constexpr uint32_t WID_PLUS = 0xFFFFFFFDu;    // the word '+'
constexpr uint32_t WID_HASH = 0xFFFFFFFCu;    // the word '#'
constexpr uint32_t WID_MAX  = 0xFFFFFFF0u;    // real ids are < WID_MAX

// node flag bits (4 bits, carried in work items and edge slots)
constexpr uint32_t F_LIT  = 1u;   // has >= 1 literal child
constexpr uint32_t F_PLUS = 2u;   // has a '+' child
constexpr uint32_t F_HASH = 4u;   // "P/#" is a filter (hash_fid valid)
constexpr uint32_t F_TERM = 8u;   // "P" itself is a filter (term_fid valid)

// Bits [4:32) of a node's flags word are a signature of its literal children:
// bit SIG_SHIFT + sig_index(w) is set for every literal child word w (set on
// insert, recomputed exactly by relayout; a stale extra bit after a delete
// only costs a probe).  A walker skips the edge probe of a word whose bit is
// clear: more than half of all literal probes of the C2 workload find no edge.
constexpr uint32_t F_BASIC = 0xFu;
constexpr uint32_t SIG_SHIFT = 4;
constexpr uint32_t SIG_BITS = 28;

// per-topic flags (egm_result.flags)
constexpr uint8_t TF_WILDCARD = 1;   // topic has a '+' or '#' word (emqx_topic.erl:53-62)
constexpr uint8_t TF_DOLLAR   = 2;   // first word starts with '$' (emqx_trie.erl:208-215)
constexpr uint8_t TF_HEAVY    = 4;   // matched by the overflow (heavy) kernel
constexpr uint8_t TF_ERROR    = 8;   // could not be matched (see egm_last_error)
constexpr uint8_t TF_SKIP     = 16;  // padding past a device-side topic count (egm_match_device_counted): no walk

#ifndef EGM_EDGE_BUCKET
#define EGM_EDGE_BUCKET 2
#endif
// Slots per bucket, the unit a key is hashed to (a walker reads one 64-B line
// = two slots at a time, starting at the key's bucket, then the next lines).
// Round 6: 2 (a key's home is any 64-B line) instead of 4 (a 128-B bucket,
// homes on every other line): at the same table size and slot load, fewer
// keys sit past their home line — C2 probes that read a second line 56.3 M ->
// 22.8 M per batch, k_walk 6.27 -> 5.86 ms; C3 166 M -> 60 M, 53.7 -> 48.9 ms.
constexpr int EDGE_BUCKET = EGM_EDGE_BUCKET;
static_assert(EDGE_BUCKET == 2 || EDGE_BUCKET == 4, "a bucket is one or two 64-B lines");
#ifndef EGM_EDGE_SPREAD
#define EGM_EDGE_SPREAD 2
#endif
// Edge slots per literal edge, at least: the table's slot load stays in
// (1/(2·SPREAD), 1/SPREAD].  A probe whose key is not in its bucket's first
// two slots (or, for an absent key, whose first two slots are both taken)
// costs the walking wave a second dependent round trip.
constexpr uint32_t EDGE_SPREAD = EGM_EDGE_SPREAD;

struct NodeRec {          // 16 B, one dwordx4 load
  uint32_t plus_child;    // node reached by '+', or NONE
  uint32_t hash_fid;      // filter id of "P/#", or NONE
  uint32_t term_fid;      // filter id of "P", or NONE
  uint32_t flags;         // F_* bits of this node
};

// A literal edge carries a copy of its child's record, so a literal
// transition is a single 64-B line read (a bucket of two 32 B slots).
struct EdgeSlot {         // 32 B
  uint32_t parent;        // NONE = empty, TOMB = deleted
  uint32_t wid;
  uint32_t child;
  uint32_t child_flags;
  uint32_t child_plus;    // copy of nodes[child].plus_child
  uint32_t child_hash;    // copy of nodes[child].hash_fid
  uint32_t child_term;    // copy of nodes[child].term_fid
  uint32_t child_pflags;  // flags of nodes[child].plus_child (0: none) — the walker skips reading
                          // a '+' child's record that would emit and push nothing (round 5)
};

struct DictSlot {         // 32 B
  uint64_t hash;
  uint32_t wid;           // NONE = empty
  uint32_t len;
  uint8_t inl[16];        // first min(len,16) bytes
};

static_assert(sizeof(NodeRec) == 16, "NodeRec");
static_assert(sizeof(EdgeSlot) == 32, "EdgeSlot");
static_assert(sizeof(DictSlot) == 32, "DictSlot");

// ---- hashing (identical on host and device) --------------------------------
constexpr uint64_t FNV_BASIS = 0xcbf29ce484222325ull;
constexpr uint64_t FNV_PRIME = 0x100000001b3ull;

EGM_HD uint64_t mix64(uint64_t x) {   // murmur3 fmix64
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Word hash: 4-byte little-endian chunks, each folded in with one 64-bit
// multiply (a quarter of byte-wise FNV-1a's serial multiplies); the tail chunk
// is zero-padded and the length is mixed in last, so "ab" != "ab\0".
EGM_HD uint64_t hash_chunk(uint64_t h, uint32_t c) { return (h ^ c) * FNV_PRIME; }

EGM_HD uint64_t word_hash_finish(uint64_t h, uint32_t len) {
  return mix64(h ^ ((uint64_t)len << 56));
}

EGM_HD uint64_t word_hash(const uint8_t* p, uint32_t len) {
  uint64_t h = FNV_BASIS;
  uint32_t i = 0;
  for (; i + 4 <= len; i += 4)
    h = hash_chunk(h, (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16) |
                          ((uint32_t)p[i + 3] << 24));
  if (i < len) {
    uint32_t c = 0;
    for (uint32_t k = 0; i + k < len; ++k) c |= (uint32_t)p[i + k] << (8 * k);
    h = hash_chunk(h, c);
  }
  return word_hash_finish(h, len);
}

// The per-pop hashes.  Round 4 tried 32-bit forms (two multiplies each
// instead of fmix64's ~27 VALU per pop): EGM_EDGE_HASH32 / EGM_SIG_HASH32,
// A/B only (profiles/r4_*): the 32-bit edge hash made the C2 walk 4 % slower.
EGM_HD uint32_t sig_index(uint32_t wid) {   // 0 .. SIG_BITS-1
#ifdef EGM_SIG_HASH32
  const uint32_t h = wid * 0x9E3779B1u;   // Fibonacci hashing of the word id
#else
  const uint32_t h = (uint32_t)(mix64(0x9E3779B97F4A7C15ull ^ wid) >> 32);
#endif
  return (uint32_t)(((uint64_t)h * SIG_BITS) >> 32);
}

EGM_HD uint32_t sig_bit(uint32_t wid) {   // literal-child signature bit of a word
  return 1u << (SIG_SHIFT + sig_index(wid));
}

EGM_HD uint32_t edge_bucket(uint32_t parent, uint32_t wid, uint32_t mask) {
#ifdef EGM_EDGE_HASH32
  uint32_t h = (parent * 0x9E3779B1u) ^ wid;   // for a fixed parent, a bijection of the word
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h & mask;
#else
  return (uint32_t)(mix64(((uint64_t)parent << 32) | wid) & mask);
#endif
}

// Multi-GPU prefix partition (SURVEY §8e "partition by root word", two words
// deep: C2's level-0 vocabulary has 16 Zipf-distributed words).  The key of a
// filter or topic is its bytes up to (not including) the second '/': "a/b" for
// a/b/..., the whole name for a one-level one.  Every topic a filter with
// literal first two words can match has that filter's key; a filter whose
// first or second word is '+' or '#' can match any key and is replicated.
// Keys hash into n_vparts virtual partitions, mapped to ranks by the host.
EGM_HD uint32_t prefix_key_len(const uint8_t* p, uint32_t len) {
  uint32_t slashes = 0;
  for (uint32_t i = 0; i < len; ++i)
    if (p[i] == '/' && ++slashes == 2) return i;
  return len;
}

EGM_HD uint32_t prefix_vpart(const uint8_t* p, uint32_t len, uint32_t n_vparts) {
  return (uint32_t)(word_hash(p, prefix_key_len(p, len)) % n_vparts);
}

// A filter that must live on every rank: '+' or '#' as its first or second word.
EGM_HD bool prefix_replicated(const uint8_t* p, uint32_t len) {
  uint32_t ws = 0, level = 0;
  for (uint32_t i = 0; i <= len && level < 2; ++i) {
    if (i < len && p[i] != '/') continue;
    if (i - ws == 1 && (p[ws] == '+' || p[ws] == '#')) return true;
    ws = i + 1;
    ++level;
  }
  return false;
}

// filter -> shard assignment for multi-GPU filter sharding
EGM_HD uint32_t filter_shard(const uint8_t* p, uint32_t len, uint32_t n_shards) {
  return (uint32_t)(word_hash(p, len) % n_shards);
}

}  // namespace egm
