// egm_kernels.h — host-callable launchers for the gfx950 kernels in
// egm_kernels.hip.  Plain pointers only (device pointers unless stated).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "egm_common.h"

namespace egm {

struct DevTable {                 // one epoch of the filter graph in HBM
  const NodeRec* nodes;
  const uint32_t* hash_child;
  const EdgeSlot* edges;
  uint32_t edge_mask;             // n_buckets - 1
  const DictSlot* dict;
  uint32_t dict_mask;
  const uint8_t* dict_blob;
  const uint64_t* dict_off;
  uint32_t sig_packed;            // word ids < 2^27: the walk stages words as id | sig_index << 27
};

struct MatchStats {               // device-side counters, zeroed per batch
  unsigned long long cursor;      // ids_tmp entries reserved (slabs, incl. slack)
  unsigned long long visited;     // NFA states created (light + heavy)
  unsigned long long pieces;      // pieces reserved (slabs, incl. slack)
  unsigned long long total_ids;   // matched ids in the batch (= row_ptr[n])
  unsigned int n_deferred;        // chunks handed to the heavy kernel
  unsigned int heavy_next;        // heavy work counter
  unsigned int overflow;          // capacity only: bit 0 ids_tmp/pieces full, bit 1 output ids full (rerun bigger)
  unsigned int errors;            // topics the heavy kernel could not walk (never for legal topics)
  unsigned int guard;             // GUARD_* bits: a kernel invariant failed (a bug, never a capacity
                                  // problem; reported instead of hanging the GPU, rows not assembled)
  unsigned int slow_lanes;        // walk literal probes that needed a second bucket read (instrumentation)
  unsigned long long iters;       // walk iterations (instrumentation)
  unsigned long long popped;      // items popped by the walk (lane occupancy = popped / (iters * 64))
  unsigned long long bounded;     // walk iterations whose pop was cut by the stack-room bound (DFS regime)
  unsigned long long lit_probes;  // walk pops that read an edge bucket (instrumentation)
  unsigned long long plus_reads;  // walk pops that read a '+' child's record (instrumentation)
  unsigned int n_deep;            // chunks handed to the deep pass of the walk (more than DEEP_MIN levels)
  unsigned int slow_iters;        // walk iterations in which some lane needed a second bucket read
  unsigned long long rec_cursor;  // flush-record slab u32 reserved (per-wave segments, incl. slack)
};

// Flush records (round 5).  The walk stages a chunk's emits in LDS and writes
// each full stage out as ONE contiguous record appended to the wave's segment
// of the record slab, so its stores are whole lines:
//   [0, 4)        header {n_entries | REC_TAG, 0, 0, 0}
//   [4, 36)       64 x u16: the entries of each of the chunk's topics
//   [36, 36 + n)  the entries' filter ids, grouped by topic (topic 0's first)
//   padded to a whole 128-B line (EGM_REC_ALIGN u32), segments line-aligned too.
// A wave reserves segments of rec_grain u32 (one device-scope atomic each:
// a counter bumped per flush would serialise across the 8 XCDs) and always
// keeps REC_HDR u32 free at a segment's end: when the next record does not
// fit it writes a jump {REC_JUMP, 0, target lo, target hi} there, so a chunk's
// records are a chain from its first one (ChunkRec).  k_rec_rows then moves
// each chunk's ids into the rows, whose starts the scan of the counts gives.
constexpr uint32_t REC_HDR = 4;
constexpr uint32_t REC_IDS = REC_HDR + 32;        // u32 before the ids
constexpr uint32_t REC_TAG = 0x5EC0u << 16;
constexpr uint32_t REC_JUMP = 0x4A4Du << 16;
constexpr uint32_t REC_GRAIN = 16384;             // default u32 per segment (EGM_REC_SEG; a multiple of 32)
constexpr uint32_t REC_DIR = 64;                  // record offsets per chunk in its directory (longer: the chain)
#ifndef EGM_REC_ALIGN
#define EGM_REC_ALIGN 32   // u32: records start on 128-B lines, so no line is shared by two flushes
#endif
__host__ __device__ constexpr uint32_t rec_size(uint32_t n_entries) {
  return (REC_IDS + n_entries + (EGM_REC_ALIGN - 1u)) & ~(EGM_REC_ALIGN - 1u);
}
// Per chunk (uint4): {first record lo, first record hi, records, flags}.
constexpr uint32_t CHUNK_WALKED = 1u;             // walked by k_walk (either pass): its records hold its ids
constexpr uint32_t CHUNK_HEAVY = 2u;              // deferred to k_heavy: its ids are in pieces

struct MatchWork {                // per-batch device workspace
  uint32_t* wid;                  // [blob_bytes + n] word ids, topic t at off[t] + t
  uint32_t* lv;                   // [n] levels
  uint8_t* tfl;                   // [n] TF_* flags
  uint32_t* cnt;                  // [n] ids of each result row (row = walk position if walk_rows, else topic)
  uint32_t walk_rows;             // rows in walk order (MatchOut::topic set): row k = the k-th topic walked
  uint32_t ct;                    // topics per chunk (walk_chunk_topics(n): 64, fewer for small batches)
  uint32_t* rec;                  // [rec_cap] flush records (u32), per-wave segments
  uint64_t rec_cap;
  uint32_t rec_grain;             // u32 per record segment
  uint32_t flush_lim;             // staged emits that trigger a flush (<= WALK_STAGE; smaller: tests)
  uint4* chunks;                  // [n / CHUNK + 1] ChunkRec per chunk
  uint32_t* dir;                  // [(n / CHUNK + 1) * REC_DIR] each chunk's first REC_DIR record offsets / 4
  uint32_t* ids_tmp;              // [ids_cap] ids of heavy topics (one piece each)
  uint64_t ids_cap;
  uint4* pieces;                  // [pieces_cap] {row, count, ids_tmp offset, 0}
  uint64_t pieces_cap;
  uint32_t* deferred;             // [n / CHUNK + 1] chunk ids for the heavy kernel
  uint32_t* deep;                 // [n / CHUNK + 1] chunk ids for the walk's deep pass
  uint4* heavy_stack;             // [heavy_waves * heavy_cap] work stacks of the heavy waves
  uint32_t heavy_waves;
  uint32_t heavy_cap;             // items per heavy wave (>= deepest possible topic + 192)
  uint64_t* tile_sums;            // scan scratch
  MatchStats* stats;
  uint32_t debug;                 // DEBUG_* bits
  // Locality order of the walk: k_tokenise keys each topic
  // by hashes of its first levels' word ids, a radix sort orders the topics'
  // records, and the walk takes its chunks from the sorted records, so the
  // topics a wave walks together share trie paths.
  uint32_t* skey;                 // [n] sort keys (k_tokenise)
  uint32_t* skey_out;             // [n]
  uint64_t* sval;                 // [n] topic records (k_tokenise): t | (D | f << 24 | fixed << 31) << 32
  uint64_t* order;                // [n] the records in walk order (null: walk in input order)
  uint32_t* wfix;                 // [n * FIX_WORDS] first word ids of each topic at a fixed stride
  void* sort_tmp;                 // radix sort scratch
  size_t sort_tmp_bytes;
  uint32_t key_shape;             // key bits per level, nibble l = level l (0: walk in input order)
  const uint32_t* n_live;         // device slot header {count, bytes, overflow, 0} (null: all n live); topics
                                  // past count are skipped padding, and an overflowed header has none live
};

constexpr uint32_t KEY_LEVELS = 4;           // levels hashed into the walk-order key
constexpr uint32_t FIX_WORDS = 8;            // word ids per topic at the fixed stride (deeper: wid[] at off[t] + t)
struct WalkOrderOut {                        // what k_tokenise writes for the sort (all null: nothing)
  uint32_t* key;
  uint64_t* val;
  uint32_t* wfix;
  uint32_t shape;
  const uint32_t* n_live;                    // slot header {count, bytes, overflow, 0}: topics at or past count
                                             // are padding (TF_SKIP), every topic if overflow != 0 (null: none)
};

constexpr uint32_t GUARD_STACK = 4u;         // a push would have overrun a work stack (the pop bound makes it impossible)
constexpr uint32_t GUARD_LOOP = 8u;          // a walk loop ran past its iteration guard

constexpr uint32_t DEBUG_FORCE_HEAVY = 1u;   // every chunk goes to k_heavy (test coverage)
constexpr uint32_t DEBUG_INPUT_ORDER = 4u;   // walk in input order (no locality sort)
constexpr uint32_t DEBUG_FORCE_GUARD = 8u;   // loop guards of 2 iterations: trips the guard (error-path test)

// walk-order key: total bits of a key shape; radix sort scratch bytes for a
// batch of n topics (the hand-written LSD radix sort, egm_kernels.hip walk_sort)
uint32_t walk_key_bits(uint32_t shape);
size_t walk_sort_temp_bytes(uint32_t n, uint32_t shape);
hipError_t launch_walk_sort(uint32_t* keys, uint32_t* keys_tmp, uint64_t* vals, uint64_t* out, void* tmp,
                            MatchStats* stats, uint32_t n, uint32_t kbits, hipStream_t s);

struct MatchOut {                 // CSR result (device)
  uint64_t* row_ptr;              // [n + 1]
  uint32_t* ids;                  // [ids_cap]
  uint64_t ids_cap;
  uint32_t* topic;                // [n] or null.  Set: rows in walk order, topic[k] = the input topic of row k
                                  // (null: row t = input topic t)
};

// launch sizing shared with the host (egm_capi.cpp)
#ifndef EGM_WALK_CHUNK
#define EGM_WALK_CHUNK 64   // topics per chunk taken by a walk wave (and deferred to k_heavy)
#endif
constexpr int WALK_CHUNK = EGM_WALK_CHUNK;
// Topics per chunk for a batch of n (a power of two <= WALK_CHUNK): a small
// batch is split into more, smaller chunks so that it still spreads over the
// whole GPU (a wave's chunk walk is a chain of dependent reads: at 64 topics
// per wave a 4096-topic batch walked on 64 waves for 123 us, round 6).
// Bounded so that n / ct <= max(n / WALK_CHUNK, WALK_MIN_CHUNKS).
constexpr uint32_t WALK_MIN_CHUNKS = 2048, WALK_MIN_CT = 4;
inline uint32_t walk_chunk_topics(uint32_t n) {
  uint32_t ct = WALK_CHUNK;
  while (ct > WALK_MIN_CT && (uint64_t)n < (uint64_t)ct * WALK_MIN_CHUNKS) ct >>= 1;
  return ct;
}
// chunks of a batch of up to n topics (every batch size <= n): the sizing of chunk arrays
inline uint64_t walk_chunk_cap(uint64_t n) {
  const uint64_t a = n / WALK_CHUNK, b = 2 * (uint64_t)WALK_MIN_CHUNKS;
  return (a > b ? a : b) + 2;
}
int walk_grid_blocks(uint32_t n_topics);
size_t scan_tiles(uint32_t n);
// items of HBM stack per heavy wave for topics of up to max_levels levels
uint32_t heavy_stack_items(uint64_t max_levels);
int deep_grid_blocks(uint32_t n_topics);
uint32_t walk_stage();       // the most emits a flush record holds (the larger pass's stage)
uint32_t walk_stage_min();   // the smaller pass's stage: records of either pass hold more than this - 256
// Record slab u32 for a batch of up to `ids` matched ids: every record carries
// REC_IDS + EGM_REC_ALIGN - 1 u32 beyond its entries and holds at least flush_lim - 256 + 1 of
// them (a flush is due once the next step could overfill the stage; the last
// record of a chunk can be shorter: one per chunk), plus every wave's segment
// tail.
inline uint64_t rec_capacity(uint64_t ids, uint32_t n, uint32_t flush_lim, uint32_t grain) {
  const uint32_t fl = flush_lim < walk_stage_min() ? flush_lim : walk_stage_min();   // the shorter pass's records
  const uint64_t per = fl > 256 ? fl - 256 : 1;
  const uint64_t chunks = walk_chunk_cap(n);
  // waves of any batch of up to n topics (their chunk counts are bounded by walk_chunk_cap)
  const uint64_t wc = walk_chunk_cap(n);
  const uint64_t waves = (wc < 256u * 32u ? wc : 256u * 32u) + (uint64_t)deep_grid_blocks(n);
  constexpr uint64_t over = REC_IDS + EGM_REC_ALIGN - 1;
  return ids + ids * (over + per - 1) / per + chunks * (over + REC_HDR) + waves * (grain + EGM_REC_ALIGN + REC_HDR);
}

// Timing hooks: when ev != nullptr, ev[0]/ev[1] bracket the walk kernel.
hipError_t launch_match(const DevTable& tab, const uint8_t* blob, const uint32_t* off, uint32_t n,
                        int mode, const MatchWork& w, const MatchOut& out, hipStream_t s,
                        hipEvent_t* ev_walk, bool* walk_sorted = nullptr);   // walk_sorted: w.order holds the batch's order

// Fan-out (emqx_broker:dispatch/2, emqx_broker.erl:283-324): expand each
// topic's filter ids through the filter -> subscriber CSR.
struct SubTable {
  const uint64_t* row;            // [n_fid_slots + 1] indexed by filter id
  const uint32_t* subs;           // subscriber ids; bit 31 set = shared group id
  uint32_t n_fid_slots;
  const uint4* rp;                // [n_fid_slots] subscriber records (launch_sub_pairs, egm_kernels.hip)
};
bool fan_uses_ds0(bool walk_order_known);   // launch_fanout needs its ds0 buffer ((nids + 1) x 16 B)
hipError_t launch_sub_pairs(const uint64_t* row, const uint32_t* subs, uint32_t n_slots, uint4* rp, hipStream_t s);
// walk_order (optional): the batch's walk order (sort values, topic in the low
// 32 bits, MatchWork::order) — the count then reads the subscriber records of
// a walk chunk's topics together (their matched filters repeat: L2 hits).
// Scratch: wsum u32[nids/64 + 1] (window totals), dsrc 16 B [nids] (each entry's subscriber record:
// packed row
// start | count), wbase u64[nids/64 + 2] (scanned window totals), dpos
// u64[nids + 1] (each entry's first delivery: the compact form's output).
hipError_t launch_fanout(const SubTable& st, const uint64_t* match_row, const uint32_t* match_ids,
                         uint32_t n, uint64_t nids, uint64_t* deliv_row, uint32_t* deliv_fid,
                         uint32_t* deliv_sub, uint64_t deliv_cap, uint32_t* wsum, uint4* dsrc,
                         uint64_t* dpos, uint64_t* wbase, uint64_t* tile_sums, unsigned int* overflow, hipStream_t s,
                         hipEvent_t* ev, const uint64_t* walk_order = nullptr);

// Filter-shard merge: G shard CSRs of one topic batch ->
// one CSR, per topic shard 0's ids first.  cnt is [G][n]; src[g].ids holds
// shard g's ids back to back (device array of G pointers); srow is scratch
// [G][n+1], tot scratch [n]; row [n+1] and out receive the merged CSR.
constexpr uint32_t MAX_SHARDS = 16;   // GPUs of one node (kernel argument, no upload)
struct ShardIds {
  const uint32_t* ids[MAX_SHARDS];
};
hipError_t launch_shard_merge(const uint32_t* cnt, uint32_t G, uint32_t n, const ShardIds& src, uint64_t* srow,
                              uint64_t* tile_sums, uint32_t* tot, uint64_t* row, uint32_t* out, uint64_t cap,
                              hipStream_t s);

// Host-visible result copy: row_ptr, the row_ptr[n] ids (<= ids_cap) and the
// flags of a device CSR into pinned host memory (16-B aligned sections).
hipError_t launch_copy_out(const uint64_t* row, uint32_t n, const uint32_t* ids, uint64_t ids_cap,
                           const uint8_t* flags, uint8_t* h_row, uint8_t* h_ids, uint8_t* h_fl, hipStream_t s,
                           const MatchStats* st = nullptr, MatchStats* h_st = nullptr);

// Prefix partition exchange (egm_common.h prefix_vpart): a rank's
// topic batch -> n_ranks slots of slot_bytes each, one per destination rank,
// laid out for an equal-split all_to_all:
//   [0, 16)          header {count, bytes, overflow, 0}
//   [16, 16 + 4Ct)   source topic index of each slot topic
//   [PO, PO + 4(Ct+1)) offsets into the slot's bytes (entries past count = bytes)
//   [PB, PB + Cb)    topic bytes
// Overflow (a destination got more than Ct topics or Cb bytes) is flagged in
// the header; the slot then holds a consistent prefix of its topics (count,
// bytes and offsets describe exactly the topics placed) and the step must be
// redone with larger capacities.  A batch holds fewer than 2^30 topics
// (PFX_TOPICS_MAX: the packed route counter) and a slot fewer than 2^32 bytes.
constexpr uint32_t PFX_TOPICS_MAX = 1u << 30;
struct PrefixSlots {
  uint32_t n_ranks, cap_topics;
  uint64_t cap_bytes;
  __host__ __device__ uint64_t off_offsets() const { return 16 + 4ull * cap_topics; }
  __host__ __device__ uint64_t off_bytes() const { return (off_offsets() + 4ull * (cap_topics + 1) + 15) & ~15ull; }
  __host__ __device__ uint64_t slot_bytes() const { return (off_bytes() + cap_bytes + 15) & ~15ull; }
};
hipError_t launch_prefix_route(const uint8_t* blob, const uint32_t* off, uint32_t n, const uint8_t* vpart_rank,
                               uint32_t n_vparts, const PrefixSlots& ps, uint8_t* send, unsigned long long* ctr,
                               uint64_t* dst, hipStream_t s);

// Scatter n records of rec_bytes (4, 16 or 32) from src[] to dst[idx[i]]:
// the incremental epoch commit of egm_capi.cpp.
hipError_t launch_patch(void* dst, uint32_t rec_bytes, const uint32_t* idx, const void* src, uint64_t n,
                        hipStream_t s);

// ---- retained reverse match (emqx_retainer_mnesia:match_messages/1) ----
constexpr uint32_t RN_TERM = 0x80000000u;   // node's own topic is stored (in n_children)
constexpr uint32_t RS_SINGLE = 0x80000000u; // range = one already-checked rank (in hi)

struct RetainView {            // a committed retained store in HBM
  const uint4* nodes;          // {first_child, n_children | RN_TERM, lo, hi}: ranks under the node
  const uint4* edges;          // 16 B {parent, word, child, 0}, 4 per 64 B bucket
  uint32_t edge_mask;          // buckets - 1
  const uint32_t* msg;         // rank -> message id
  const uint64_t* expiry;      // rank -> expiry time in ms (0 = never)
  uint32_t n_topics;
};

struct RetainWork {            // per query batch
  const uint32_t* off;         // filter offsets (wid layout of k_tokenise)
  const uint32_t* wid;
  const uint32_t* lv;
  const uint8_t* tfl;
  uint32_t* pc;                // per frontier pair: pairs it creates
  uint32_t* paux;              // per frontier pair: first created node
  uint64_t* poff;              // scan of pc
  uint64_t* tiles;
  uint32_t *rf, *rlo, *rhi;    // emitted rank ranges (filter, lo, hi | RS_SINGLE)
  uint32_t* n_ranges;
  uint32_t range_cap;
  uint32_t* alive;             // per rank: alive at `now` (strict rule)
  uint64_t* apre;              // scan of alive
  uint32_t* fcnt;              // per filter: ids
  uint32_t* roff;              // per range: offset inside the filter's row
  uint64_t now;
  int ge_plain;                // dispatch: plain topics use read_message's Et >= Now
};

hipError_t launch_tokenise(const DevTable& tab, const uint8_t* blob, const uint32_t* off, uint32_t n, uint32_t* wid,
                           uint32_t* lv, uint8_t* tfl, hipStream_t s);
hipError_t launch_rs_alive(const RetainView& v, const RetainWork& w, hipStream_t s);
hipError_t launch_rs_init(uint32_t n, uint32_t* pf, uint32_t* pn, hipStream_t s);
hipError_t launch_rs_level(const RetainView& v, const RetainWork& w, uint32_t level, uint32_t np,
                           const uint32_t* pf, const uint32_t* pn, hipStream_t s);
hipError_t launch_rs_fill(const RetainWork& w, uint32_t np, uint64_t nnext, const uint32_t* pf, uint32_t* pf2,
                          uint32_t* pn2, hipStream_t s);
hipError_t launch_rs_rows(const RetainWork& w, uint32_t nr, uint32_t n, uint64_t* row, hipStream_t s);
hipError_t launch_rs_expand(const RetainView& v, const RetainWork& w, uint32_t nr, const uint64_t* row,
                            uint32_t* ids, hipStream_t s);

}  // namespace egm
