/*
 * emqx_gpu_match.h — C-ABI of libemqx_gpu_match.so, the MI355X (gfx950)
 * drop-in for EMQX's publish-time route lookup.
 *
 * Each entry point replaces a reference interface (EMQ X 5.0-alpha.3, paths
 * relative to the reference root):
 *
 *   egm_table_build / egm_table_apply_delta / egm_table_commit
 *       <- emqx_trie:insert/1, delete/1   apps/emqx/src/emqx_trie.erl:82-96
 *          (driven by emqx_router:do_add_route/2, do_delete_route/2,
 *           apps/emqx/src/emqx_router.erl:114-125,164-170,230-248)
 *   egm_table_empty       <- emqx_trie:empty/0        emqx_trie.erl:117-118
 *   egm_match_batch (EGM_MODE_TRIE)
 *                         <- emqx_trie:match/1        emqx_trie.erl:99-114
 *   egm_match_batch (EGM_MODE_ROUTES)
 *                         <- emqx_router:match_routes/1's filter set
 *                                                      emqx_router.erl:128-145
 *   egm_fanout_batch      <- emqx_broker:dispatch/2 subscriber expansion
 *                                                      emqx_broker.erl:283-324
 *   egm_filter_bytes      <- the filter binaries match/1 returns (id -> bytes)
 *
 * Conventions: plain pointers and sizes only; every function returns 0 or a
 * negative EGM_E* code and never throws; host buffers are borrowed for the
 * duration of the call; results are library-allocated and released with
 * egm_result_free().  One context = one HIP device; calls on a context are
 * serialised internally (a dirty-scheduler NIF may call from any thread).
 * The device entry points may be given any HIP stream — NULL is the HIP
 * default (null) stream, ordered with the caller's own work there (e.g. a
 * PyTorch default-stream tensor fill), never a stream of the library's own:
 * launches that share the context's workspaces are ordered across streams by
 * the library (a launch on a new stream waits for the previous one), and a
 * table commit waits for every launch still reading the epoch it overwrites.
 * Table changes are all-or-nothing: a delta or build with an invalid id
 * leaves the staged table unchanged.
 */
#ifndef EMQX_GPU_MATCH_H
#define EMQX_GPU_MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EGM_OK 0
#define EGM_E_INVAL (-1)     /* bad argument (mirrors the reference's function_clause) */
#define EGM_E_NOMEM (-2)     /* host or device allocation failed */
#define EGM_E_DEVICE (-3)    /* HIP runtime / kernel failure */
#define EGM_E_OVERFLOW (-4)  /* a topic's frontier exceeded the heavy-path stack */
#define EGM_E_STATE (-5)     /* call not valid in the current state */
#define EGM_E_NOTFOUND (-6)  /* unknown filter id */

/* Match semantics. */
#define EGM_MODE_TRIE 0   /* emqx_trie:match/1 over the table's filters            */
#define EGM_MODE_ROUTES 1 /* filters whose routes emqx_router:match_routes/1 returns */

/* egm_result.flags[i] bits */
#define EGM_TF_WILDCARD 1u /* topic has a '+' or '#' word (TRIE mode: no matches) */
#define EGM_TF_DOLLAR 2u   /* first word starts with '$'                          */
#define EGM_TF_HEAVY 4u    /* matched by the overflow (heavy) kernel              */
#define EGM_TF_ERROR 8u    /* not matched: frontier exceeded the heavy stack      */

typedef struct egm_ctx egm_ctx;

typedef struct egm_config {
  int32_t device;        /* HIP device ordinal                                        */
  int32_t compact_mode;  /* broker.perf.trie_compaction (emqx_trie.erl:272-276);
                            match sets do not depend on it — kept for API parity      */
  uint32_t max_batch;    /* expected topics per call (pre-sizes workspaces; 0 = lazy) */
  uint32_t linger_us;    /* host batcher linger hint (emqx_batch.erl:50-81)           */
} egm_config;

typedef struct egm_delta {
  const uint8_t* blob;      /* filters back to back                                 */
  const uint32_t* offsets;  /* [n+1] byte offsets into blob                         */
  uint32_t n;
  const uint32_t* ids;      /* optional [n] filter ids for inserts (NULL = assign)  */
} egm_delta;

typedef struct egm_result {
  uint32_t n_topics;
  uint64_t n_ids;
  uint32_t* counts;    /* [n_topics]    matches per topic                           */
  uint64_t* row_ptr;   /* [n_topics+1]  CSR row starts                              */
  uint32_t* ids;       /* [n_ids]       filter ids (a set per row, no duplicates)   */
  uint8_t* flags;      /* [n_topics]    EGM_TF_* bits                               */
  uint64_t epoch;      /* table epoch the batch was matched against                 */
  uint64_t visited;    /* NFA states expanded (instrumentation)                     */
  uint32_t n_heavy;    /* topics routed through the heavy kernel                    */
  uint32_t n_error;    /* topics flagged EGM_TF_ERROR                               */
  /* The packed form (a pipeline batch submitted with EGM_RESULT_PACKED, when
     every filter id of its epoch is below 2^24; round 6): id_bytes == 3,
     row_ptr and ids are NULL, row32 holds the row starts as u32 and ids24 the
     ids as 3-byte little-endian values — 3 bytes per id and 4 per row start
     cross PCIe instead of 4 and 8.  Otherwise id_bytes == 4 and row32/ids24
     are NULL.  Read either form with egm_result_row()/egm_result_id(). */
  uint32_t id_bytes;
  const uint32_t* row32;  /* [n_topics+1] (packed form)                             */
  const uint8_t* ids24;   /* [3 * n_ids]  (packed form)                             */
} egm_result;

/* mode flag of egm_match_submit / egm_match_batch: the packed result form */
#define EGM_RESULT_PACKED 0x100

static inline uint64_t egm_result_row(const egm_result* r, uint32_t i) {
  return r->row32 ? (uint64_t)r->row32[i] : r->row_ptr[i];
}
static inline uint32_t egm_result_id(const egm_result* r, uint64_t k) {
  if (r->ids24) {
    const uint8_t* p = r->ids24 + 3 * k;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
  }
  return r->ids[k];
}

typedef struct egm_delivery {
  uint32_t n_topics;
  uint64_t n_deliveries;
  uint64_t* row_ptr;   /* [n_topics+1]                                              */
  uint32_t* fid;       /* [n_deliveries] matched filter id                          */
  uint32_t* sub;       /* [n_deliveries] subscriber id, or group id | 0x80000000    */
} egm_delivery;

/* ---- context ---- */
int egm_open(const egm_config* cfg, egm_ctx** out);
void egm_close(egm_ctx* ctx);
const char* egm_last_error(egm_ctx* ctx);
const char* egm_version(void);

/* ---- filter table (emqx_trie content) ---- */
/* Replace the whole table with n filters; filter_ids optional (NULL = 0..n-1
   in order).  Duplicate filters keep their first id (insert/1 is idempotent).
   Publishes a new epoch. */
int egm_table_build(egm_ctx* ctx, const uint8_t* filters_blob, const uint32_t* offsets, uint32_t n,
                    const uint32_t* filter_ids);
/* Stage inserts then deletes (either may be NULL); visible after commit. */
int egm_table_apply_delta(egm_ctx* ctx, const egm_delta* ins, const egm_delta* del);
/* Publish the staged table as a new epoch (readers in flight keep the old).
   Incremental: the device keeps two copies of the image; a commit writes the
   one no reader is using and patches into it only the records the staged
   deltas changed (a rebuild — relayout, table growth — copies whole).
   The whole-table analogue of the mnesia transaction around
   emqx_trie:insert/delete, apps/emqx/src/emqx_router.erl:252-303. */
int egm_table_commit(egm_ctx* ctx, uint64_t* epoch);
/* What the last commit moved: host->device bytes, device->device bytes,
   records patched, host wall time (ms). */
int egm_last_commit_stats(egm_ctx* ctx, uint64_t* h2d_bytes, uint64_t* d2d_bytes, uint64_t* patched,
                          double* ms);
/* The current (last published) epoch.  A batch submitted after this call is
   matched against this epoch or a later one, so a caller that keeps filters
   published after it in an overlay (erl/emqx_gpu_routes.erl) never misses one.
   No reference counterpart: emqx_trie reads the committed mnesia table. */
int egm_table_epoch(egm_ctx* ctx, uint64_t* epoch);
/* 1 if the committed table holds no filter, 0 otherwise. */
int egm_table_empty(egm_ctx* ctx);
/* Counts of the committed table: filters, trie nodes, literal edges, words. */
int egm_table_stats(egm_ctx* ctx, uint64_t* n_filters, uint64_t* n_nodes, uint64_t* n_edges,
                    uint64_t* n_words, uint64_t* device_bytes);
/* Filter id of given bytes in the staged table, or EGM_E_NOTFOUND. */
int egm_filter_id(egm_ctx* ctx, const uint8_t* filter, uint32_t len, uint32_t* id);
/* Bytes of a filter id (pointer valid until the next table mutation). */
int egm_filter_bytes(egm_ctx* ctx, uint32_t id, const uint8_t** bytes, uint32_t* len);

/* ---- matching ---- */
/* Host buffers in, CSR result out (allocated; free with egm_result_free). */
int egm_match_batch(egm_ctx* ctx, const uint8_t* topics_blob, const uint32_t* topic_offsets,
                    uint32_t n_topics, int mode, egm_result** out);

/* Pipelined host batches (the drop-in's NIF path; SURVEY §8b ownership):
   egm_match_submit copies the caller's borrowed batch into pinned staging at
   once (the caller may reuse its buffers when it returns), queues the
   host->device copy on a copy stream and the match on the context stream, and
   hands back a ticket; egm_match_wait blocks for that ticket and returns the
   CSR result in pinned memory (no extra host copy), valid until
   egm_result_free.  With two tickets in flight, batch k's device->host copy
   overlaps batch k+1's match.  At most 8 tickets or unreleased results per
   context (EGM_E_STATE beyond); free pipeline results before egm_close.
   A ticket carries a generation: a stale, repeated or cancelled ticket is
   refused with EGM_E_STATE (never answered with another batch's result).
   egm_match_cancel gives a ticket up without waiting: its slot is reclaimed
   once its batch has finished (for a waiter that will never call wait).  It
   never blocks: while another call holds the context (a bulk build or a
   commit can for seconds) the cancel is queued and applied by the next
   pipeline call, so it may run on a normal Erlang scheduler or in a resource
   destructor; a queued cancel of a stale ticket is dropped.  Return value:
   EGM_OK when the cancel was applied OR queued (a queued cancel is not
   validated: EGM_OK then says nothing about the ticket), EGM_E_STATE only
   when the context was free and the ticket is unknown, stale or already
   waited.  Callers must not branch on the difference (the NIF's cancel/2
   returns ok in both cases).  A queued cancel keeps its slot busy until the
   next submit, wait or cancel drains the queue.
   egm_match_batch is submit + wait on a slot of its own: concurrent callers
   never see "pipeline full" (extra slots up to 16, then they queue for one).
   A walk guard trip (a kernel invariant failed, egm_last_guard) makes wait
   return EGM_E_DEVICE; only a capacity overflow is retried.
   mode may carry EGM_RESULT_PACKED: a batch of more than 16 384 topics then
   returns the packed form (egm_result.id_bytes == 3) when its epoch's filter
   ids all fit 24 bits — the host path is bound by the PCIe link, and the
   packed form moves ~28 % fewer bytes.  Smaller batches, and tables with
   larger filter ids, return the plain form; read both with egm_result_row()
   and egm_result_id(). */
int egm_match_submit(egm_ctx* ctx, const uint8_t* topics_blob, const uint32_t* topic_offsets, uint32_t n_topics,
                     int mode, uint64_t* ticket);
int egm_match_wait(egm_ctx* ctx, uint64_t ticket, egm_result** out);
int egm_match_cancel(egm_ctx* ctx, uint64_t ticket);

/* Device-resident variant: d_blob (4-byte aligned, blob_bytes >= d_offsets[n])
   and d_offsets are device pointers (d_offsets[0] == 0); results stay in device buffers owned by the caller
   (d_row_ptr[n+1], d_ids[ids_cap], d_flags[n] may be NULL).  Asynchronous on
   `hip_stream` (NULL = the HIP default stream).  After the stream completes,
   d_row_ptr[n] holds the number of ids; egm_last_stats() reports overflow. */
int egm_match_device(egm_ctx* ctx, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_offsets,
                     uint32_t n_topics, int mode, void* hip_stream, uint64_t* d_row_ptr, uint32_t* d_ids,
                     uint64_t ids_cap, uint8_t* d_flags);
/* egm_match_device with the rows in the walk's order (round 5; SURVEY §8b,
   the result form the NIF consumes): row k holds the matches of input topic
   d_topic[k] (every topic exactly once), d_row_ptr[n+1] is that CSR.  The
   walk visits topics sorted by their first levels; in this
   form each chunk of 64 consecutive rows is one contiguous run of d_ids, so
   no row is scattered and there is no second pass over the ids to put them
   in input order.  The sets are egm_match_device's: topic d_topic[k]'s row
   there equals row k here, as a set.  Asynchronous on hip_stream (NULL = the
   HIP default stream); egm_last_stats() reports overflow (rerun with a larger
   ids_cap). */
int egm_match_device_ordered(egm_ctx* ctx, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_offsets,
                             uint32_t n_topics, int mode, void* hip_stream, uint64_t* d_row_ptr, uint32_t* d_topic,
                             uint32_t* d_ids, uint64_t ids_cap);
/* egm_match_device over a batch whose topic count is on the device: d_n is a
   device slot header {count, bytes, overflow, 0} (u32 x 4, egm_prefix_route's
   layout).  The first count (<= n_max) topics are matched, the rest (padding;
   their offsets must still be valid, e.g. empty topics at the end) get empty
   rows without a walk; a header with overflow != 0 is matched as an empty
   batch (every row empty: the step must be redone, its partial slot is never
   walked).  For batches whose size only the device knows — the received slots
   of the prefix partition exchange (egm_prefix_route) — so the host never
   waits for a count.  d_row_ptr[n_max] holds the number of ids. */
int egm_match_device_counted(egm_ctx* ctx, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_offsets,
                             uint32_t n_max, const uint32_t* d_n, int mode, void* hip_stream, uint64_t* d_row_ptr,
                             uint32_t* d_ids, uint64_t ids_cap);
/* egm_match_device_counted with the rows in the walk's order (as
   egm_match_device_ordered): row k holds the matches of slot topic d_topic[k];
   the first count rows are the counted topics (padding sorts last), the rest
   are empty. */
int egm_match_device_counted_ordered(egm_ctx* ctx, const uint8_t* d_blob, uint64_t blob_bytes,
                                     const uint32_t* d_offsets, uint32_t n_max, const uint32_t* d_n, int mode,
                                     void* hip_stream, uint64_t* d_row_ptr, uint32_t* d_topic, uint32_t* d_ids,
                                     uint64_t ids_cap);
/* Synchronises the last device batch and reports its counters.  overflow != 0
   means ids_cap was too small (rerun with a larger buffer) — capacity only.
   Returns EGM_E_DEVICE (counters still filled) when a walk guard tripped:
   a kernel invariant failed, the batch's rows were not assembled, and a
   larger buffer would not help (egm_last_guard has the bits). */
int egm_last_stats(egm_ctx* ctx, uint64_t* n_ids, uint64_t* visited, uint32_t* n_deferred_chunks,
                   uint32_t* overflow, uint32_t* n_error);
/* Guard bits of the last batch (0 = none): 4 = a work stack would have
   overrun (impossible by the pop bound: a bug), 8 = a walk loop ran past its
   iteration guard (reported instead of hanging the GPU). */
int egm_last_guard(egm_ctx* ctx, uint32_t* guard);
/* Instrumentation: walk iterations and items popped of the last batch (lane
   occupancy = popped / (iters*64)), the iterations whose pop the stack-room
   bound cut short (the depth-first regime of deep, wide frontiers), and the
   pops that read an edge bucket / a '+' child's record (the walk's random
   line reads).  Any pointer may be NULL. */
int egm_last_walk_counters(egm_ctx* ctx, uint64_t* iters, uint64_t* popped, uint64_t* bounded, uint64_t* lit_probes,
                           uint64_t* plus_reads);
/* Instrumentation: the last batch's literal probes that needed a second
   (dependent) bucket read, and the walk iterations in which any lane did. */
int egm_last_walk_probes(egm_ctx* ctx, uint64_t* slow_lanes, uint64_t* slow_iters);
/* Enable per-kernel timing with HIP events on the launch stream (0/1) and read
   the accumulated walk-kernel time (ms) and launch count. */
int egm_set_timing(egm_ctx* ctx, int enable);
/* Test hooks: bit 0 routes every chunk through the heavy kernel; bit 1 makes
   the next table commit fail after it has taken the staged changes (they must
   survive into the following commit). */
#define EGM_DEBUG_FORCE_HEAVY 1u
#define EGM_DEBUG_FAIL_COMMIT 2u
#define EGM_DEBUG_INPUT_ORDER 4u   /* walk the batch in input order (no locality sort; A/B and tests) */
#define EGM_DEBUG_FORCE_GUARD 8u   /* loop guards of 2 iterations: trips the walk guard (error-path test) */
int egm_set_debug(egm_ctx* ctx, uint32_t flags);
/* Test hook: the walk-order radix sort alone (egm_kernels.hip walk_sort, the
   hand-written LSD sort every sorted batch runs): d_out[i] = d_vals of the
   i-th pair in a STABLE sort by the key's kbits (1..32) high bits; n < 2^29.
   Inputs are not modified.  EGM_E_DEVICE if a look-back guard tripped. */
int egm_debug_walk_sort(egm_ctx* ctx, const uint32_t* d_keys, const uint64_t* d_vals, uint32_t n, uint32_t kbits,
                        uint64_t* d_out);
int egm_get_timing(egm_ctx* ctx, double* walk_ms, uint64_t* walk_launches, double* fanout_ms,
                   uint64_t* fanout_launches);

/* ---- subscriber fan-out (emqx_broker:dispatch/2) ---- */
/* filter id -> subscriber ids CSR (sub | 0x80000000 marks a shared group id). */
int egm_subs_build(egm_ctx* ctx, const uint64_t* row_ptr, uint32_t n_fid_slots, const uint32_t* subs);
/* Incremental subscriber changes, the table kept by emqx_broker's
   subscribe/3, unsubscribe/1 and subscriber_down/1 (apps/emqx/src/
   emqx_broker.erl:144-197, 331-345; emqx_broker_helper.erl:133-163 purges a
   dead subscriber): add / remove (filter id, subscriber) pairs on the host —
   a pair already present is not added twice (an ets bag keeps one copy of an
   identical object), removing an absent one does nothing, a list keeps its
   order — then egm_subs_commit publishes them to the fan-out in one epoch.
   The commit appends the changed rows to the device entries and patches
   their records into the record copy no fan-out in flight reads (after its
   last readers finished), then makes it current: fan-outs already launched
   keep the epoch they started with.  A new filter id past the table, a row of
   2^24 subscribers, or appended rows past the reserve make it a full build
   (egm_subs_last_commit reports which), sized from the largest filter id
   that still has a subscriber.  EGM_E_STATE before egm_subs_build.
   Contract of one egm_subs_apply_delta call: `add` and `del` are the NET
   changes since the caller's previous call, so no (fid, sub) pair may appear
   in both (adds are applied before removes; "unsubscribe X then subscribe X
   again" is the add alone, or nothing if X was there) — a pair in both lists
   is refused with EGM_E_INVAL and nothing is applied.  An added fid must be
   below the table's slots + 2^22 (filter ids are dense); a larger one is
   refused with EGM_E_INVAL.  Host allocation failures return EGM_E_NOMEM
   (no entry point throws). */
typedef struct egm_sub_pair {
  uint32_t fid;   /* filter id */
  uint32_t sub;   /* subscriber id, or a $share group id | 0x80000000 */
} egm_sub_pair;
int egm_subs_apply_delta(egm_ctx* ctx, const egm_sub_pair* add, uint64_t n_add, const egm_sub_pair* del,
                         uint64_t n_del);
int egm_subs_commit(egm_ctx* ctx, uint64_t* epoch);
/* What the last egm_subs_commit did: subscriber entries appended, records
   patched, whether it was a full build, entries now on the device. */
int egm_subs_last_commit(egm_ctx* ctx, uint64_t* appended, uint64_t* patched, int* rebuilt, uint64_t* entries);
/* Filter-id slots of the device subscriber records (ids at or past it have no
   subscribers): the build's ids + a quarter + 4096 spare, re-sized by a full
   build from the largest filter id that still has a subscriber. */
int egm_subs_slots(egm_ctx* ctx, uint32_t* n_fid_slots);
int egm_fanout_batch(egm_ctx* ctx, const egm_result* matched, egm_delivery** out);
/* Device variant over a device CSR match result.  match_ids_len = entries
   d_match_ids holds: a match row whose total exceeds it (an overflowed match
   batch) returns EGM_E_OVERFLOW before any kernel reads the ids. */
int egm_fanout_device(egm_ctx* ctx, const uint64_t* d_match_row, const uint32_t* d_match_ids,
                      uint64_t match_ids_len, uint32_t n_topics, void* hip_stream, uint64_t* d_deliv_row, uint32_t* d_fid,
                      uint32_t* d_sub, uint64_t deliv_cap);
/* The compact form of egm_fanout_device: only the subscriber ids are written
   (4 B per delivery instead of 8), and d_entry_pos[match_ids + 1] receives
   each match entry's first delivery — so delivery k of match entry i, i.e.
   of filter d_match_ids[i], is d_sub[d_entry_pos[i] + k]; a topic's
   deliveries are its match row's entries' in order (d_deliv_row as above).
   The same delivery lists as the pair form, half the bytes written (C4 writes
   ~4.6 G deliveries per 10M-topic batch). */
int egm_fanout_device_compact(egm_ctx* ctx, const uint64_t* d_match_row, const uint32_t* d_match_ids,
                              uint64_t match_ids_len, uint32_t n_topics, void* hip_stream, uint64_t* d_deliv_row,
                              uint64_t* d_entry_pos, uint32_t* d_sub, uint64_t deliv_cap);
/* Synchronises the last fan-out and reports its delivery total and whether
   deliv_cap was too small (overflow != 0: d_fid/d_sub were not written;
   rerun with deliv_cap >= n_deliveries). */
int egm_last_fanout(egm_ctx* ctx, uint64_t* n_deliveries, uint32_t* overflow);

/* ---- multi-GPU filter sharding ----
   Merge the match results of one topic batch against n_shards disjoint filter
   shards (each matched on its own GPU, gathered here over RCCL) into one CSR:
   per topic, shard 0's ids, then shard 1's, ...  The union is disjoint (a
   filter lives in exactly one shard), so no dedup.  The reference has no
   counterpart: it replicates the whole table to every node
   (apps/emqx/src/emqx_trie.erl:53, apps/emqx/src/emqx_router.erl:71).
   d_counts: device [n_shards][n] per-topic counts; d_shard_ids: host array of
   n_shards (<= 16) device pointers (shard g's ids back to back, topic order);
   total_ids: the sum of all counts (EGM_E_OVERFLOW if > ids_cap).
   Asynchronous on hip_stream (NULL = the HIP default stream). */
int egm_shard_merge(egm_ctx* ctx, uint32_t n_shards, uint32_t n_topics, const uint32_t* d_counts,
                    const uint32_t* const* d_shard_ids, uint64_t total_ids, void* hip_stream, uint64_t* d_row_ptr,
                    uint32_t* d_ids, uint64_t ids_cap);

/* ---- multi-GPU prefix partition ("partition by root word") ----
   Filters and topics are keyed by their bytes before the second '/' (the
   first two words, or the whole of a one-level name); keys hash into
   n_vparts virtual partitions that map to ranks.  A filter whose first or
   second word is '+' or '#' can match any key and lives on every rank
   (EGM_PREFIX_ALL); every other filter only on its key's rank — every topic
   it can match has its key.  A topic is matched on exactly one rank, against
   all the filters that can match it, so the ranks' rows together are the
   whole table's with no merge, and a topic batch crosses xGMI once (one
   all_to_all), with no broadcast and no gather.  The reference replicates its
   tables instead (apps/emqx/src/emqx_trie.erl:53, emqx_router.erl:71).
   egm_prefix_assign (host): vpart_rank[n_vparts] (greedy by filter counts,
   deterministic) and filter_rank[n] (a rank or EGM_PREFIX_ALL).
   egm_prefix_route (device, async on hip_stream): a batch -> n_ranks slots of
   egm_prefix_slot_bytes() each in d_send, slot r for rank r:
     [0,16) {count, bytes, overflow, 0}; [16, 16+4*cap_topics) source topic
     index of each slot topic; then offsets u32[cap_topics+1] (entries past
     count = bytes); then the topic bytes (cap_bytes), all 16-B aligned.
   A slot past its capacity sets overflow: it then holds the topics placed
   before the capacity ran out, and count, bytes and offsets describe exactly
   those (a consistent, incomplete slot; egm_match_device_counted matches it as
   empty); redo the step with larger capacities (dist.PrefixExchange.run does).
   n_topics and cap_topics < 2^30, cap_bytes < 2^32, n_ranks <= 16, else
   EGM_E_INVAL. */
#define EGM_PREFIX_ALL 0xFFFFFFFFu
int egm_prefix_assign(const uint8_t* blob, const uint32_t* offsets, uint32_t n, uint32_t n_vparts, uint32_t n_ranks,
                      uint8_t* vpart_rank, uint32_t* filter_rank);
uint64_t egm_prefix_slot_bytes(uint32_t n_ranks, uint32_t cap_topics, uint64_t cap_bytes);
int egm_prefix_route(egm_ctx* ctx, const uint8_t* d_blob, const uint32_t* d_offsets, uint32_t n_topics,
                     const uint8_t* d_vpart_rank, uint32_t n_vparts, uint32_t n_ranks, uint32_t cap_topics,
                     uint64_t cap_bytes, void* hip_stream, uint8_t* d_send);

void egm_result_free(void* result);

/* ---- retained messages: reverse match ----
   One subscription filter against every stored retained topic, for a batch of
   filters.  Replaces apps/emqx_retainer/src/emqx_retainer_mnesia.erl:
     egm_rstore_put     <- store_retained/2  :73-101 (one record per topic;
                           topics with a '+'/'#' word are rejected: EGM_E_INVAL)
     egm_rstore_delete  <- delete_message/2  :114-129 (plain topic)
     egm_rstore_clean   <- clean/1           :148-150
     egm_rstore_match   <- match_messages/1  :200-204 with condition/1 :215-220
                           and make_match_spec/1 :222-228: '+' matches any one
                           word, a last '#' any rest (also none), NO '$' rule;
                           alive when expiry == 0 or expiry > now_ms.
                           EGM_RMODE_DISPATCH routes plain topics through
                           read_messages/1 :187-198 instead (alive when expiry
                           >= now_ms), as emqx_retainer:dispatch/4 does
                           (apps/emqx_retainer/src/emqx_retainer.erl:107-117).
   Result rows hold message ids (order within a row unspecified: the reference
   sorts by timestamp, sort_retained/1 :154-159, on the host).  Changes are
   visible to the next match (the device image is rebuilt on demand). */
typedef struct egm_rstore egm_rstore;
enum { EGM_RMODE_MATCH = 0, EGM_RMODE_DISPATCH = 1 };
int egm_rstore_open(int device, egm_rstore** out);
void egm_rstore_close(egm_rstore* rs);
const char* egm_rstore_last_error(egm_rstore* rs);
int egm_rstore_put(egm_rstore* rs, const uint8_t* topic, uint32_t len, uint32_t msg_id, uint64_t expiry_ms);
int egm_rstore_delete(egm_rstore* rs, const uint8_t* topic, uint32_t len);
int egm_rstore_clean(egm_rstore* rs);
int egm_rstore_size(egm_rstore* rs, uint64_t* n);
/* Upload the current records now (otherwise done by the next match). */
int egm_rstore_commit(egm_rstore* rs);
int egm_rstore_match(egm_rstore* rs, const uint8_t* filters_blob, const uint32_t* offsets, uint32_t n,
                     uint64_t now_ms, int mode, egm_result** out);

/* ---- host-only table image (diagnostics; needs no device) ----
   Builds the same HBM image egm_table_commit uploads, so the layout can be
   inspected and tested on a host without a GPU. */
typedef struct egm_image egm_image;
typedef struct egm_image_view {
  const void* nodes;      uint64_t n_nodes;      /* 16 B {plus_child, hash_fid, term_fid, meta} */
  const uint32_t* hash_child;
  const void* edges;      uint64_t n_edge_slots; /* 32 B {parent, word, child, child record}, 4 per bucket */
  uint32_t edge_mask;                            /* buckets - 1 */
  const void* dict;       uint64_t n_dict_slots; /* 32 B {hash64, word, len, inline[16]} */
  uint32_t dict_mask;
  const uint8_t* dict_blob; const uint64_t* dict_off; uint64_t n_words;
  uint64_t n_filters; uint64_t n_live_nodes; uint64_t n_edges;
} egm_image_view;
egm_image* egm_image_new(void);
void egm_image_free(egm_image* im);
/* 0 inserted, 1 already present, <0 error (id NONE = 0xFFFFFFFF assigns) */
int egm_image_insert(egm_image* im, const uint8_t* filter, uint32_t len, uint32_t id);
/* 0 removed, 1 absent */
int egm_image_remove(egm_image* im, const uint8_t* filter, uint32_t len);
void egm_image_relayout(egm_image* im);
/* The whole image from n filters at once (what egm_table_build does from
   EGM_BULK_MIN = 65 536 filters on): the image of inserting them in order
   (first occurrence of a repeat wins) + relayout, built level by level on
   `threads` host threads (0 = the usable CPUs).  ids NULL = 0..n-1; no id may
   be NONE. */
int egm_image_build(egm_image* im, const uint8_t* blob, const uint32_t* offsets, uint32_t n, const uint32_t* ids,
                    uint32_t threads);
int egm_image_get_view(egm_image* im, egm_image_view* out);
/* Records of the image changed since the previous call (sorted, unique
   indices; *_full = the array was rebuilt): what egm_table_commit patches.
   Pointers stay valid until the next call. */
typedef struct egm_dirty_view {
  const uint32_t* nodes;  uint64_t n_nodes;   /* indices into nodes[] and hash_child[] */
  const uint32_t* edges;  uint64_t n_edges;   /* edge slot indices */
  const uint32_t* dict;   uint64_t n_dict;    /* dictionary slot indices */
  uint32_t nodes_full, edges_full, dict_full, words_full;
} egm_dirty_view;
int egm_image_take_dirty(egm_image* im, egm_dirty_view* out);
/* Filter -> shard for multi-GPU filter sharding: out[i] =
   word_hash(filter i) mod n_shards.  Host-only. */
int egm_shard_assign(const uint8_t* blob, const uint32_t* offsets, uint32_t n, uint32_t n_shards,
                     uint32_t* out);
/* the 64-bit word hash and the edge bucket function the kernels use */
uint64_t egm_word_hash(const uint8_t* p, uint32_t len);
uint32_t egm_edge_bucket(uint32_t parent, uint32_t word, uint32_t mask);

#ifdef __cplusplus
}
#endif
#endif /* EMQX_GPU_MATCH_H */
