// egm_capi.cpp — the C-ABI of libemqx_gpu_match.so (include/emqx_gpu_match.h).
//
// Owns: one HIP stream per context, the staged host table (egm_table.cpp),
// the committed device epochs (double-buffered through shared_ptr so a batch
// in flight keeps the epoch it started with — the race-free analogue of the
// reference's mnesia transactions around emqx_trie:insert/delete,
// apps/emqx/src/emqx_router.erl:252-303), and the per-batch workspaces.
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/emqx_gpu_match.h"
#include "egm_alloc.h"
#include "egm_dma.h"
#include "egm_pack.h"
#include "egm_kernels.h"
#include "egm_table.h"

using namespace egm;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    size_t b = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&p, b);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = b;
    return hipSuccess;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

// Pinned host memory (page-locked: DMA at full PCIe rate, asynchronous copies).
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  PinBuf() = default;
  PinBuf(const PinBuf&) = delete;
  PinBuf& operator=(const PinBuf&) = delete;
  ~PinBuf() { release(); }
  void release() {
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    const size_t b = bytes + bytes / 4 + 4096;   // grow with headroom: pinning is slow
    hipError_t e = hipHostMalloc(&p, b, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = b;
    return hipSuccess;
  }
};

// One batch of the host pipeline (egm_match_submit / egm_match_wait): its
// pinned input copy, device input and output, and the pinned result the
// caller reads until egm_result_free.
struct PipeSlot {
  bool busy = false;       // submitted, not yet waited for
  bool waiting = false;    // a thread is in egm_match_wait for it
  bool held = false;       // its result is with the caller
  bool sync = false;       // taken by egm_match_batch (not a ticket of egm_match_submit)
  bool abandoned = false;  // egm_match_cancel: reclaimed once its batch has finished
  uint32_t gen = 0;        // bumped at every submit: part of the ticket, so a stale ticket is refused
  uint32_t n = 0;
  int mode = 0;
  bool want_packed = false;   // submitted with EGM_RESULT_PACKED
  bool packed = false;        // this launch's result is packed (egm_pack.h): row32 + 3-byte ids
  uint64_t bytes = 0, maxlen = 0, cap = 0;
  uint64_t o_off = 0;      // the offsets' place after the blob in h_in and d_in (one H2D copy)
  PinBuf h_in, h_out, h_stats;
  DevBuf d_in, d_row, d_ids, d_flags, d_row32, d_pk;
  // ev_in: staged input copied in; ev_match: matched (stream s); ev_done: the
  // CSR in h_out (the copier's D2H copies, or the copy-out kernel)
  hipEvent_t ev_in = nullptr, ev_match = nullptr, ev_done = nullptr;
  uint64_t epoch = 0;
  // launches of this slot / of them, how many the copier has enqueued the
  // D2H of (ev_done is recorded for launch k once copied_gen == k; guarded by
  // egm_ctx::cq_mu)
  uint64_t launch_gen = 0, copied_gen = 0;
  bool copy_failed = false;   // the copier's DMA reported an error (guarded by cq_mu)
  ~PipeSlot() {
    if (ev_in) hipEventDestroy(ev_in);
    if (ev_match) hipEventDestroy(ev_match);
    if (ev_done) hipEventDestroy(ev_done);
  }
};

// Layout of a pipeline result in the slot's pinned buffer (h_out): header,
// egm_result, then row_ptr, ids (room for `cap`), flags, counts — each 16-B
// aligned, as the copy-out kernel writes them.
struct OutLayout {
  size_t o_res, o_row, o_ids, o_fl, o_cnt, total;
};
inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
inline OutLayout out_layout(uint64_t n, uint64_t cap) {
  OutLayout o;
  o.o_res = sizeof(ResultHdr);
  o.o_row = al16(o.o_res + sizeof(egm_result));
  o.o_ids = al16(o.o_row + (n + 1) * 8);
  o.o_fl = al16(o.o_ids + cap * 4);
  o.o_cnt = al16(o.o_fl + n);
  o.total = o.o_cnt + n * 4 + 16;
  return o;
}
constexpr uint32_t PREFIX_RANKS_MAX = 16;   // ranks of one prefix partition (kernel limit)
constexpr size_t PIPE_MAX_SLOTS = 8;     // tickets of egm_match_submit busy or held at once
constexpr size_t PIPE_HARD_SLOTS = 16;   // all slots, egm_match_batch's included (then it waits); each
                                         // keeps buffers for the largest batch it saw (~ dirty schedulers)
constexpr int PIPE_BATCH_WAIT_MS = 30000;   // egm_match_batch's longest wait for a slot

// ticket = generation << 16 | (slot index + 1)
inline uint64_t make_ticket(size_t k, uint32_t gen) { return ((uint64_t)gen << 16) | (uint64_t)(k + 1); }
inline size_t ticket_slot(uint64_t t) { return (size_t)(t & 0xFFFFu) - 1; }
inline uint32_t ticket_gen(uint64_t t) { return (uint32_t)(t >> 16); }

// One match workspace: the per-batch scratch of launch_match.
struct MatchWs {
  DevBuf wid, lv, tfl, cnt, ids_tmp, pieces, deferred, heavy_stack, tile_sums, stats;
  DevBuf skey, skey_out, sval, order, wfix, sort_tmp;   // walk-order sort
  DevBuf rec, chunks, dir;                               // flush records, per-chunk chains and directories
  uint64_t pieces_cap = 0, ids_tmp_cap = 0, rec_cap = 0;
  uint32_t rec_grain = REC_GRAIN, flush_lim = 0;
  uint32_t heavy_cap = 0;        // stack items per heavy wave
  hipEvent_t ev = nullptr;       // recorded after its last batch
  hipStream_t stream = nullptr;  // stream of its last batch
  uint64_t used = 0;             // LRU clock
  ~MatchWs() {
    if (ev) hipEventDestroy(ev);
  }
};
constexpr uint32_t MATCH_WORKSPACES = 2;

// One device copy of the table image.  Two slots alternate: a commit writes
// the slot that is NOT current, so batches still reading the current epoch are
// never disturbed, and it brings that slot up to date with the records the
// host changed since the slot was last written (its pending log + this
// commit's) instead of re-uploading the whole image.
struct Slot {
  DevBuf nodes, hash_child, edges, dict, dict_blob, dict_off;
  uint64_t n_nodes = 0, n_hc = 0, n_edges = 0, n_dict = 0, n_blob = 0, n_off = 0;   // elements held
  bool valid = false;
  DirtyLog pending;                                          // host changes not yet applied here
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;      // last reading launch per stream
  uint64_t bytes() const {
    return nodes.cap + hash_child.cap + edges.cap + dict.cap + dict_blob.cap + dict_off.cap;
  }
};

// The subscriber table of the fan-out (emqx_subscriber, emqx_broker.erl:144-197,
// 331-345), kept incrementally: the authoritative lists on the host (the CSR
// of the last full build + the lists changed since), and on the device the
// entries (sub_ids: the build's rows, then every changed row appended) and
// two copies of the per-filter records the fan-out reads (k_sub_pairs'
// layout).  A commit appends the changed rows past the entries any reader
// can reach, patches them into the record copy no reader uses (after its
// last readers finished) and makes it current — the table's two-slot epoch
// scheme (egm_table_commit) for the subscriber side.
struct SubsState {
  bool built = false;
  std::vector<uint64_t> row;                                  // the last full build's CSR
  std::vector<uint32_t> subs;
  std::unordered_map<uint32_t, std::vector<uint32_t>> lists;  // filters changed since that build
  std::unordered_map<uint32_t, uint4> recs;                   // their current records
  std::vector<uint32_t> pending;                              // changed since the last commit
  std::vector<uint32_t> stale[2];                             // records a copy lacks (changed since it was written)
  uint64_t tail = 0, garbage = 0;                             // device entries in use / superseded
  int cur = 0;                                                // the record copy the fan-out reads
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses[2];    // last reading launch per stream, per copy
  uint64_t epoch = 0;
  uint64_t last_appended = 0, last_patched = 0;
  bool last_rebuilt = false;
};

struct Epoch {
  DevTable view{};
  int slot = 0;
  uint64_t id = 0;
  uint64_t n_filters = 0, n_nodes = 0, n_edges = 0, n_words = 0, bytes = 0;
  uint64_t fid_end = 0;   // every filter id of the epoch is below this (packed results: < 2^24)
};

struct CommitStats {
  uint64_t h2d = 0, d2d = 0, patched = 0;
  double ms = 0;
};

}  // namespace

struct egm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::recursive_mutex mu;
  HostTable table;
  std::shared_ptr<Epoch> cur;
  uint64_t next_epoch = 1;
  Slot slots[2];
  int cur_slot = -1;
  uint8_t* patch_host = nullptr;     // pinned staging of patch records
  size_t patch_host_cap = 0;
  DevBuf patch_dev;
  CommitStats last_commit;
  std::string err;

  // per-batch match workspaces: batches on different streams get different
  // ones, so consecutive batches overlap (one's compaction with the next one's
  // walk); a workspace reused from another stream waits for its last batch
  MatchWs ws[MATCH_WORKSPACES];
  uint32_t cur_ws = 0;           // workspace of the last batch (egm_last_stats)
  uint64_t ws_clock = 0;
  DevBuf in_blob, in_off, out_row, out_ids;
  uint32_t heavy_waves = 64;     // waves of the heavy kernel (rare path; each owns an HBM stack)
  uint32_t debug = 0;
  MatchStats last{};
  bool last_pending = false;
  hipStream_t last_stream = nullptr;

  // shard merge
  DevBuf m_srow, m_tiles, m_tot;
  // prefix partition routing
  DevBuf p_ctr, p_dst;

  // fan-out
  DevBuf sub_row, sub_rp, sub_rp2, sub_ids, f_dc, f_ds0, f_dpos, f_wbase, f_tiles, f_ovf, f_mrow, f_mids, f_drow,
      f_dfid, f_dsub;
  uint32_t n_fid_slots = 0;
  SubsState subs;
  DevBuf& sub_rec(int k) { return k ? sub_rp2 : sub_rp; }

  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_walk;   // pairs
  std::vector<hipEvent_t> ev_fan;
  std::vector<hipEvent_t> ev_free;
  double walk_ms = 0, fan_ms = 0;
  uint64_t walk_n = 0, fan_n = 0;

  // The per-context workspaces (match, fan-out, merge) are shared by every
  // launch, whatever stream the caller gives: a launch on a new stream first
  // waits for the last launch that used them (one event, recorded after each).
  hipEvent_t work_ev = nullptr;
  hipStream_t work_stream = nullptr;
  bool work_used = false;   // (the null stream is a stream: work_stream may be 0 after a launch)
  void work_begin(hipStream_t s) {
    if (work_used && work_stream != s && work_ev) hipStreamWaitEvent(s, work_ev, 0);
  }
  void work_end(hipStream_t s) {
    if (!work_ev && hipEventCreateWithFlags(&work_ev, hipEventDisableTiming) != hipSuccess) work_ev = nullptr;
    if (work_ev) hipEventRecord(work_ev, s);
    work_stream = s;
    work_used = true;
  }
  // host pipeline (egm_match_submit / egm_match_wait)
  std::vector<std::unique_ptr<PipeSlot>> pipe;
  std::condition_variable_any pipe_cv;   // a slot was freed (wait done, result freed, ticket cancelled)
  std::mutex cancel_mu;                  // guards cancel_q only (never held across another lock)
  std::vector<uint64_t> cancel_q;        // cancels that found the context busy (egm_match_cancel)
  hipStream_t copy_stream = nullptr;   // pipeline host->device copies
  hipStream_t d2h_stream = nullptr;    // pipeline device->host copies (PCIe is full duplex)
  hipStream_t d2h_stream2 = nullptr;   // ... the second half of the ids
  hipStream_t small_streams[MATCH_WORKSPACES] = {};   // small pipeline batches, round robin: they run side by side
  uint32_t small_rr = 0;
  // The copier thread (round 4): it waits for each launched batch's match
  // (ev_match; the stats, copied before it in stream order, hold the exact id
  // total) and enqueues the result's D2H as DMA copies of exactly that size.
  // A copy-out kernel storing to pinned memory instead (EGM_PIPE_COPY=kernel)
  // stalls the next batch's memory-bound kernels behind the PCIe writes
  // (k_tokenise 0.1 -> 1-2 ms beside it, profiles/r4_host_trace.json).
  std::thread copier;
  std::mutex cq_mu;                    // guards cq, cq_stop and every slot's launch/copied gens
  std::condition_variable cq_cv;       // work for the copier
  std::condition_variable copied_cv;   // a slot's D2H was enqueued
  std::vector<std::pair<PipeSlot*, uint64_t>> cq;
  bool cq_stop = false;
  uint64_t pipe_cap_hint = 0;
  // the last match launch's walk order, for a fan-out of the same rows (k_fan_count_ord)
  struct {
    const uint64_t* order = nullptr;   // null: that batch was walked in input order
    const uint64_t* row = nullptr;
    uint32_t n = 0, ws = 0;
  } last_walk;          // ids room a batch needed (overflow reruns): new slots start there
  // last fan-out (egm_last_fanout)
  const uint64_t* fan_drow = nullptr;
  uint32_t fan_topics = 0;
  hipStream_t fan_stream = nullptr;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip_fail(hipError_t e, const char* where) {
    err = std::string(where) + ": " + hipGetErrorString(e);
    return EGM_E_DEVICE;
  }
  hipEvent_t take_event() {
    if (!ev_free.empty()) {
      hipEvent_t e = ev_free.back();
      ev_free.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
  }
  void drain_timing() {
    for (size_t i = 0; i + 1 < ev_walk.size(); i += 2) {
      float ms = 0;
      hipEventSynchronize(ev_walk[i + 1]);
      hipEventElapsedTime(&ms, ev_walk[i], ev_walk[i + 1]);
      walk_ms += ms;
      ++walk_n;
      ev_free.push_back(ev_walk[i]);
      ev_free.push_back(ev_walk[i + 1]);
    }
    ev_walk.clear();
    for (size_t i = 0; i + 1 < ev_fan.size(); i += 2) {
      float ms = 0;
      hipEventSynchronize(ev_fan[i + 1]);
      hipEventElapsedTime(&ms, ev_fan[i], ev_fan[i + 1]);
      fan_ms += ms;
      ++fan_n;
      ev_free.push_back(ev_fan[i]);
      ev_free.push_back(ev_fan[i + 1]);
    }
    ev_fan.clear();
  }
};

static int set_device(egm_ctx* c) {
  hipError_t e = hipSetDevice(c->device);
  return e == hipSuccess ? 0 : c->hip_fail(e, "hipSetDevice");
}

// Wait for every queued launch that reads slot x (it is about to be written).
static void drain_slot(Slot& sl) {
  for (auto& u : sl.uses) {
    hipEventSynchronize(u.second);
    hipEventDestroy(u.second);
  }
  sl.uses.clear();
}

static void drain_uses(std::vector<std::pair<hipStream_t, hipEvent_t>>& u) {
  for (auto& p : u) {
    hipEventSynchronize(p.second);
    hipEventDestroy(p.second);
  }
  u.clear();
}

static void note_use(egm_ctx* c, int slot, hipStream_t s) {
  auto& u = c->slots[slot].uses;
  for (auto& p : u)
    if (p.first == s) {
      hipEventRecord(p.second, s);
      return;
    }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return;
  hipEventRecord(e, s);
  u.push_back({s, e});
}

// Sorted, unique indices.  Large logs go through a bitmap over the array
// (O(n + size/64)) rather than a sort.
static void sort_unique(std::vector<uint32_t>& v, uint64_t size = 0) {
  if (v.size() < 8192 || size == 0 || size > (1ull << 32)) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    return;
  }
  std::vector<uint64_t> bits((size + 63) / 64, 0);
  for (uint32_t i : v)
    if (i < size) bits[i >> 6] |= 1ull << (i & 63);
  v.clear();
  for (uint64_t w = 0; w < bits.size(); ++w)
    for (uint64_t b = bits[w]; b; b &= b - 1) v.push_back((uint32_t)(w * 64 + __builtin_ctzll(b)));
}

// out[i] = rec[idx[i]] for records of R bytes; the records are random reads
// of a multi-GB host image, so large patches use several threads.
template <size_t R>
static void gather(uint8_t* out, const void* rec, const std::vector<uint32_t>& idx) {
  const uint8_t* base = (const uint8_t*)rec;
  auto work = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) memcpy(out + i * R, base + (size_t)idx[i] * R, R);
  };
  const size_t n = idx.size();
  unsigned nt = std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  if (n < 65536 || nt == 1) {
    work(0, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n + nt - 1) / nt;
  for (unsigned k = 0; k < nt; ++k) {
    size_t lo = k * per, hi = std::min(n, lo + per);
    if (lo < hi) th.emplace_back(work, lo, hi);
  }
  for (auto& x : th) x.join();
}

// Bring one array of slot `dst` to the host image.  Preference order:
//  1. patch in place: the slot holds the image minus `need` (its pending log
//     plus this commit's), and it is big enough;
//  2. device copy from the current slot (which lacks only this commit's
//     changes `d`) followed by a patch of `d` — the slot was stale or too
//     small, the changes were not a rebuild;
//  3. whole upload from the host (rebuild: relayout, rehash, clear).
// Returns the indices still to patch in *idx (sorted, unique).
template <class T>
static int sync_array(egm_ctx* c, DevBuf& dst, uint64_t& held, const DevBuf* src, uint64_t src_held,
                      const std::vector<T>& host, bool need_full, bool d_full, const std::vector<uint32_t>& need,
                      const std::vector<uint32_t>& d, uint64_t headroom, std::vector<uint32_t>* idx,
                      const char* what) {
  const uint64_t n = host.size(), sz = sizeof(T);
  hipStream_t s = c->stream;
  hipError_t e;
  idx->clear();
  if (!need_full && held <= n && n * sz <= dst.cap && dst.p) {
    *idx = need;
  } else if (!d_full && src && src->p && src_held <= n) {
    if ((e = dst.ensure((n + headroom) * sz)) != hipSuccess) return c->hip_fail(e, what);
    if (src_held && (e = hipMemcpyAsync(dst.p, src->p, src_held * sz, hipMemcpyDeviceToDevice, s)) != hipSuccess)
      return c->hip_fail(e, what);
    c->last_commit.d2d += src_held * sz;
    *idx = d;
    for (uint64_t i = src_held; i < n; ++i) idx->push_back((uint32_t)i);   // appended beyond the copy
  } else {
    if ((e = dst.ensure((n + headroom) * sz + 16)) != hipSuccess) return c->hip_fail(e, what);
    if (n && (e = hipMemcpyAsync(dst.p, host.data(), n * sz, hipMemcpyHostToDevice, s)) != hipSuccess)
      return c->hip_fail(e, what);
    c->last_commit.h2d += n * sz;
  }
  sort_unique(*idx, n);
  while (!idx->empty() && idx->back() >= n) idx->pop_back();
  held = n;
  return EGM_OK;
}

// Append-only arrays (dictionary words and their offsets): upload the tail.
template <class T>
static int sync_tail(egm_ctx* c, DevBuf& dst, uint64_t& held, const DevBuf* src, uint64_t src_held,
                     const std::vector<T>& host, bool need_full, bool d_full, const char* what) {
  const uint64_t n = host.size(), sz = sizeof(T);
  hipStream_t s = c->stream;
  hipError_t e;
  uint64_t from;
  if (!need_full && held <= n && n * sz <= dst.cap && dst.p) {
    from = held;
  } else if (!d_full && src && src->p && src_held <= n) {
    if ((e = dst.ensure(n * sz + n * sz / 4 + 4096)) != hipSuccess) return c->hip_fail(e, what);
    if (src_held && (e = hipMemcpyAsync(dst.p, src->p, src_held * sz, hipMemcpyDeviceToDevice, s)) != hipSuccess)
      return c->hip_fail(e, what);
    c->last_commit.d2d += src_held * sz;
    from = src_held;
  } else {
    if ((e = dst.ensure(n * sz + n * sz / 4 + 4096)) != hipSuccess) return c->hip_fail(e, what);
    from = 0;
  }
  if (n > from) {
    if ((e = hipMemcpyAsync((uint8_t*)dst.p + from * sz, host.data() + from, (n - from) * sz,
                            hipMemcpyHostToDevice, s)) != hipSuccess)
      return c->hip_fail(e, what);
    c->last_commit.h2d += (n - from) * sz;
  }
  held = n;
  return EGM_OK;
}

static uint8_t* patch_stage(egm_ctx* c, size_t bytes) {
  if (bytes > c->patch_host_cap) {
    if (c->patch_host) hipHostFree(c->patch_host);
    c->patch_host = nullptr;
    c->patch_host_cap = 0;
    size_t want = bytes + bytes / 2 + 65536;
    if (hipHostMalloc((void**)&c->patch_host, want, hipHostMallocDefault) != hipSuccess) return nullptr;
    c->patch_host_cap = want;
  }
  return c->patch_host;
}

// Publish the host table as a new epoch (egm_table_commit).
static int commit_locked(egm_ctx* c, uint64_t* epoch) {
  auto t0 = std::chrono::steady_clock::now();
  c->last_commit = CommitStats{};
  const HostTable& t = c->table;
  DirtyLog d = c->table.take_dirty();
  // on any failure below, the changes go back into the table's log, so the
  // next commit publishes them (the half-written slot stays invalid)
  struct Restore {
    egm_ctx* c;
    const DirtyLog& d;
    bool armed = true;
    ~Restore() {
      if (armed) c->table.restore_dirty(d);
    }
  } restore{c, d};
  if (c->debug & EGM_DEBUG_FAIL_COMMIT) {   // test hook: a commit that fails after taking the log (one shot)
    c->debug &= ~EGM_DEBUG_FAIL_COMMIT;
    return c->fail(EGM_E_DEVICE, "commit: injected failure");
  }
  const int x = c->cur_slot < 0 ? 0 : 1 - c->cur_slot;
  Slot& S = c->slots[x];
  Slot* C = c->cur_slot < 0 ? nullptr : &c->slots[c->cur_slot];
  drain_slot(S);
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return c->hip_fail(e, "commit: stream");
  DirtyLog need = S.pending;
  need.merge(d);
  if (!S.valid) need.nodes_full = need.edges_full = need.dict_full = need.words_full = true;
  // a failure below leaves S half-written: it stays invalid (full copy next time)
  S.valid = false;
  const uint64_t nn = t.nodes.size();
  std::vector<uint32_t> in, ih, ie, id;
  int r;
  if ((r = sync_array(c, S.nodes, S.n_nodes, C ? &C->nodes : nullptr, C ? C->n_nodes : 0, t.nodes,
                      need.nodes_full, d.nodes_full, need.nodes, d.nodes, nn / 8 + 4096, &in, "nodes")) ||
      (r = sync_array(c, S.hash_child, S.n_hc, C ? &C->hash_child : nullptr, C ? C->n_hc : 0, t.hash_child,
                      need.nodes_full, d.nodes_full, need.nodes, d.nodes, nn / 8 + 4096, &ih, "hash_child")) ||
      (r = sync_array(c, S.edges, S.n_edges, C ? &C->edges : nullptr, C ? C->n_edges : 0, t.edges,
                      need.edges_full, d.edges_full, need.edges, d.edges, 0, &ie, "edges")) ||
      (r = sync_array(c, S.dict, S.n_dict, C ? &C->dict : nullptr, C ? C->n_dict : 0, t.dict, need.dict_full,
                      d.dict_full, need.dict, d.dict, 0, &id, "dict")) ||
      (r = sync_tail(c, S.dict_blob, S.n_blob, C ? &C->dict_blob : nullptr, C ? C->n_blob : 0, t.dict_blob,
                     need.words_full, d.words_full, "dict_blob")) ||
      (r = sync_tail(c, S.dict_off, S.n_off, C ? &C->dict_off : nullptr, C ? C->n_off : 0, t.dict_off,
                     need.words_full, d.words_full, "dict_off")))
    return r;
  // pack {indices, records} of all four patched arrays into one pinned buffer
  auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
  const size_t o_in = 0, o_rn = al(o_in + in.size() * 4), o_ih = o_rn + in.size() * 16,
               o_rh = al(o_ih + ih.size() * 4), o_ie = al(o_rh + ih.size() * 4), o_re = al(o_ie + ie.size() * 4),
               o_id = o_re + ie.size() * 32, o_rd = al(o_id + id.size() * 4), total = o_rd + id.size() * 32;
  const uint64_t np = in.size() + ih.size() + ie.size() + id.size();
  if (np) {
    uint8_t* h = patch_stage(c, total);
    if (!h) return c->fail(EGM_E_NOMEM, "commit: pinned staging");
    memcpy(h + o_in, in.data(), in.size() * 4);
    memcpy(h + o_ih, ih.data(), ih.size() * 4);
    memcpy(h + o_ie, ie.data(), ie.size() * 4);
    memcpy(h + o_id, id.data(), id.size() * 4);
    gather<16>(h + o_rn, t.nodes.data(), in);
    gather<4>(h + o_rh, t.hash_child.data(), ih);
    gather<32>(h + o_re, t.edges.data(), ie);
    gather<32>(h + o_rd, t.dict.data(), id);
    if ((e = c->patch_dev.ensure(total)) != hipSuccess) return c->hip_fail(e, "commit: patch buffer");
    if ((e = hipMemcpyAsync(c->patch_dev.p, h, total, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "commit: patch upload");
    c->last_commit.h2d += total;
    uint8_t* dp = (uint8_t*)c->patch_dev.p;
    if ((e = launch_patch(S.nodes.p, 16, (const uint32_t*)(dp + o_in), dp + o_rn, in.size(), c->stream)) ||
        (e = launch_patch(S.hash_child.p, 4, (const uint32_t*)(dp + o_ih), dp + o_rh, ih.size(), c->stream)) ||
        (e = launch_patch(S.edges.p, 32, (const uint32_t*)(dp + o_ie), dp + o_re, ie.size(), c->stream)) ||
        (e = launch_patch(S.dict.p, 32, (const uint32_t*)(dp + o_id), dp + o_rd, id.size(), c->stream)))
      return c->hip_fail(e, "commit: patch");
    c->last_commit.patched = np;
  }
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "commit: sync");
  restore.armed = false;
  S.valid = true;
  S.pending.clear();
  if (C) C->pending.merge(d);   // the previous epoch's slot now lacks this commit's changes

  auto ep = std::make_shared<Epoch>();
  ep->slot = x;
  ep->view.nodes = S.nodes.as<NodeRec>();
  ep->view.hash_child = S.hash_child.as<uint32_t>();
  ep->view.edges = S.edges.as<EdgeSlot>();
  ep->view.edge_mask = t.edge_mask();
  ep->view.dict = S.dict.as<DictSlot>();
  ep->view.dict_mask = t.dict_mask();
  ep->view.dict_blob = S.dict_blob.as<uint8_t>();
  ep->view.dict_off = S.dict_off.as<uint64_t>();
  ep->view.sig_packed = t.n_words() <= (1u << 27) ? 1u : 0u;
  ep->n_filters = t.n_filters();
  ep->n_nodes = t.n_nodes_live();
  ep->n_edges = t.n_edges();
  ep->n_words = t.n_words();
  ep->fid_end = t.next_fid();
  ep->bytes = S.bytes();
  ep->id = c->next_epoch++;
  c->cur = ep;
  c->cur_slot = x;
  if (epoch) *epoch = ep->id;
  c->last_commit.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return EGM_OK;
}

// Walk order: the sort key's bits per level as hex nibbles,
// level 0 in the lowest; 0 walks in input order.  EGM_WALK_KEY is a tuning
// knob for A/B runs (read at every batch); the default is the measured best:
// 4/6/7/7 bits over four levels — 24 bits, three sort passes (round 5, one
// process: 11.63 ms per C2 step against 11.75-11.78 for round 4's 6/8/10/8,
// whose fourth sort pass bought no walk time with the flush records; the
// walk 8.57 vs 8.58-8.61 ms; profiles/r5_walk_key_ab.jsonl).
constexpr uint32_t WALK_KEY_DEFAULT = 0x7764u;
static uint32_t walk_key_shape() {
  const char* v = getenv("EGM_WALK_KEY");
  const uint32_t shape = (v && *v) ? (uint32_t)strtoul(v, nullptr, 16) & 0xFFFFu : WALK_KEY_DEFAULT;   // KEY_LEVELS nibbles
  return walk_key_bits(shape) <= 32 ? shape : WALK_KEY_DEFAULT;
}

// EGM_WALK_SORT_MIN_BYTES: tables smaller than this are walked in input order.
// Sorting pays when the table is far larger than the caches (C2: 2.85 GB,
// 13.3 -> 12.7 ms per step); at C1 (357 MB, mostly MALL-resident) the walk
// gains 0.16 ms and the sort costs 0.4.
static uint64_t walk_sort_min_bytes() {
  const char* v = getenv("EGM_WALK_SORT_MIN_BYTES");
  return (v && *v) ? strtoull(v, nullptr, 10) : (1ull << 30);
}

// Test and A/B knobs of the flush records: EGM_FLUSH_AT — staged emits that
// trigger a flush (1..WALK_STAGE, default WALK_STAGE: small values make many
// short records per chunk); EGM_REC_SEG — u32 per record segment (default
// REC_GRAIN; small values make chunks' record chains jump between segments).
static uint32_t env_u32(const char* name, uint32_t dflt, uint32_t lo, uint32_t hi) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  const long long k = atoll(v);
  return (uint32_t)std::min<long long>(std::max<long long>(k, lo), hi);
}
static uint32_t flush_lim() { return env_u32("EGM_FLUSH_AT", walk_stage(), 1, walk_stage()); }
static uint32_t rec_grain() { return env_u32("EGM_REC_SEG", REC_GRAIN, 64, 1u << 24) & ~(uint32_t)(EGM_REC_ALIGN - 1); }

// The workspace for a batch on stream s: the one that last ran on s (stream
// order protects it), else the least recently used one, ordered after its
// last batch on the other stream.
static MatchWs& pick_ws(egm_ctx* c, hipStream_t s) {
  uint32_t k = 0;
  for (uint32_t i = 0; i < MATCH_WORKSPACES; ++i) {
    if (c->ws[i].stream == s && c->ws[i].used) {
      k = i;
      break;
    }
    if (c->ws[i].used < c->ws[k].used) k = i;
  }
  MatchWs& W = c->ws[k];
  if (W.used && W.stream != s && W.ev) hipStreamWaitEvent(s, W.ev, 0);   // (stream 0 is a stream too)
  c->cur_ws = k;
  W.used = ++c->ws_clock;
  return W;
}

// max_levels: an upper bound on the levels of any topic of the batch (the
// heavy kernel's stack must hold the deepest one's DFS, egm_kernels.hip).
static int ensure_work(egm_ctx* c, MatchWs& W, uint32_t n, uint64_t blob_bytes, uint64_t ids_cap,
                       uint64_t max_levels) {
  hipError_t e;
  const uint64_t nn = (uint64_t)n + 1;
  if ((e = W.wid.ensure((blob_bytes + nn) * 4)) != hipSuccess) return c->hip_fail(e, "wid");
  if ((e = W.lv.ensure(nn * 4)) != hipSuccess) return c->hip_fail(e, "lv");
  if ((e = W.tfl.ensure(nn)) != hipSuccess) return c->hip_fail(e, "tfl");
  if ((e = W.cnt.ensure(nn * 4)) != hipSuccess) return c->hip_fail(e, "cnt");
  // flush records: sized for the worst case of the batch's id capacity
  W.flush_lim = flush_lim();
  W.rec_grain = rec_grain();
  const uint64_t rcap = rec_capacity(ids_cap, n, W.flush_lim, W.rec_grain);
  if ((e = W.rec.ensure(rcap * 4)) != hipSuccess) return c->hip_fail(e, "flush records");
  W.rec_cap = W.rec.cap / 4;
  if (W.rec_cap >= (1ull << 34)) return c->fail(EGM_E_INVAL, "batch too large: > 16G u32 of flush records (split it)");
  if ((e = W.chunks.ensure(walk_chunk_cap(n) * 16)) != hipSuccess) return c->hip_fail(e, "chunk records");
  if ((e = W.dir.ensure(walk_chunk_cap(n) * REC_DIR * 4)) != hipSuccess)
    return c->hip_fail(e, "chunk directories");
  // heavy topics: their ids (count then fill, one piece per topic)
  const uint64_t tcap = ids_cap + 4096;
  if (tcap >= 0xFFFFFFF0ull) return c->fail(EGM_E_INVAL, "batch too large: > 4G matched ids (split it)");
  if ((e = W.ids_tmp.ensure(tcap * 4)) != hipSuccess) return c->hip_fail(e, "ids_tmp");
  W.ids_tmp_cap = W.ids_tmp.cap / 4;
  if ((e = W.pieces.ensure(((uint64_t)n + 4096) * 16)) != hipSuccess) return c->hip_fail(e, "pieces");
  W.pieces_cap = std::min<uint64_t>(W.pieces.cap / 16, 0xFFFFFFF0ull);
  if ((e = W.deferred.ensure(walk_chunk_cap(n) * 4 * 2)) != hipSuccess) return c->hip_fail(e, "deferred");
  const uint32_t hcap = heavy_stack_items(max_levels);
  if ((e = W.heavy_stack.ensure((uint64_t)c->heavy_waves * hcap * 16)) != hipSuccess)
    return c->hip_fail(e, "heavy stack");
  W.heavy_cap = (uint32_t)std::min<uint64_t>(W.heavy_stack.cap / 16 / c->heavy_waves, 0xFFFFFFFFull);
  if ((e = W.tile_sums.ensure((scan_tiles(n) + 2) * 8)) != hipSuccess) return c->hip_fail(e, "tile_sums");
  if ((e = W.stats.ensure(sizeof(MatchStats))) != hipSuccess) return c->hip_fail(e, "stats");
  const uint32_t shape = walk_key_shape();
  if (shape) {
    if ((e = W.skey.ensure(nn * 4)) != hipSuccess) return c->hip_fail(e, "sort keys");
    if ((e = W.skey_out.ensure(nn * 4)) != hipSuccess) return c->hip_fail(e, "sort keys");
    if ((e = W.sval.ensure(nn * 8)) != hipSuccess) return c->hip_fail(e, "sort values");
    if ((e = W.order.ensure(nn * 8)) != hipSuccess) return c->hip_fail(e, "walk order");
    if ((e = W.wfix.ensure(nn * 4 * FIX_WORDS)) != hipSuccess) return c->hip_fail(e, "fixed-stride words");

    if ((e = W.sort_tmp.ensure(walk_sort_temp_bytes(n, shape))) != hipSuccess) return c->hip_fail(e, "sort scratch");
  }
  if (!W.ev && (e = hipEventCreateWithFlags(&W.ev, hipEventDisableTiming)) != hipSuccess)
    return c->hip_fail(e, "workspace event");
  return EGM_OK;
}

static MatchWork work_view(egm_ctx* c, MatchWs& W) {
  MatchWork w{};
  w.wid = W.wid.as<uint32_t>();
  w.lv = W.lv.as<uint32_t>();
  w.tfl = W.tfl.as<uint8_t>();
  w.cnt = W.cnt.as<uint32_t>();
  w.rec = W.rec.as<uint32_t>();
  w.rec_cap = W.rec_cap;
  w.rec_grain = W.rec_grain;
  w.flush_lim = W.flush_lim;
  w.chunks = W.chunks.as<uint4>();
  w.dir = W.dir.as<uint32_t>();
  w.ids_tmp = W.ids_tmp.as<uint32_t>();
  w.ids_cap = W.ids_tmp_cap;   // ids_tmp entries (the output capacity is MatchOut's)
  w.pieces = W.pieces.as<uint4>();
  w.pieces_cap = W.pieces_cap;
  w.deferred = W.deferred.as<uint32_t>();
  w.deep = w.deferred + W.deferred.cap / 8;   // the second half: the walk's deep-pass list
  w.heavy_stack = W.heavy_stack.as<uint4>();
  w.heavy_waves = c->heavy_waves;
  w.heavy_cap = W.heavy_cap;
  w.tile_sums = W.tile_sums.as<uint64_t>();
  w.stats = W.stats.as<MatchStats>();
  w.debug = c->debug;
  w.key_shape = walk_key_shape();
  if (w.key_shape && W.order.p) {
    w.skey = W.skey.as<uint32_t>();
    w.skey_out = W.skey_out.as<uint32_t>();
    w.sval = W.sval.as<uint64_t>();
    w.order = W.order.as<uint64_t>();
    w.wfix = W.wfix.as<uint32_t>();

    w.sort_tmp = W.sort_tmp.p;
    w.sort_tmp_bytes = W.sort_tmp.cap;
  } else {
    w.key_shape = 0;
  }

  return w;
}

static int run_match(egm_ctx* c, MatchWs& W, const Epoch& ep, const uint8_t* d_blob, const uint32_t* d_off,
                     uint32_t n, int mode, hipStream_t s, uint64_t* d_row, uint32_t* d_ids, uint64_t ids_cap,
                     const uint32_t* d_n_live = nullptr, uint32_t* d_topic = nullptr) {
  MatchWork w = work_view(c, W);
  w.n_live = d_n_live;
  if (ep.bytes < walk_sort_min_bytes()) w.key_shape = 0;   // the table fits the caches: the order buys nothing
  MatchOut o{d_row, d_ids, ids_cap, d_topic};
  hipEvent_t evp[2] = {nullptr, nullptr};
  if (c->timing) {
    evp[0] = c->take_event();
    evp[1] = c->take_event();
  }
  bool walk_sorted = false;
  hipError_t e = launch_match(ep.view, d_blob, d_off, n, mode, w, o, s, c->timing ? evp : nullptr, &walk_sorted);
  c->last_walk.order = (walk_sorted && !d_topic) ? w.order : nullptr;   // (walk-order rows: already in that order)
  c->last_walk.row = d_row;
  c->last_walk.n = n;
  c->last_walk.ws = (uint32_t)(&W - c->ws);
  note_use(c, ep.slot, s);   // a later commit must not overwrite this slot before the walk is done
  if (c->timing) {
    c->ev_walk.push_back(evp[0]);
    c->ev_walk.push_back(evp[1]);
  }
  if (e != hipSuccess) return c->hip_fail(e, "launch_match");
  c->last_pending = true;
  c->last_stream = s;
  return EGM_OK;
}

// After the batch's last use of W on s (a flags/counts copy included).
static void ws_done(MatchWs& W, hipStream_t s) {
  hipEventRecord(W.ev, s);
  W.stream = s;
}

static int sync_last(egm_ctx* c) {
  if (!c->last_pending) return EGM_OK;
  hipError_t e = hipStreamSynchronize(c->last_stream);
  if (e != hipSuccess) return c->hip_fail(e, "hipStreamSynchronize");
  e = hipMemcpy(&c->last, c->ws[c->cur_ws].stats.p, sizeof(MatchStats), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return c->hip_fail(e, "stats readback");
  c->last_pending = false;
  return EGM_OK;
}

static bool valid_offsets(const uint32_t* off, uint32_t n) {
  if (!off) return false;
  for (uint32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return false;
  return true;
}

// Check a batch of inserts against the table before changing anything (the
// reference applies route changes in all-or-nothing mnesia transactions,
// emqx_router.erl:252-303): every new filter's id must be < WID_MAX, unused by
// a live filter (deletes of the same delta apply after the inserts) and not
// claimed twice in the batch.  Filters already present (or repeated in the
// batch) are idempotent no-ops (emqx_trie.erl:84-86).
static bool validate_inserts(const HostTable& t, const uint8_t* blob, const uint32_t* off, uint32_t n,
                             const uint32_t* ids, bool from_empty, std::string* why) {
  if (!ids) return true;   // ids assigned by the table
  std::unordered_set<std::string> seen_bytes;
  std::unordered_set<uint32_t> seen_ids;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* p = blob + off[i];
    const uint32_t len = off[i + 1] - off[i];
    std::string key((const char*)p, len);
    if (!from_empty && t.lookup(p, len) != NONE) continue;
    if (!seen_bytes.insert(key).second) continue;
    const uint32_t id = ids[i];
    if (id == NONE) continue;
    if (id >= WID_MAX || (!from_empty && t.id_in_use(id)) || !seen_ids.insert(id).second) {
      *why = "bad or duplicate filter id at index " + std::to_string(i);
      return false;
    }
  }
  return true;
}

// egm_table_build uses the parallel bulk build from EGM_BULK_MIN filters on
// (default 65 536; 0 = always), unless an id asks to be assigned (NONE).
static bool use_bulk_build(uint32_t n, const uint32_t* ids) {
  const char* e = getenv("EGM_BULK_MIN");
  const uint64_t lim = (e && *e) ? strtoull(e, nullptr, 10) : 65536;
  if (n < lim) return false;
  if (ids)
    for (uint32_t i = 0; i < n; ++i)
      if (ids[i] == NONE) return false;
  return true;
}

// fn(lo, hi) over [0, n) on up to 8 threads, `grain` items or more each
// (the host side of a 1M-topic batch: one core stages ~10 GB/s into pinned
// memory, the PCIe link takes ~50; round 3 copied a 39 MB batch on one core).
template <class F>
static void par_for(size_t n, size_t grain, F fn) {
  const unsigned nt = (unsigned)std::min<size_t>(8, std::max<size_t>(1, n / std::max<size_t>(grain, 1)));
  if (nt <= 1) {
    fn((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (n + nt - 1) / nt;
  for (unsigned k = 1; k < nt; ++k) {
    const size_t lo = k * per, hi = std::min(n, lo + per);
    if (lo < hi) th.emplace_back([=] { fn(lo, hi); });
  }
  fn((size_t)0, std::min(n, per));
  for (auto& x : th) x.join();
}

extern "C" {

const char* egm_version(void) { return "emqx_gpu_match 0.1 (gfx950)"; }

int egm_open(const egm_config* cfg, egm_ctx** out) {
  if (!out) return EGM_E_INVAL;
  *out = nullptr;
  egm_ctx* c = new (std::nothrow) egm_ctx();
  if (!c) return EGM_E_NOMEM;
  c->device = cfg ? cfg->device : 0;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= c->device || c->device < 0) {
    delete c;
    return EGM_E_DEVICE;
  }
  if (set_device(c) != 0 || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return EGM_E_DEVICE;
  }
  if (commit_locked(c, nullptr) != EGM_OK) {  // empty epoch
    hipStreamDestroy(c->stream);
    delete c;
    return EGM_E_DEVICE;
  }
  if (cfg && cfg->max_batch)
    ensure_work(c, c->ws[0], cfg->max_batch, (uint64_t)cfg->max_batch * 64, (uint64_t)cfg->max_batch * 4, 1024);
  *out = c;
  return EGM_OK;
}

void egm_close(egm_ctx* c) {
  if (!c) return;
  {
    std::lock_guard<std::recursive_mutex> g(c->mu);
    set_device(c);
    hipStreamSynchronize(c->stream);
    c->drain_timing();
    for (hipEvent_t e : c->ev_free) hipEventDestroy(e);
    c->cur.reset();
    drain_slot(c->slots[0]);
    drain_slot(c->slots[1]);
    if (c->patch_host) hipHostFree(c->patch_host);
    c->patch_host = nullptr;
    drain_uses(c->subs.uses[0]);
    drain_uses(c->subs.uses[1]);
    if (c->work_ev) hipEventDestroy(c->work_ev);
    c->work_ev = nullptr;
    if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
  }
  if (c->copier.joinable()) {   // outside the context lock: the copier never takes it
    {
      std::lock_guard<std::mutex> q(c->cq_mu);
      c->cq_stop = true;
    }
    c->cq_cv.notify_all();
    c->copier.join();
  }
  {
    std::lock_guard<std::recursive_mutex> g(c->mu);
    set_device(c);
    if (c->d2h_stream) hipStreamSynchronize(c->d2h_stream);
    if (c->d2h_stream2) hipStreamSynchronize(c->d2h_stream2);
    for (auto& ss : c->small_streams)
      if (ss) {
        hipStreamSynchronize(ss);
        hipStreamDestroy(ss);
        ss = nullptr;
      }
    c->pipe.clear();
    if (c->copy_stream) hipStreamDestroy(c->copy_stream);
    if (c->d2h_stream) hipStreamDestroy(c->d2h_stream);
    if (c->d2h_stream2) hipStreamDestroy(c->d2h_stream2);
    c->copy_stream = c->d2h_stream = c->d2h_stream2 = nullptr;
  }
  hipStreamDestroy(c->stream);
  delete c;
}

const char* egm_last_error(egm_ctx* c) { return c ? c->err.c_str() : "null context"; }

// A host allocation failure inside an entry point is reported, never thrown
// across the C ABI (a std::bad_alloc escaping an extern "C" function would
// terminate the embedding BEAM node).
extern "C++" {
template <class F>
inline int no_throw(egm_ctx* c, const char* what, F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return c->fail(EGM_E_NOMEM, what);
  } catch (const std::exception& ex) {
    return c->fail(EGM_E_DEVICE, ex.what());
  }
}
}  // extern "C++"

int egm_table_build(egm_ctx* c, const uint8_t* blob, const uint32_t* off, uint32_t n, const uint32_t* ids) {
  if (!c || (n && (!blob || !valid_offsets(off, n)))) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  return no_throw(c, "table build: host allocation", [&] {
  std::string why;
  if (!validate_inserts(c->table, blob, off, n, ids, true, &why)) return c->fail(EGM_E_INVAL, why);
  if (use_bulk_build(n, ids)) {   // parallel: the same image as the insert loop below (egm_bulk.cpp)
    if (c->table.bulk_build(blob, off, n, ids, 0) < 0) {
      c->table.clear();
      return c->fail(EGM_E_INVAL, "table too large (node ids exhausted)");
    }
    return commit_locked(c, nullptr);
  }
  c->table.clear();
  for (uint32_t i = 0; i < n; ++i) {
    int r = c->table.insert(blob + off[i], off[i + 1] - off[i], ids ? ids[i] : i, nullptr);
    if (r < 0) return c->fail(EGM_E_INVAL, "bad or duplicate filter id at index " + std::to_string(i));
  }
  c->table.relayout();
  return commit_locked(c, nullptr);
  });
}

int egm_table_apply_delta(egm_ctx* c, const egm_delta* ins, const egm_delta* del) {
  if (!c) return EGM_E_INVAL;
  if (ins && ins->n && (!ins->blob || !valid_offsets(ins->offsets, ins->n))) return EGM_E_INVAL;
  if (del && del->n && (!del->blob || !valid_offsets(del->offsets, del->n))) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  return no_throw(c, "table delta: host allocation", [&] {
  std::string why;
  if (ins && !validate_inserts(c->table, ins->blob, ins->offsets, ins->n, ins->ids, false, &why))
    return c->fail(EGM_E_INVAL, why);   // nothing staged
  if (ins)
    for (uint32_t i = 0; i < ins->n; ++i) {
      int r = c->table.insert(ins->blob + ins->offsets[i], ins->offsets[i + 1] - ins->offsets[i],
                              ins->ids ? ins->ids[i] : NONE, nullptr);
      if (r < 0) return c->fail(EGM_E_INVAL, "bad or duplicate filter id at insert " + std::to_string(i));
    }
  if (del)
    for (uint32_t i = 0; i < del->n; ++i)
      c->table.remove(del->blob + del->offsets[i], del->offsets[i + 1] - del->offsets[i]);
  return EGM_OK;
  });
}

int egm_table_commit(egm_ctx* c, uint64_t* epoch) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  return no_throw(c, "table commit: host allocation", [&] { return commit_locked(c, epoch); });
}

int egm_table_epoch(egm_ctx* c, uint64_t* epoch) {
  if (!c || !epoch) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  *epoch = c->cur ? c->cur->id : 0;
  return EGM_OK;
}

int egm_table_empty(egm_ctx* c) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  return c->cur->n_filters == 0 ? 1 : 0;
}

int egm_table_stats(egm_ctx* c, uint64_t* nf, uint64_t* nn, uint64_t* ne, uint64_t* nw, uint64_t* bytes) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (nf) *nf = c->cur->n_filters;
  if (nn) *nn = c->cur->n_nodes;
  if (ne) *ne = c->cur->n_edges;
  if (nw) *nw = c->cur->n_words;
  if (bytes) *bytes = c->cur->bytes;
  return EGM_OK;
}

int egm_filter_id(egm_ctx* c, const uint8_t* f, uint32_t len, uint32_t* id) {
  if (!c || (!f && len) || !id) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  uint32_t r = c->table.lookup(f, len);
  if (r == NONE) return EGM_E_NOTFOUND;
  *id = r;
  return EGM_OK;
}

int egm_filter_bytes(egm_ctx* c, uint32_t id, const uint8_t** bytes, uint32_t* len) {
  if (!c || !bytes || !len) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  const uint8_t* p = c->table.filter_bytes(id, len);
  if (!p) return EGM_E_NOTFOUND;
  *bytes = p;
  return EGM_OK;
}

int egm_match_device(egm_ctx* c, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_off, uint32_t n,
                     int mode, void* hip_stream, uint64_t* d_row, uint32_t* d_ids, uint64_t ids_cap,
                     uint8_t* d_flags) {
  if (!c || (mode != EGM_MODE_TRIE && mode != EGM_MODE_ROUTES) || !d_row) return EGM_E_INVAL;
  if (n && (!d_blob || !d_off || ((uintptr_t)d_blob & 3))) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  // a topic has at most (its bytes + 1) levels, and a legal one at most 65 536
  // (emqx_topic.erl:45, 99-100): bound the device batch's depth by its blob
  MatchWs& W = pick_ws(c, s);
  int r = ensure_work(c, W, n, blob_bytes, ids_cap, std::min<uint64_t>(blob_bytes, 65535) + 1);
  if (r) return r;
  std::shared_ptr<Epoch> ep = c->cur;
  r = run_match(c, W, *ep, d_blob, d_off, n, mode, s, d_row, d_ids, ids_cap);
  if (r == EGM_OK && d_flags && n) {
    hipError_t e = hipMemcpyAsync(d_flags, W.tfl.p, n, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) r = c->hip_fail(e, "flags copy");
  }
  ws_done(W, s);
  return r;
}

int egm_match_device_ordered(egm_ctx* c, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_off,
                             uint32_t n, int mode, void* hip_stream, uint64_t* d_row, uint32_t* d_topic,
                             uint32_t* d_ids, uint64_t ids_cap) {
  if (!c || (mode != EGM_MODE_TRIE && mode != EGM_MODE_ROUTES) || !d_row || (n && !d_topic)) return EGM_E_INVAL;
  if (n && (!d_blob || !d_off || ((uintptr_t)d_blob & 3))) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  MatchWs& W = pick_ws(c, s);
  int r = ensure_work(c, W, n, blob_bytes, ids_cap, std::min<uint64_t>(blob_bytes, 65535) + 1);
  if (r) return r;
  std::shared_ptr<Epoch> ep = c->cur;
  r = run_match(c, W, *ep, d_blob, d_off, n, mode, s, d_row, d_ids, ids_cap, nullptr, d_topic ? d_topic : nullptr);
  ws_done(W, s);
  return r;
}

int egm_match_device_counted(egm_ctx* c, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_off,
                             uint32_t n_max, const uint32_t* d_n, int mode, void* hip_stream, uint64_t* d_row,
                             uint32_t* d_ids, uint64_t ids_cap) {
  return egm_match_device_counted_ordered(c, d_blob, blob_bytes, d_off, n_max, d_n, mode, hip_stream, d_row, nullptr,
                                          d_ids, ids_cap);
}

int egm_match_device_counted_ordered(egm_ctx* c, const uint8_t* d_blob, uint64_t blob_bytes, const uint32_t* d_off,
                                     uint32_t n_max, const uint32_t* d_n, int mode, void* hip_stream, uint64_t* d_row,
                                     uint32_t* d_topic, uint32_t* d_ids, uint64_t ids_cap) {
  if (!c || (mode != EGM_MODE_TRIE && mode != EGM_MODE_ROUTES) || !d_row || !d_n) return EGM_E_INVAL;
  if (n_max && (!d_blob || !d_off || ((uintptr_t)d_blob & 3))) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  MatchWs& W = pick_ws(c, s);
  int r = ensure_work(c, W, n_max, blob_bytes, ids_cap, std::min<uint64_t>(blob_bytes, 65535) + 1);
  if (r) return r;
  std::shared_ptr<Epoch> ep = c->cur;
  r = run_match(c, W, *ep, d_blob, d_off, n_max, mode, s, d_row, d_ids, ids_cap, d_n, d_topic);
  ws_done(W, s);
  return r;
}

int egm_last_commit_stats(egm_ctx* c, uint64_t* h2d_bytes, uint64_t* d2d_bytes, uint64_t* patched,
                          double* ms) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (h2d_bytes) *h2d_bytes = c->last_commit.h2d;
  if (d2d_bytes) *d2d_bytes = c->last_commit.d2d;
  if (patched) *patched = c->last_commit.patched;
  if (ms) *ms = c->last_commit.ms;
  return EGM_OK;
}

int egm_last_walk_counters(egm_ctx* c, uint64_t* iters, uint64_t* popped, uint64_t* bounded, uint64_t* lit_probes,
                           uint64_t* plus_reads) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  int r = sync_last(c);
  if (r) return r;
  if (iters) *iters = c->last.iters;
  if (popped) *popped = c->last.popped;
  if (bounded) *bounded = c->last.bounded;
  if (lit_probes) *lit_probes = c->last.lit_probes;
  if (plus_reads) *plus_reads = c->last.plus_reads;
  return EGM_OK;
}

int egm_last_walk_probes(egm_ctx* c, uint64_t* slow_lanes, uint64_t* slow_iters) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  int r = sync_last(c);
  if (r) return r;
  if (slow_lanes) *slow_lanes = c->last.slow_lanes;
  if (slow_iters) *slow_iters = c->last.slow_iters;
  return EGM_OK;
}

int egm_last_stats(egm_ctx* c, uint64_t* n_ids, uint64_t* visited, uint32_t* n_def, uint32_t* overflow,
                   uint32_t* n_error) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  int r = sync_last(c);
  if (r) return r;
  if (n_ids) *n_ids = c->last.total_ids;
  if (visited) *visited = c->last.visited;
  if (n_def) *n_def = c->last.n_deferred;
  if (overflow) *overflow = c->last.overflow;
  if (n_error) *n_error = c->last.errors;
  if (c->last.guard)   // a kernel invariant failed: the batch's rows are not valid (never a capacity problem)
    return c->fail(EGM_E_DEVICE, "walk guard tripped (bits " + std::to_string(c->last.guard) +
                                     "): kernel invariant failed, batch not matched");
  return EGM_OK;
}

int egm_last_guard(egm_ctx* c, uint32_t* guard) {
  if (!c || !guard) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  int r = sync_last(c);
  if (r) return r;
  *guard = c->last.guard;
  return EGM_OK;
}

int egm_set_debug(egm_ctx* c, uint32_t flags) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->debug = flags;
  return EGM_OK;
}

int egm_set_timing(egm_ctx* c, int enable) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->drain_timing();
  c->timing = enable != 0;
  c->walk_ms = c->fan_ms = 0;
  c->walk_n = c->fan_n = 0;
  return EGM_OK;
}

int egm_get_timing(egm_ctx* c, double* walk_ms, uint64_t* walk_n, double* fan_ms, uint64_t* fan_n) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->drain_timing();
  if (walk_ms) *walk_ms = c->walk_ms;
  if (walk_n) *walk_n = c->walk_n;
  if (fan_ms) *fan_ms = c->fan_ms;
  if (fan_n) *fan_n = c->fan_n;
  return EGM_OK;
}

static void par_copy(void* dst, const void* src, size_t bytes) {
  par_for(bytes, 4u << 20, [=](size_t lo, size_t hi) { memcpy((uint8_t*)dst + lo, (const uint8_t*)src + lo, hi - lo); });
}

// How a pipeline result reaches pinned memory (EGM_PIPE_COPY, A/B):
//   dma (default) — the copier thread, SDMA engines through the HSA runtime
//   hip           — the copier thread, hipMemcpyAsync (a blit kernel here)
//   kernel        — a copy-out kernel on the d2h stream, sized on the device
enum { PIPE_DMA = 0, PIPE_HIP = 1, PIPE_KERNEL = 2 };
static int pipe_copy_mode() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("EGM_PIPE_COPY");
    v = (e && strcmp(e, "kernel") == 0) ? PIPE_KERNEL : (e && strcmp(e, "hip") == 0) ? PIPE_HIP : PIPE_DMA;
  }
  return v;
}
static bool pipe_copy_kernel() { return pipe_copy_mode() == PIPE_KERNEL; }
// EGM_PIPE_COPY set explicitly: every batch takes that copy (A/B), small ones too
static bool pipe_copy_forced() {
  static const bool v = getenv("EGM_PIPE_COPY") != nullptr;
  return v;
}
// Batches up to this many topics take the small-batch result path (pipe_launch).
constexpr uint64_t PIPE_SMALL_TOPICS = 16384;   // (65536 measured: the copy-out on the match's
                                                 // stream then costs more than the SDMA path's overlap)

// EGM_PIPE_TRACE=1: one stderr line per pipeline event with a ms clock
// (diagnostics of the host pipeline's bubbles).
static void ptrace(const char* what, const void* slot, uint64_t gen) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("EGM_PIPE_TRACE");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  if (v != 1) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fprintf(stderr, "[pipe] %10.3f %-14s %p %llu\n", ms, what, slot, (unsigned long long)gen);
}

// Enqueue one staged batch of slot S: H2D on the copy stream, the match on
// the context stream once the input is in, then the batch's flags and
// counters copied out in stream order (the next batch reuses the workspace).
static int pipe_launch(egm_ctx* c, PipeSlot& S) {
  hipError_t e;
  hipStream_t s = c->stream;
  const uint64_t n = S.n;
  const bool small = n <= PIPE_SMALL_TOPICS && !pipe_copy_forced();
  if (small) {
    // a small batch fills a fraction of the GPU: consecutive ones run side by
    // side, each on its own stream and workspace (pick_ws orders a workspace
    // last used on another stream after that use)
    hipStream_t& ss = c->small_streams[c->small_rr++ % MATCH_WORKSPACES];
    if (!ss && (e = hipStreamCreateWithFlags(&ss, hipStreamNonBlocking)) != hipSuccess)
      return c->hip_fail(e, "small-batch stream");
    s = ss;
  }
  std::shared_ptr<Epoch> ep = c->cur;
  S.epoch = ep->id;
  MatchWs& W = pick_ws(c, s);
  int r = ensure_work(c, W, S.n, S.bytes, S.cap, S.maxlen + 1);
  if (r) return r;
  if ((e = S.d_row.ensure((n + 1) * 8)) != hipSuccess) return c->hip_fail(e, "pipe row");
  if ((e = S.d_ids.ensure((S.cap + 4) * 4)) != hipSuccess) return c->hip_fail(e, "pipe ids");   // (+4: the packer reads groups of 4)
  if ((e = S.d_flags.ensure(n + 8)) != hipSuccess) return c->hip_fail(e, "pipe flags");
  if ((e = S.h_stats.ensure(sizeof(MatchStats))) != hipSuccess) return c->hip_fail(e, "pipe stats");
  const OutLayout ol = out_layout(n, S.cap);
  if ((e = S.h_out.ensure(ol.total)) != hipSuccess) return c->hip_fail(e, "pipe pinned result");
  if ((e = hipStreamWaitEvent(s, S.ev_in, 0)) != hipSuccess) return c->hip_fail(e, "pipe wait input");
  r = run_match(c, W, *ep, S.d_in.as<uint8_t>(), (const uint32_t*)(S.d_in.as<uint8_t>() + S.o_off), S.n, S.mode, s,
                S.d_row.as<uint64_t>(), S.d_ids.as<uint32_t>(), S.cap);
  if (r) {
    ws_done(W, s);
    return r;
  }
  c->last_pending = false;   // this batch's counters travel with the slot
  // the packed form (EGM_RESULT_PACKED, egm_pack.h): large batches on the copier's path whose
  // epoch's filter ids fit 24 bits; the packer runs on the match's stream, before ev_match
  S.packed = S.want_packed && !small && !pipe_copy_kernel() && ep->fid_end <= (1ull << 24) && S.cap < (1ull << 31);
  if (S.packed) {
    if ((e = S.d_row32.ensure((n + 1) * 4)) != hipSuccess || (e = S.d_pk.ensure(S.cap * 3 + 16)) != hipSuccess ||
        (e = launch_pack_result(S.d_row.as<uint64_t>(), (uint32_t)n, S.d_ids.as<uint32_t>(), S.cap,
                                S.d_row32.as<uint32_t>(), S.d_pk.as<uint8_t>(), s)) != hipSuccess) {
      ws_done(W, s);
      return c->hip_fail(e, "pipe pack");
    }
  }
  if (small) {
    // A small batch (the Erlang batcher's: 4096 by default) is latency-bound,
    // not bandwidth-bound: its result goes to pinned memory by a copy-out
    // kernel on the match's own stream — flags read from the workspace, the
    // counters too — so no D2D copy, no copier-thread hand-off and no SDMA
    // round trips (round 6: ~330 us -> see DESIGN §6 "small batches").
    uint8_t* h = (uint8_t*)S.h_out.p;
    if ((e = launch_copy_out(S.d_row.as<uint64_t>(), (uint32_t)n, S.d_ids.as<uint32_t>(), S.cap, W.tfl.as<uint8_t>(),
                             h + ol.o_row, h + ol.o_ids, h + ol.o_fl, s, W.stats.as<MatchStats>(),
                             (MatchStats*)S.h_stats.p)) != hipSuccess ||
        (e = hipEventRecord(S.ev_match, s)) != hipSuccess || (e = hipEventRecord(S.ev_done, s)) != hipSuccess) {
      ws_done(W, s);
      return c->hip_fail(e, "pipe copy-out (small batch)");
    }
    ws_done(W, s);
    std::lock_guard<std::mutex> q(c->cq_mu);
    S.copied_gen = ++S.launch_gen;
    return EGM_OK;
  }
  if ((n && (e = hipMemcpyAsync(S.d_flags.p, W.tfl.p, n, hipMemcpyDeviceToDevice, s)) != hipSuccess) ||
      (e = hipMemcpyAsync(S.h_stats.p, W.stats.p, sizeof(MatchStats), hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipEventRecord(S.ev_match, s)) != hipSuccess) {
    ws_done(W, s);
    return c->hip_fail(e, "pipe epilogue");
  }
  ws_done(W, s);
  if (pipe_copy_kernel()) {
    // the CSR straight into pinned memory by a kernel, sized on the device
    uint8_t* h = (uint8_t*)S.h_out.p;
    if ((e = hipStreamWaitEvent(c->d2h_stream, S.ev_match, 0)) != hipSuccess ||
        (e = launch_copy_out(S.d_row.as<uint64_t>(), (uint32_t)n, S.d_ids.as<uint32_t>(), S.cap,
                             S.d_flags.as<uint8_t>(), h + ol.o_row, h + ol.o_ids, h + ol.o_fl, c->d2h_stream)) !=
            hipSuccess ||
        (e = hipEventRecord(S.ev_done, c->d2h_stream)) != hipSuccess)
      return c->hip_fail(e, "pipe copy-out");
    std::lock_guard<std::mutex> q(c->cq_mu);
    S.copied_gen = ++S.launch_gen;
    return EGM_OK;
  }
  {   // the copier enqueues the D2H once the match is done
    std::lock_guard<std::mutex> q(c->cq_mu);
    c->cq.emplace_back(&S, ++S.launch_gen);
  }
  c->cq_cv.notify_one();
  return EGM_OK;
}

// The copier thread's loop (egm_ctx::copier): in launch order, wait for a
// batch's match, then enqueue its result's D2H — row_ptr and flags and the
// first half of the ids on one DMA stream, the second half on another (one
// stream alone measured 17-57 GB/s, two 56) — and record ev_done.  It never
// takes the context lock; a slot it holds is not reused before copied_gen
// reaches its launch (the waiter and the cancel path check it).
static void copier_main(egm_ctx* c) {
  hipSetDevice(c->device);
  hipEvent_t join = nullptr;
  hipEventCreateWithFlags(&join, hipEventDisableTiming);
  Dma* dma = pipe_copy_mode() == PIPE_DMA ? dma_open(c->device) : nullptr;   // null: hipMemcpyAsync
  for (;;) {
    std::pair<PipeSlot*, uint64_t> it;
    {
      std::unique_lock<std::mutex> q(c->cq_mu);
      c->cq_cv.wait(q, [&] { return c->cq_stop || !c->cq.empty(); });
      if (c->cq.empty()) break;   // stopping, nothing left
      it = c->cq.front();
      c->cq.erase(c->cq.begin());
    }
    PipeSlot& S = *it.first;
    ptrace("copier-take", &S, it.second);
    hipError_t e = hipEventSynchronize(S.ev_match);   // (a host-synchronised event: device writes released)
    ptrace("match-done", &S, it.second);
    const MatchStats st = *(const MatchStats*)S.h_stats.p;   // copied before ev_match, in stream order
    bool failed = e != hipSuccess;   // the match itself failed: nothing is copied, the waiter reports EGM_E_DEVICE
    if (e == hipSuccess && !st.overflow && !st.guard && dma) {
      const uint64_t n = S.n, nids = std::min<uint64_t>(st.total_ids, S.cap);
      // the ids in two halves (two SDMA queues), then row starts and flags; packed: 3 bytes per id, u32 rows
      const uint64_t ib = nids * (S.packed ? 3 : 4), h1 = std::min<uint64_t>((ib / 2 + 15) & ~15ull, ib);
      const OutLayout ol = out_layout(n, S.cap);
      uint8_t* h = (uint8_t*)S.h_out.p;
      const uint8_t* di = S.packed ? S.d_pk.as<uint8_t>() : S.d_ids.as<uint8_t>();
      const uint64_t rb = (n + 1) * (S.packed ? 4 : 8);
      const DmaPart parts[4] = {{h + ol.o_ids, di, h1},
                                {h + ol.o_ids + h1, di + h1, ib - h1},
                                {h + ol.o_row, S.packed ? S.d_row32.p : S.d_row.p, rb},
                                {h + ol.o_fl, S.d_flags.p, n}};
      failed = !dma_copy_d2h(dma, parts, 4);
    } else if (e == hipSuccess && !st.overflow && !st.guard) {
      const uint64_t n = S.n, nids = std::min<uint64_t>(st.total_ids, S.cap);
      const uint64_t ib = nids * (S.packed ? 3 : 4), h1 = std::min<uint64_t>((ib / 2 + 15) & ~15ull, ib);
      const OutLayout ol = out_layout(n, S.cap);
      uint8_t* h = (uint8_t*)S.h_out.p;
      const uint8_t* di = S.packed ? S.d_pk.as<uint8_t>() : S.d_ids.as<uint8_t>();
      hipMemcpyAsync(h + ol.o_row, S.packed ? S.d_row32.p : S.d_row.p, (n + 1) * (S.packed ? 4 : 8),
                     hipMemcpyDeviceToHost, c->d2h_stream);
      if (n) hipMemcpyAsync(h + ol.o_fl, S.d_flags.p, n, hipMemcpyDeviceToHost, c->d2h_stream);
      if (h1) hipMemcpyAsync(h + ol.o_ids, di, h1, hipMemcpyDeviceToHost, c->d2h_stream);
      if (ib > h1) {
        hipMemcpyAsync(h + ol.o_ids + h1, di + h1, ib - h1, hipMemcpyDeviceToHost, c->d2h_stream2);
        hipEventRecord(join, c->d2h_stream2);
        hipStreamWaitEvent(c->d2h_stream, join, 0);
      }
    }
    // an overflowed or guarded batch copies nothing: the waiter reads the stats
    ptrace("copied", &S, it.second);
    hipEventRecord(S.ev_done, c->d2h_stream);
    {
      std::lock_guard<std::mutex> q(c->cq_mu);
      S.copied_gen = it.second;
      S.copy_failed = failed;
    }
    c->copied_cv.notify_all();
  }
  if (join) hipEventDestroy(join);
  dma_close(dma);
}

// Whether the slot's last launch has its D2H enqueued (ev_done recorded).
static bool slot_copied(egm_ctx* c, PipeSlot& S) {
  std::lock_guard<std::mutex> q(c->cq_mu);
  return S.copied_gen == S.launch_gen;
}

// A free pipeline slot for a batch (index into c->pipe), or -1.  Slots whose
// ticket was cancelled are reclaimed here once their batch has finished.
static PipeSlot* ticket_slot_of(egm_ctx* c, uint64_t ticket);

// Apply the cancels queued while the context was busy (context lock held).
static void drain_cancels(egm_ctx* c) {
  std::vector<uint64_t> q;
  {
    std::lock_guard<std::mutex> g(c->cancel_mu);
    q.swap(c->cancel_q);
  }
  for (uint64_t t : q)
    if (PipeSlot* sp = ticket_slot_of(c, t)) sp->abandoned = true;   // a stale ticket: dropped
  if (!q.empty()) c->pipe_cv.notify_all();
}

static long pipe_free_slot(egm_ctx* c) {
  drain_cancels(c);
  for (size_t k = 0; k < c->pipe.size(); ++k) {
    PipeSlot& S = *c->pipe[k];
    if (S.busy && S.abandoned && !S.waiting && slot_copied(c, S) && hipEventQuery(S.ev_done) == hipSuccess) {
      S.busy = S.abandoned = false;   // a cancelled ticket whose batch is done
    }
    if (!S.busy && !S.held) return (long)k;
  }
  return -1;
}

static int pipe_new_slot(egm_ctx* c, long* k) {
  c->pipe.emplace_back(new PipeSlot());
  PipeSlot& N = *c->pipe.back();
  if (hipEventCreateWithFlags(&N.ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&N.ev_match, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&N.ev_done, hipEventDisableTiming) != hipSuccess) {
    c->pipe.pop_back();
    return c->fail(EGM_E_DEVICE, "pipe events");
  }
  *k = (long)c->pipe.size() - 1;
  return EGM_OK;
}

// Submit with the context lock held once by the caller (g).  A ticket of
// egm_match_submit (sync = false) is refused when PIPE_MAX_SLOTS tickets are
// busy or unreleased; egm_match_batch (sync = true) takes any free slot, adds
// slots up to PIPE_HARD_SLOTS and beyond that waits for one to be freed, so
// concurrent synchronous callers queue instead of failing.
static int submit_locked(egm_ctx* c, std::unique_lock<std::recursive_mutex>& g, const uint8_t* blob,
                         const uint32_t* off, uint32_t n, int mode, bool sync, uint64_t* ticket) {
  if (set_device(c)) return EGM_E_DEVICE;
  hipError_t e;
  if (!c->copy_stream && (e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking)) != hipSuccess)
    return c->hip_fail(e, "copy stream");
  if (!c->d2h_stream && (e = hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking)) != hipSuccess)
    return c->hip_fail(e, "d2h stream");
  if (!c->d2h_stream2 && (e = hipStreamCreateWithFlags(&c->d2h_stream2, hipStreamNonBlocking)) != hipSuccess)
    return c->hip_fail(e, "d2h stream");
  if (!c->copier.joinable()) c->copier = std::thread(copier_main, c);
  if (!sync) {
    size_t tickets = 0;
    for (auto& p : c->pipe)   // a cancelled ticket no longer counts (its slot comes back when its batch is done)
      tickets += (!p->sync && !p->abandoned && (p->busy || p->held)) ? 1u : 0u;
    if (tickets >= PIPE_MAX_SLOTS) return c->fail(EGM_E_STATE, "pipeline full: wait for a ticket or free its result");
  }
  long k = pipe_free_slot(c);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(PIPE_BATCH_WAIT_MS);
  while (k < 0) {
    if (c->pipe.size() < PIPE_HARD_SLOTS) {
      const int r = pipe_new_slot(c, &k);
      if (r) return r;
      break;
    }
    if (!sync) return c->fail(EGM_E_STATE, "pipeline full: wait for a ticket or free its result");
    // every slot busy: wait for a release (polling too, for cancelled tickets)
    if (std::chrono::steady_clock::now() > deadline)
      return c->fail(EGM_E_STATE, "no pipeline slot freed within 30 s (results not released?)");
    c->pipe_cv.wait_for(g, std::chrono::milliseconds(2));
    k = pipe_free_slot(c);
  }
  PipeSlot& S = *c->pipe[(size_t)k];
  // stage the caller's (borrowed) batch in pinned memory, offsets rebased to 0
  const uint32_t base0 = n ? off[0] : 0;
  const uint64_t bytes = n ? (uint64_t)off[n] - base0 : 0;
  const uint64_t o_off = (bytes + 15) & ~15ull, in_sz = o_off + ((uint64_t)n + 1) * 4;
  // the previous use of this slot's staging must be finished (its H2D)
  if ((e = hipEventSynchronize(S.ev_in)) != hipSuccess) return c->hip_fail(e, "pipe input reuse");
  if ((e = S.h_in.ensure(in_sz)) != hipSuccess) return c->hip_fail(e, "pipe pinned input");
  uint8_t* hin = (uint8_t*)S.h_in.p;
  if (bytes) par_copy(hin, blob + base0, bytes);
  uint32_t* hoff = (uint32_t*)(hin + o_off);
  std::atomic<uint64_t> maxlen{0};
  hoff[0] = 0;
  par_for(n, 1u << 18, [&](size_t lo, size_t hi) {   // offsets rebased to 0, and the longest topic
    uint64_t m = 0;
    for (size_t i = lo; i < hi; ++i) {
      hoff[i + 1] = off[i + 1] - base0;
      m = std::max<uint64_t>(m, (uint64_t)off[i + 1] - off[i]);
    }
    uint64_t cur = maxlen.load();
    while (m > cur && !maxlen.compare_exchange_weak(cur, m)) {
    }
  });
  S.n = n;
  S.mode = mode & ~EGM_RESULT_PACKED;
  S.want_packed = (mode & EGM_RESULT_PACKED) != 0;
  S.bytes = bytes;
  S.maxlen = maxlen.load();
  S.cap = std::max<uint64_t>(std::max<uint64_t>((uint64_t)n * 4 + 1024, S.cap),
                             std::max<uint64_t>(c->out_ids.cap / 4, c->pipe_cap_hint));
  // blob and offsets in one copy (the staging already holds them back to back)
  S.o_off = o_off;
  if ((e = S.d_in.ensure(in_sz + 16)) != hipSuccess) return c->hip_fail(e, "pipe input");
  if ((e = hipMemcpyAsync(S.d_in.p, hin, in_sz, hipMemcpyHostToDevice, c->copy_stream)) != hipSuccess ||
      (e = hipEventRecord(S.ev_in, c->copy_stream)) != hipSuccess)
    return c->hip_fail(e, "pipe H2D");
  int r = pipe_launch(c, S);
  if (r) return r;
  S.busy = true;
  S.sync = sync;
  S.abandoned = false;
  S.gen = (S.gen + 1) & 0x7FFFFFFFu;
  if (S.gen == 0) S.gen = 1;
  *ticket = make_ticket((size_t)k, S.gen);
  return EGM_OK;
}

static bool pipe_mode_ok(int mode) {   // EGM_MODE_TRIE / EGM_MODE_ROUTES, optionally | EGM_RESULT_PACKED
  const int m = mode & ~EGM_RESULT_PACKED;
  return m == EGM_MODE_TRIE || m == EGM_MODE_ROUTES;
}

int egm_match_submit(egm_ctx* c, const uint8_t* blob, const uint32_t* off, uint32_t n, int mode, uint64_t* ticket) {
  if (!c || !ticket || !pipe_mode_ok(mode)) return EGM_E_INVAL;
  if (n && (!off || !valid_offsets(off, n) || (!blob && off[n] > off[0]))) return EGM_E_INVAL;
  ptrace("submit-enter", nullptr, n);
  std::unique_lock<std::recursive_mutex> g(c->mu);
  const int r = submit_locked(c, g, blob, off, n, mode, false, ticket);
  ptrace("submit-exit", nullptr, *ticket);
  return r;
}

// The slot of a live ticket (submitted, not yet waited for or cancelled), or null.
static PipeSlot* ticket_slot_of(egm_ctx* c, uint64_t ticket) {
  const size_t k = ticket_slot(ticket);
  if (ticket == 0 || k >= c->pipe.size()) return nullptr;
  PipeSlot& S = *c->pipe[k];
  if (!S.busy || S.waiting || S.abandoned || S.gen != ticket_gen(ticket)) return nullptr;
  return &S;
}

// The device syncs happen without the context lock, so another thread can
// submit (stage + enqueue) the next batch while this one waits.
int egm_match_wait(egm_ctx* c, uint64_t ticket, egm_result** out) {
  if (!c || !out || ticket == 0) return EGM_E_INVAL;
  *out = nullptr;
  std::unique_lock<std::recursive_mutex> g(c->mu);
  drain_cancels(c);
  PipeSlot* sp = ticket_slot_of(c, ticket);
  if (!sp) return c->fail(EGM_E_STATE, "unknown, stale or already waited ticket");
  if (set_device(c)) return EGM_E_DEVICE;
  PipeSlot& S = *sp;
  S.waiting = true;
  auto done = [&](int rc) {   // the slot is free again (its result, if any, held by the caller)
    if (!g.owns_lock()) g.lock();
    S.busy = S.waiting = false;
    c->pipe_cv.notify_all();
    return rc;
  };
  hipError_t e;
  MatchStats st{};
  ptrace("wait-enter", &S, ticket);
  for (int attempt = 0;; ++attempt) {
    g.unlock();
    bool copy_failed = false;
    {   // the copier has copied this launch's result (DMA) or enqueued its D2H (ev_done recorded)
      std::unique_lock<std::mutex> q(c->cq_mu);
      c->copied_cv.wait(q, [&] { return S.copied_gen == S.launch_gen; });
      copy_failed = S.copy_failed;
    }
    e = hipEventSynchronize(S.ev_done);
    g.lock();
    if (e != hipSuccess) return done(c->hip_fail(e, "pipe wait"));
    if (copy_failed) return done(c->fail(EGM_E_DEVICE, "pipe result copy (SDMA) failed"));
    st = *(const MatchStats*)S.h_stats.p;
    if (st.guard) {   // a kernel invariant failed: a bug, never a capacity problem (no retry)
      c->last = st;
      return done(c->fail(EGM_E_DEVICE, "walk guard tripped (bits " + std::to_string(st.guard) +
                                             "): kernel invariant failed, batch not matched"));
    }
    if (!st.overflow) break;
    if (attempt == 2) return done(c->fail(EGM_E_NOMEM, "ids capacity"));
    // the exact total is known even on overflow: rerun the staged batch once with room for it
    S.cap = st.total_ids + st.total_ids / 8 + 1024;
    c->pipe_cap_hint = std::max(c->pipe_cap_hint, S.cap);
    const int r = pipe_launch(c, S);
    if (r) return done(r);
  }
  c->last = st;   // egm_last_stats reports the waited batch
  const uint64_t n = S.n, nids = st.total_ids;
  // the copy-out kernel wrote row_ptr, ids and flags into h_out (ev_done)
  const OutLayout ol = out_layout(n, S.cap);
  uint8_t* h = (uint8_t*)S.h_out.p;
  ResultHdr* hdr = (ResultHdr*)h;
  egm_result* res = (egm_result*)(h + ol.o_res);
  memset(res, 0, sizeof(*res));
  res->n_topics = S.n;
  res->n_ids = nids;
  res->counts = (uint32_t*)(h + ol.o_cnt);
  if (S.packed) {   // row starts as u32, ids as 3 bytes (egm_result_row / egm_result_id)
    res->id_bytes = 3;
    res->row32 = (const uint32_t*)(h + ol.o_row);
    res->ids24 = h + ol.o_ids;
  } else {
    res->id_bytes = 4;
    res->row_ptr = (uint64_t*)(h + ol.o_row);
    res->ids = (uint32_t*)(h + ol.o_ids);
  }
  res->flags = (uint8_t*)(h + ol.o_fl);
  res->epoch = S.epoch;
  res->visited = st.visited;
  res->n_error = st.errors;
  g.unlock();
  // host work outside the lock, on up to 8 threads: counts (not copied over
  // PCIe: row_ptr has them) and the heavy-topic total
  std::atomic<uint32_t> heavy_n{0};
  {
    const uint64_t* rp = res->row_ptr;
    const uint32_t* r32 = res->row32;
    uint32_t* cn = res->counts;
    const uint8_t* fl = res->flags;
    par_for(n, 1u << 17, [&](size_t lo, size_t hi) {
      uint32_t h = 0;
      for (size_t i = lo; i < hi; ++i) {
        cn[i] = r32 ? r32[i + 1] - r32[i] : (uint32_t)(rp[i + 1] - rp[i]);
        h += (fl[i] & TF_HEAVY) ? 1u : 0u;
      }
      heavy_n += h;
    });
  }
  const uint32_t heavy = heavy_n.load();
  g.lock();
  if (egm_result_row(res, (uint32_t)n) != nids) return done(c->fail(EGM_E_DEVICE, "row_ptr total mismatch"));
  res->n_heavy = heavy;
  hdr->magic = RES_PIPE;
  hdr->owner = c;
  hdr->slot = ticket_slot(ticket);
  S.held = true;
  done(EGM_OK);
  ptrace("wait-exit", &S, ticket);
  *out = res;
  if (res->n_error) {
    c->err = "some topics could not be walked (flag EGM_TF_ERROR)";
    return EGM_E_OVERFLOW;
  }
  return EGM_OK;
}

// Give up a ticket without its result: the slot is reclaimed as soon as its
// batch has finished (no wait here).  For a waiter that will never call
// egm_match_wait (e.g. the NIF ticket resource collected unwaited).
int egm_match_cancel(egm_ctx* c, uint64_t ticket) {
  if (!c || ticket == 0) return EGM_E_INVAL;
  std::unique_lock<std::recursive_mutex> g(c->mu, std::try_to_lock);
  if (!g.owns_lock()) {   // busy (a build or commit can hold the context for seconds): queue it
    std::lock_guard<std::mutex> q(c->cancel_mu);
    c->cancel_q.push_back(ticket);
    return EGM_OK;
  }
  drain_cancels(c);
  PipeSlot* sp = ticket_slot_of(c, ticket);
  if (!sp) return c->fail(EGM_E_STATE, "unknown, stale or already waited ticket");
  sp->abandoned = true;
  c->pipe_cv.notify_all();
  return EGM_OK;
}

// One synchronous batch: submit + wait on a pipeline slot of its own.  Host
// buffers are staged in pinned memory and the result is read in place from
// pinned memory (released by egm_result_free).  Concurrent callers never get
// "pipeline full": they take extra slots, then wait for one to be released.
int egm_match_batch(egm_ctx* c, const uint8_t* blob, const uint32_t* off, uint32_t n, int mode,
                    egm_result** out) {
  if (!c || !out || !pipe_mode_ok(mode)) return EGM_E_INVAL;
  *out = nullptr;
  if (n && (!off || !valid_offsets(off, n) || (!blob && off[n] > off[0]))) return EGM_E_INVAL;
  uint64_t t = 0;
  {
    std::unique_lock<std::recursive_mutex> g(c->mu);
    const int r = submit_locked(c, g, blob, off, n, mode, true, &t);
    if (r) return r;
  }
  return egm_match_wait(c, t, out);
}

// egm_result_free for a pipeline result: the slot's pinned memory is free again.
static void pipe_release(egm_ctx* c, uint64_t slot) {
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (slot < c->pipe.size()) c->pipe[slot]->held = false;
  c->pipe_cv.notify_all();
}

// ---------------------------------------------------------------- fan-out --
// The record of filter f with subscribers L whose row (if stored) starts at
// `start` — k_sub_pairs' layout (egm_kernels.hip): x = the third subscriber
// of a row of at most FAN_INLINE_ALL (3), else the row start's low 32 bits;
// y = start bits 32-39 | count (24 bits, saturated) << 8; z, w = the first two.
static uint4 sub_record(const uint32_t* L, uint64_t cnt, uint64_t start) {
  const uint32_t cs = (uint32_t)std::min<uint64_t>(cnt, (1u << 24) - 1);
  const uint32_t x = cnt <= 3 ? (cnt > 2 ? L[2] : 0u) : (uint32_t)start;
  const uint32_t y = (cnt <= 3 ? 0u : ((uint32_t)(start >> 32) & 0xFFu)) | (cs << 8);
  return make_uint4(x, y, cnt > 0 ? L[0] : 0u, cnt > 1 ? L[1] : 0u);
}

// Full build from the host lists (egm_subs_build, and a commit that cannot patch).
static int subs_upload(egm_ctx* c, const uint64_t* row, uint32_t n_slots, const uint32_t* subs) {
  const uint64_t ns = row[n_slots];
  hipError_t e;
  drain_uses(c->subs.uses[0]);
  drain_uses(c->subs.uses[1]);
  if ((e = hipDeviceSynchronize()) != hipSuccess) return c->hip_fail(e, "subs: device sync");
  if ((e = c->sub_row.ensure(((uint64_t)n_slots + 1) * 8)) != hipSuccess) return c->hip_fail(e, "sub_row");
  // room for appended rows: a quarter of the table + 64K entries before the next full build
  if ((e = c->sub_ids.ensure((ns + ns / 4 + 65536) * 4 + 16)) != hipSuccess) return c->hip_fail(e, "sub_ids");
  if ((e = hipMemcpy(c->sub_row.p, row, ((uint64_t)n_slots + 1) * 8, hipMemcpyHostToDevice)) != hipSuccess)
    return c->hip_fail(e, "H2D sub_row");
  if (ns && (e = hipMemcpy(c->sub_ids.p, subs, ns * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return c->hip_fail(e, "H2D subs");
  for (int k = 0; k < 2; ++k)
    if ((e = c->sub_rec(k).ensure(((uint64_t)n_slots + 1) * 16)) != hipSuccess) return c->hip_fail(e, "sub_rp");
  if ((e = launch_sub_pairs(c->sub_row.as<uint64_t>(), c->sub_ids.as<uint32_t>(), n_slots, c->sub_rp.as<uint4>(),
                            c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(c->sub_rp2.p, c->sub_rp.p, (uint64_t)n_slots * 16, hipMemcpyDeviceToDevice, c->stream)) !=
          hipSuccess ||
      (e = hipStreamSynchronize(c->stream)) != hipSuccess)
    return c->hip_fail(e, "sub pairs");
  c->n_fid_slots = n_slots;
  SubsState& S = c->subs;
  S.lists.clear();
  S.recs.clear();
  S.pending.clear();
  S.stale[0].clear();
  S.stale[1].clear();
  S.tail = ns;
  S.garbage = 0;
  S.cur = 0;
  S.built = true;
  S.epoch += 1;
  return EGM_OK;
}

int egm_subs_build(egm_ctx* c, const uint64_t* row, uint32_t n_slots, const uint32_t* subs) {
  if (!c || !row) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  for (uint32_t i = 0; i < n_slots; ++i)
    if (row[i + 1] < row[i]) return EGM_E_INVAL;
  const uint64_t ns = row[n_slots];
  if (ns && !subs) return EGM_E_INVAL;
  if (ns >= (1ull << 40)) return c->fail(EGM_E_INVAL, "subscriber table: at most 2^40 entries (40-bit row starts)");
  return no_throw(c, "subscriber build: host allocation", [&] {
  // the host keeps the lists: the base of later incremental changes (egm_subs_apply_delta)
  SubsState& S = c->subs;
  // record slots beyond the given filter ids (empty rows): new filters subscribed
  // later are patched in, not rebuilt
  const uint32_t cap_slots = (uint32_t)std::min<uint64_t>(WID_MAX, (uint64_t)n_slots + n_slots / 4 + 4096);
  S.row.assign(row, row + (uint64_t)n_slots + 1);
  S.row.resize((uint64_t)cap_slots + 1, row[n_slots]);
  if (subs)
    S.subs.assign(subs, subs + ns);
  else
    S.subs.clear();
  return subs_upload(c, S.row.data(), cap_slots, S.subs.data());
  });
}

// The current subscriber list of filter f (host).
static std::vector<uint32_t>* subs_list(SubsState& S, uint32_t f, bool create) {
  auto it = S.lists.find(f);
  if (it != S.lists.end()) return &it->second;
  if (!create) return nullptr;
  std::vector<uint32_t>& L = S.lists[f];
  if ((uint64_t)f + 1 < S.row.size()) L.assign(S.subs.begin() + S.row[f], S.subs.begin() + S.row[f + 1]);
  return &L;
}

// New filter ids a delta may introduce past the table's current slots.  Filter
// ids are dense (the table builder assigns them in insertion order), so one
// delta never legitimately reaches millions of ids past the table; a larger id
// is a stale or garbage id from the caller, refused before it can size a
// rebuild (one id near WID_MAX asked for a ~34 GB row vector).
static constexpr uint64_t SUBS_FID_GROWTH = 1ull << 22;

static int subs_apply_delta(egm_ctx* c, const egm_sub_pair* add, uint64_t n_add, const egm_sub_pair* del,
                            uint64_t n_del) {
  SubsState& S = c->subs;
  if (!S.built) return c->fail(EGM_E_STATE, "subscriber table: egm_subs_build first");
  const uint64_t fid_limit = std::max<uint64_t>(c->n_fid_slots, S.row.size() - 1) + SUBS_FID_GROWTH;
  for (uint64_t i = 0; i < n_add; ++i)
    if (add[i].fid >= WID_MAX || add[i].fid >= fid_limit)
      return c->fail(EGM_E_INVAL, "subscriber delta: filter id out of range");
  // The two lists are NET effects since the caller's last delta, so a pair
  // may not be in both: adds are applied before removes, and "unsubscribe X,
  // subscribe X" passed as Adds=[X], Dels=[X] would silently drop X.  Refused
  // before anything is applied.
  if (n_add && n_del) {
    std::unordered_set<uint64_t> adds;
    adds.reserve(n_add * 2);
    for (uint64_t i = 0; i < n_add; ++i) adds.insert((uint64_t)add[i].fid << 32 | add[i].sub);
    for (uint64_t i = 0; i < n_del; ++i)
      if (adds.count((uint64_t)del[i].fid << 32 | del[i].sub))
        return c->fail(EGM_E_INVAL, "subscriber delta: a (filter, subscriber) pair is both added and removed");
  }
  // subscribe: a subscriber is in a filter's bag at most once (an ets bag keeps
  // one copy of an identical object, emqx_broker.erl:144-157)
  for (uint64_t i = 0; i < n_add; ++i) {
    std::vector<uint32_t>& L = *subs_list(S, add[i].fid, true);
    if (std::find(L.begin(), L.end(), add[i].sub) == L.end()) L.push_back(add[i].sub);
    S.pending.push_back(add[i].fid);
  }
  // unsubscribe / subscriber_down: removed wherever present, order kept (:178-190, 331-345)
  for (uint64_t i = 0; i < n_del; ++i) {
    if (del[i].fid >= WID_MAX) continue;
    std::vector<uint32_t>* L = subs_list(S, del[i].fid, (uint64_t)del[i].fid + 1 < S.row.size());
    if (!L) continue;
    auto it = std::find(L->begin(), L->end(), del[i].sub);
    if (it != L->end()) {
      L->erase(it);
      S.pending.push_back(del[i].fid);
    }
  }
  return EGM_OK;
}

int egm_subs_apply_delta(egm_ctx* c, const egm_sub_pair* add, uint64_t n_add, const egm_sub_pair* del,
                         uint64_t n_del) {
  if (!c || (n_add && !add) || (n_del && !del)) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  return no_throw(c, "subscriber delta: host allocation", [&] { return subs_apply_delta(c, add, n_add, del, n_del); });
}

static int subs_commit(egm_ctx* c, uint64_t* epoch);

int egm_subs_commit(egm_ctx* c, uint64_t* epoch) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  return no_throw(c, "subscriber commit: host allocation", [&] { return subs_commit(c, epoch); });
}

static int subs_commit(egm_ctx* c, uint64_t* epoch) {
  SubsState& S = c->subs;
  if (!S.built) return c->fail(EGM_E_STATE, "subscriber table: egm_subs_build first");
  S.last_appended = S.last_patched = 0;
  S.last_rebuilt = false;
  std::vector<uint32_t> P = S.pending;
  sort_unique(P);
  // a full build instead of a patch: a new filter id past the table's slots, a
  // row too long for the record's 24-bit count, no room left for appended rows,
  // or more superseded entries than live ones
  bool rebuild = false;
  uint64_t append = 0;
  for (uint32_t f : P) {
    const std::vector<uint32_t>& L = *subs_list(S, f, true);
    if (f >= c->n_fid_slots) rebuild = true;
    if (L.size() >= (1u << 24) - 1) rebuild = true;
    if (L.size() > 3) append += L.size();
  }
  const uint64_t cap_ids = c->sub_ids.cap / 4;
  if (S.tail + append + 16 > cap_ids || S.garbage + append > S.tail / 2 + 65536) rebuild = true;
  if (rebuild) {
    // flatten: the build's lists with every changed list in place (and new
    // empty slots).  Sized from the largest LIVE filter id — a non-empty base
    // row or changed list, or a new id — not from the padded slot count, so
    // repeated rebuilds under churn do not grow the table.
    uint64_t hi = 0;
    for (uint64_t f = S.row.size() - 1; f > 0; --f)
      if (S.row[f] > S.row[f - 1]) {
        hi = f;
        break;
      }
    for (const auto& kv : S.lists)
      if (!kv.second.empty()) hi = std::max<uint64_t>(hi, (uint64_t)kv.first + 1);
    for (uint32_t f : P)
      if (f >= c->n_fid_slots) hi = std::max<uint64_t>(hi, (uint64_t)f + 1);
    const uint32_t n = (uint32_t)std::min<uint64_t>(WID_MAX, hi + hi / 4 + 4096);
    std::vector<uint64_t> row((uint64_t)n + 1, 0);
    for (uint32_t f = 0; f < n; ++f) {
      auto it = S.lists.find(f);
      const uint64_t k = it != S.lists.end() ? it->second.size()
                         : ((uint64_t)f + 1 < S.row.size() ? S.row[f + 1] - S.row[f] : 0);
      row[f + 1] = row[f] + k;
    }
    std::vector<uint32_t> flat(row[n]);
    for (uint32_t f = 0; f < n; ++f) {
      auto it = S.lists.find(f);
      if (it != S.lists.end())
        std::copy(it->second.begin(), it->second.end(), flat.begin() + row[f]);
      else if ((uint64_t)f + 1 < S.row.size())
        std::copy(S.subs.begin() + S.row[f], S.subs.begin() + S.row[f + 1], flat.begin() + row[f]);
    }
    if (row[n] >= (1ull << 40)) return c->fail(EGM_E_INVAL, "subscriber table: at most 2^40 entries");
    S.row.swap(row);
    S.subs.swap(flat);
    const int r = subs_upload(c, S.row.data(), n, S.subs.data());
    if (r == EGM_OK) S.last_rebuilt = true;
    if (epoch) *epoch = S.epoch;
    return r;
  }
  // appended rows and the new records of the changed filters
  std::vector<uint32_t> app;
  app.reserve(append);
  const uint64_t base = S.tail;
  for (uint32_t f : P) {
    const std::vector<uint32_t>& L = *subs_list(S, f, true);
    const uint64_t start = L.size() > 3 ? base + app.size() : 0;
    if (L.size() > 3) app.insert(app.end(), L.begin(), L.end());
    auto old = S.recs.find(f);
    const uint64_t old_cnt = old != S.recs.end() ? (old->second.y >> 8)
                             : ((uint64_t)f + 1 < S.row.size() ? S.row[f + 1] - S.row[f] : 0);
    if (old_cnt > 3) S.garbage += old_cnt;
    S.recs[f] = sub_record(L.data(), L.size(), start);
  }
  // the copy no reader uses: its last readers first, then every record it lacks
  const int x = 1 - S.cur;
  drain_uses(S.uses[x]);
  std::vector<uint32_t> need = S.stale[x];
  need.insert(need.end(), P.begin(), P.end());
  sort_unique(need);
  hipError_t e;
  const size_t o_app = 0, o_idx = (app.size() * 4 + 15) & ~(size_t)15, o_rec = (o_idx + need.size() * 4 + 15) & ~(size_t)15;
  const size_t total = o_rec + need.size() * 16;
  if (total) {
    uint8_t* h = patch_stage(c, total);
    if (!h) return c->fail(EGM_E_NOMEM, "subs commit: pinned staging");
    memcpy(h + o_app, app.data(), app.size() * 4);
    memcpy(h + o_idx, need.data(), need.size() * 4);
    for (size_t i = 0; i < need.size(); ++i) memcpy(h + o_rec + 16 * i, &S.recs[need[i]], 16);
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "subs commit: stream");
    if ((e = c->patch_dev.ensure(total)) != hipSuccess) return c->hip_fail(e, "subs commit: patch buffer");
    if ((e = hipMemcpyAsync(c->patch_dev.p, h, total, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      return c->hip_fail(e, "subs commit: upload");
    uint8_t* dp = (uint8_t*)c->patch_dev.p;
    // appended rows lie past every entry a reader of either copy can reach
    if (!app.empty() &&
        (e = hipMemcpyAsync(c->sub_ids.as<uint32_t>() + base, dp + o_app, app.size() * 4, hipMemcpyDeviceToDevice,
                            c->stream)) != hipSuccess)
      return c->hip_fail(e, "subs commit: rows");
    if ((e = launch_patch(c->sub_rec(x).p, 16, (const uint32_t*)(dp + o_idx), dp + o_rec, need.size(), c->stream)) !=
        hipSuccess)
      return c->hip_fail(e, "subs commit: patch");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return c->hip_fail(e, "subs commit: sync");
  }
  S.tail = base + app.size();
  S.stale[x].clear();
  S.stale[S.cur].insert(S.stale[S.cur].end(), P.begin(), P.end());   // the old copy now lacks this commit
  S.cur = x;
  S.pending.clear();
  S.epoch += 1;
  S.last_appended = app.size();
  S.last_patched = need.size();
  if (epoch) *epoch = S.epoch;
  return EGM_OK;
}

int egm_subs_slots(egm_ctx* c, uint32_t* n_fid_slots) {
  if (!c || !n_fid_slots) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  *n_fid_slots = c->n_fid_slots;
  return EGM_OK;
}

int egm_subs_last_commit(egm_ctx* c, uint64_t* appended, uint64_t* patched, int* rebuilt, uint64_t* entries) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (appended) *appended = c->subs.last_appended;
  if (patched) *patched = c->subs.last_patched;
  if (rebuilt) *rebuilt = c->subs.last_rebuilt ? 1 : 0;
  if (entries) *entries = c->subs.tail;
  return EGM_OK;
}

static int run_fanout(egm_ctx* c, const uint64_t* d_mrow, const uint32_t* d_mids, uint64_t mids_len, uint32_t n,
                      hipStream_t s,
                      uint64_t* d_drow, uint32_t* d_fid, uint32_t* d_sub, uint64_t cap, uint64_t* total,
                      uint64_t* d_entry_pos = nullptr) {
  uint64_t nids = 0;
  hipError_t e = hipMemcpyAsync(&nids, d_mrow + n, 8, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return c->hip_fail(e, "match_row readback");
  if (nids >= 0xFFFFFFF0ull) return c->fail(EGM_E_INVAL, "too many matched ids for one fan-out batch");
  if (nids > mids_len) return c->fail(EGM_E_OVERFLOW, "match row total exceeds the id buffer (overflowed match batch)");
  const uint64_t nwin = (nids + 63) / 64;
  if ((e = c->f_dc.ensure((nwin + 1) * 4)) != hipSuccess) return c->hip_fail(e, "f_dc");   // window totals
  const bool ord = c->last_walk.order && c->last_walk.row == d_mrow && c->last_walk.n == n;
  if (fan_uses_ds0(ord) && (e = c->f_ds0.ensure((nids + 1) * 16)) != hipSuccess)
    return c->hip_fail(e, "f_ds0");   // entry records (the two-pass form)
  if ((e = c->f_wbase.ensure((nwin + 2) * 8)) != hipSuccess) return c->hip_fail(e, "f_wbase");
  if (!d_entry_pos && (e = c->f_dpos.ensure((nids + 2) * 8)) != hipSuccess) return c->hip_fail(e, "f_dpos");
  uint64_t* dpos = d_entry_pos ? d_entry_pos : c->f_dpos.as<uint64_t>();   // the caller's, in the compact form
  if ((e = c->f_tiles.ensure((scan_tiles((uint32_t)nwin) + 2) * 8)) != hipSuccess) return c->hip_fail(e, "f_tiles");
  if ((e = c->f_ovf.ensure(16)) != hipSuccess) return c->hip_fail(e, "f_ovf");
  const int rk = c->subs.cur;   // the current record copy; a commit patches the other one
  SubTable st{c->sub_row.as<uint64_t>(), c->sub_ids.as<uint32_t>(), c->n_fid_slots, c->sub_rec(rk).as<uint4>()};
  hipEvent_t evp[2] = {nullptr, nullptr};
  if (c->timing) {
    evp[0] = c->take_event();
    evp[1] = c->take_event();
  }
  c->work_begin(s);
  // these rows are the last match's: count in its walk order (the workspace
  // holding it is then protected until this fan-out has read it)
  MatchWs* OW = ord ? &c->ws[c->last_walk.ws] : nullptr;
  if (OW && OW->used && OW->stream != s && OW->ev) hipStreamWaitEvent(s, OW->ev, 0);   // (stream 0 is a stream too)
  e = launch_fanout(st, d_mrow, d_mids, n, nids, d_drow, d_fid, d_sub, cap, c->f_dc.as<uint32_t>(),
                    c->f_ds0.as<uint4>(), dpos, c->f_wbase.as<uint64_t>(), c->f_tiles.as<uint64_t>(),
                    c->f_ovf.as<unsigned int>(), s, c->timing ? evp : nullptr, ord ? c->last_walk.order : nullptr);
  if (OW) ws_done(*OW, s);
  {   // a later subscriber commit must not patch this copy before the fan-out has read it
    auto& u = c->subs.uses[rk];
    bool found = false;
    for (auto& p : u)
      if (p.first == s) {
        hipEventRecord(p.second, s);
        found = true;
      }
    hipEvent_t ev = nullptr;
    if (!found && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
      hipEventRecord(ev, s);
      u.push_back({s, ev});
    }
  }
  if (c->timing) {
    c->ev_fan.push_back(evp[0]);
    c->ev_fan.push_back(evp[1]);
  }
  c->work_end(s);
  c->fan_drow = d_drow;
  c->fan_topics = n;
  c->fan_stream = s;
  if (e != hipSuccess) return c->hip_fail(e, "launch_fanout");
  if (total) {
    unsigned int ovf = 0;
    if ((e = hipMemcpyAsync(total, d_drow + n, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(&ovf, c->f_ovf.p, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
      return c->hip_fail(e, "fanout readback");
    if (ovf) return EGM_E_OVERFLOW;
  }
  return EGM_OK;
}

int egm_fanout_device(egm_ctx* c, const uint64_t* d_mrow, const uint32_t* d_mids, uint64_t mids_len, uint32_t n,
                      void* hip_stream,
                      uint64_t* d_drow, uint32_t* d_fid, uint32_t* d_sub, uint64_t cap) {
  if (!c || !d_mrow || !d_drow) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  return run_fanout(c, d_mrow, d_mids, mids_len, n, s, d_drow, d_fid, d_sub, cap, nullptr);
}

int egm_fanout_device_compact(egm_ctx* c, const uint64_t* d_mrow, const uint32_t* d_mids, uint64_t mids_len,
                              uint32_t n, void* hip_stream, uint64_t* d_drow, uint64_t* d_entry_pos, uint32_t* d_sub,
                              uint64_t cap) {
  if (!c || !d_mrow || !d_drow || !d_entry_pos) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  return run_fanout(c, d_mrow, d_mids, mids_len, n, s, d_drow, nullptr, d_sub, cap, nullptr, d_entry_pos);
}

int egm_fanout_batch(egm_ctx* c, const egm_result* m, egm_delivery** out) {
  if (!c || !m || !out) return EGM_E_INVAL;
  *out = nullptr;
  if (!m->row_ptr || (m->n_ids && !m->ids))   // a packed result (EGM_RESULT_PACKED) is not taken here
    return c->fail(EGM_E_INVAL, "egm_fanout_batch takes the plain result form (match without EGM_RESULT_PACKED)");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = c->stream;
  const uint32_t n = m->n_topics;
  const uint64_t nids = m->row_ptr[n];
  hipError_t e;
  if ((e = c->f_mrow.ensure(((uint64_t)n + 1) * 8)) != hipSuccess) return c->hip_fail(e, "f_mrow");
  if ((e = c->f_mids.ensure(nids * 4 + 16)) != hipSuccess) return c->hip_fail(e, "f_mids");
  if ((e = hipMemcpyAsync(c->f_mrow.p, m->row_ptr, ((uint64_t)n + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess)
    return c->hip_fail(e, "H2D match rows");
  if (nids && (e = hipMemcpyAsync(c->f_mids.p, m->ids, nids * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
    return c->hip_fail(e, "H2D match ids");
  uint64_t cap = nids * 2 + 1024, total = 0;
  if ((e = c->f_drow.ensure(((uint64_t)n + 1) * 8)) != hipSuccess) return c->hip_fail(e, "f_drow");
  for (int attempt = 0; attempt < 2; ++attempt) {
    if ((e = c->f_dfid.ensure(cap * 4)) != hipSuccess) return c->hip_fail(e, "f_dfid");
    if ((e = c->f_dsub.ensure(cap * 4)) != hipSuccess) return c->hip_fail(e, "f_dsub");
    int r = run_fanout(c, c->f_mrow.as<uint64_t>(), c->f_mids.as<uint32_t>(), nids, n, s, c->f_drow.as<uint64_t>(),
                       c->f_dfid.as<uint32_t>(), c->f_dsub.as<uint32_t>(), cap, &total);
    if (r == EGM_OK) break;
    if (r != EGM_E_OVERFLOW || attempt == 1) return r;
    cap = total + 1024;
  }
  size_t sz = sizeof(egm_delivery);
  size_t o_row = sz;
  sz += ((uint64_t)n + 1) * 8;
  size_t o_fid = sz;
  sz += (total * 4 + 7) & ~7ull;
  size_t o_sub = sz;
  sz += (total * 4 + 7) & ~7ull;
  uint8_t* mem = (uint8_t*)result_alloc(sz);
  if (!mem) return c->fail(EGM_E_NOMEM, "delivery");
  egm_delivery* d = (egm_delivery*)mem;
  d->n_topics = n;
  d->n_deliveries = total;
  d->row_ptr = (uint64_t*)(mem + o_row);
  d->fid = (uint32_t*)(mem + o_fid);
  d->sub = (uint32_t*)(mem + o_sub);
  if ((e = hipMemcpy(d->row_ptr, c->f_drow.p, ((uint64_t)n + 1) * 8, hipMemcpyDeviceToHost)) != hipSuccess ||
      (total && (e = hipMemcpy(d->fid, c->f_dfid.p, total * 4, hipMemcpyDeviceToHost)) != hipSuccess) ||
      (total && (e = hipMemcpy(d->sub, c->f_dsub.p, total * 4, hipMemcpyDeviceToHost)) != hipSuccess)) {
    result_discard(mem);
    return c->hip_fail(e, "D2H deliveries");
  }
  *out = d;
  return EGM_OK;
}

// ------------------------------------------------------------ shard merge --
int egm_debug_walk_sort(egm_ctx* c, const uint32_t* d_keys, const uint64_t* d_vals, uint32_t n, uint32_t kbits,
                        uint64_t* d_out) {
  if (!c || !d_keys || !d_vals || !d_out || !n || n >= (1u << 29) || !kbits || kbits > 32) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  DevBuf k1, k2, v1, tmp, st;
  // a shape whose levels sum to kbits (the scratch size depends only on the bits)
  const uint32_t shape = kbits <= 15 ? kbits : (kbits <= 30 ? (15u | ((kbits - 15) << 4)) : (15u | (15u << 4) | ((kbits - 30) << 8)));
  hipError_t e;
  if ((e = k1.ensure((size_t)n * 4)) != hipSuccess || (e = k2.ensure((size_t)n * 4)) != hipSuccess ||
      (e = v1.ensure((size_t)n * 8)) != hipSuccess || (e = tmp.ensure(walk_sort_temp_bytes(n, shape))) != hipSuccess ||
      (e = st.ensure(sizeof(MatchStats))) != hipSuccess)
    return c->hip_fail(e, "debug sort: scratch");
  if ((e = hipMemcpyAsync(k1.p, d_keys, (size_t)n * 4, hipMemcpyDeviceToDevice, c->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(v1.p, d_vals, (size_t)n * 8, hipMemcpyDeviceToDevice, c->stream)) != hipSuccess ||
      (e = hipMemsetAsync(st.p, 0, sizeof(MatchStats), c->stream)) != hipSuccess ||
      (e = launch_walk_sort(k1.as<uint32_t>(), k2.as<uint32_t>(), v1.as<uint64_t>(), d_out, tmp.p, st.as<MatchStats>(),
                            n, kbits, c->stream)) != hipSuccess)
    return c->hip_fail(e, "debug sort: launch");
  MatchStats hs{};
  if ((e = hipMemcpyAsync(&hs, st.p, sizeof hs, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(c->stream)) != hipSuccess)
    return c->hip_fail(e, "debug sort: sync");
  if (hs.guard) return c->fail(EGM_E_DEVICE, "debug sort: look-back guard tripped");
  return EGM_OK;
}

int egm_shard_merge(egm_ctx* c, uint32_t n_shards, uint32_t n, const uint32_t* d_counts,
                    const uint32_t* const* d_shard_ids, uint64_t total_ids, void* hip_stream, uint64_t* d_row,
                    uint32_t* d_ids, uint64_t ids_cap) {
  if (!c || n_shards == 0 || n_shards > MAX_SHARDS || !d_counts || !d_shard_ids || !d_row) return EGM_E_INVAL;
  if (total_ids > ids_cap || (total_ids && !d_ids)) return EGM_E_OVERFLOW;
  for (uint32_t g = 0; g < n_shards; ++g)
    if (!d_shard_ids[g] && total_ids) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  hipError_t e;
  const uint64_t nn = (uint64_t)n + 1;
  if ((e = c->m_srow.ensure(nn * n_shards * 8)) != hipSuccess) return c->hip_fail(e, "merge srow");
  if ((e = c->m_tiles.ensure((scan_tiles(n) + 2) * 8)) != hipSuccess) return c->hip_fail(e, "merge tiles");
  if ((e = c->m_tot.ensure(nn * 4)) != hipSuccess) return c->hip_fail(e, "merge tot");
  ShardIds src{};
  for (uint32_t k = 0; k < n_shards; ++k) src.ids[k] = d_shard_ids[k];
  c->work_begin(s);
  e = launch_shard_merge(d_counts, n_shards, n, src, c->m_srow.as<uint64_t>(),
                         c->m_tiles.as<uint64_t>(), c->m_tot.as<uint32_t>(), d_row, d_ids, ids_cap, s);
  c->work_end(s);
  if (e != hipSuccess) return c->hip_fail(e, "launch_shard_merge");
  return EGM_OK;
}

int egm_last_fanout(egm_ctx* c, uint64_t* n_deliveries, uint32_t* overflow) {
  if (!c) return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (!c->fan_drow) return c->fail(EGM_E_STATE, "no fan-out launched");
  if (set_device(c)) return EGM_E_DEVICE;
  uint64_t tot = 0;
  unsigned int ovf = 0;
  hipError_t e;
  if ((e = hipStreamSynchronize(c->fan_stream)) != hipSuccess ||
      (e = hipMemcpy(&tot, c->fan_drow + c->fan_topics, 8, hipMemcpyDeviceToHost)) != hipSuccess ||
      (e = hipMemcpy(&ovf, c->f_ovf.p, 4, hipMemcpyDeviceToHost)) != hipSuccess)
    return c->hip_fail(e, "fan-out readback");
  if (n_deliveries) *n_deliveries = tot;
  if (overflow) *overflow = ovf;
  return EGM_OK;
}

void egm_result_free(void* r) {
  if (!r) return;
  ResultHdr* h = (ResultHdr*)r - 1;
  if (h->magic == RES_PIPE) pipe_release((egm_ctx*)h->owner, h->slot);
  else result_discard(r);
}

// ---------------------------------------------------- host-only image API --
struct egm_image {
  HostTable t;
  DirtyLog d;   // the log egm_image_take_dirty last handed out
};

egm_image* egm_image_new(void) { return new (std::nothrow) egm_image(); }
void egm_image_free(egm_image* im) { delete im; }
int egm_image_insert(egm_image* im, const uint8_t* f, uint32_t len, uint32_t id) {
  if (!im || (!f && len)) return EGM_E_INVAL;
  return im->t.insert(f, len, id, nullptr);
}
int egm_image_remove(egm_image* im, const uint8_t* f, uint32_t len) {
  if (!im || (!f && len)) return EGM_E_INVAL;
  return im->t.remove(f, len);
}
void egm_image_relayout(egm_image* im) {
  if (im) im->t.relayout();
}
int egm_image_build(egm_image* im, const uint8_t* blob, const uint32_t* off, uint32_t n, const uint32_t* ids,
                    uint32_t threads) {
  if (!im || (n && (!blob || !valid_offsets(off, n)))) return EGM_E_INVAL;
  std::string why;
  if (!validate_inserts(im->t, blob, off, n, ids, true, &why)) return EGM_E_INVAL;
  if (ids)
    for (uint32_t i = 0; i < n; ++i)
      if (ids[i] == NONE) return EGM_E_INVAL;
  return im->t.bulk_build(blob, off, n, ids, threads) < 0 ? EGM_E_INVAL : EGM_OK;
}
int egm_image_take_dirty(egm_image* im, egm_dirty_view* v) {
  if (!im || !v) return EGM_E_INVAL;
  im->d = im->t.take_dirty();
  sort_unique(im->d.nodes, im->t.nodes.size());
  sort_unique(im->d.edges, im->t.edges.size());
  sort_unique(im->d.dict, im->t.dict.size());
  v->nodes = im->d.nodes.data();
  v->n_nodes = im->d.nodes.size();
  v->edges = im->d.edges.data();
  v->n_edges = im->d.edges.size();
  v->dict = im->d.dict.data();
  v->n_dict = im->d.dict.size();
  v->nodes_full = im->d.nodes_full;
  v->edges_full = im->d.edges_full;
  v->dict_full = im->d.dict_full;
  v->words_full = im->d.words_full;
  return EGM_OK;
}
int egm_image_get_view(egm_image* im, egm_image_view* v) {
  if (!im || !v) return EGM_E_INVAL;
  const HostTable& t = im->t;
  v->nodes = t.nodes.data();
  v->n_nodes = t.nodes.size();
  v->hash_child = t.hash_child.data();
  v->edges = t.edges.data();
  v->n_edge_slots = t.edges.size();
  v->edge_mask = t.edge_mask();
  v->dict = t.dict.data();
  v->n_dict_slots = t.dict.size();
  v->dict_mask = t.dict_mask();
  v->dict_blob = t.dict_blob.data();
  v->dict_off = t.dict_off.data();
  v->n_words = t.n_words();
  v->n_filters = t.n_filters();
  v->n_live_nodes = t.n_nodes_live();
  v->n_edges = t.n_edges();
  return EGM_OK;
}
int egm_shard_assign(const uint8_t* blob, const uint32_t* off, uint32_t n, uint32_t g, uint32_t* out) {
  if (!off || !out || g == 0 || (n && !blob)) return EGM_E_INVAL;
  for (uint32_t i = 0; i < n; ++i) out[i] = filter_shard(blob + off[i], off[i + 1] - off[i], g);
  return EGM_OK;
}
// ---- prefix partition ----
int egm_prefix_assign(const uint8_t* blob, const uint32_t* off, uint32_t n, uint32_t n_vparts, uint32_t n_ranks,
                      uint8_t* vpart_rank, uint32_t* filter_rank) {
  if (!off || !vpart_rank || !filter_rank || n_vparts == 0 || n_ranks == 0 || n_ranks > PREFIX_RANKS_MAX ||
      (n && !blob))
    return EGM_E_INVAL;
  std::vector<uint64_t> load(n_vparts, 0);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* p = blob + off[i];
    const uint32_t len = off[i + 1] - off[i];
    if (prefix_replicated(p, len)) {
      filter_rank[i] = EGM_PREFIX_ALL;
    } else {
      const uint32_t v = prefix_vpart(p, len, n_vparts);
      filter_rank[i] = v;   // the vpart for now, its rank below
      load[v] += 1;
    }
  }
  // greedy: the heaviest virtual partitions first, each to the least loaded
  // rank (ties: the lower vpart, the lower rank) — deterministic on every rank
  std::vector<uint32_t> order(n_vparts);
  for (uint32_t v = 0; v < n_vparts; ++v) order[v] = v;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return load[a] > load[b]; });
  std::vector<uint64_t> rl(n_ranks, 0);
  for (uint32_t v : order) {
    uint32_t best = 0;
    for (uint32_t k = 1; k < n_ranks; ++k)
      if (rl[k] < rl[best]) best = k;
    vpart_rank[v] = (uint8_t)best;
    rl[best] += load[v];
  }
  for (uint32_t i = 0; i < n; ++i)
    if (filter_rank[i] != EGM_PREFIX_ALL) filter_rank[i] = vpart_rank[filter_rank[i]];
  return EGM_OK;
}

uint64_t egm_prefix_slot_bytes(uint32_t n_ranks, uint32_t cap_topics, uint64_t cap_bytes) {
  const PrefixSlots ps{n_ranks, cap_topics, cap_bytes};
  return ps.slot_bytes();
}

int egm_prefix_route(egm_ctx* c, const uint8_t* d_blob, const uint32_t* d_off, uint32_t n, const uint8_t* d_vpart_rank,
                     uint32_t n_vparts, uint32_t n_ranks, uint32_t cap_topics, uint64_t cap_bytes, void* hip_stream,
                     uint8_t* d_send) {
  if (!c || !d_vpart_rank || !d_send || n_vparts == 0 || n_ranks == 0 || n_ranks > PREFIX_RANKS_MAX ||
      (n && (!d_blob || !d_off)) || cap_bytes >= (1ull << 32) || n >= PFX_TOPICS_MAX || cap_topics >= PFX_TOPICS_MAX)
    return EGM_E_INVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (set_device(c)) return EGM_E_DEVICE;
  hipStream_t s = (hipStream_t)hip_stream;   // NULL: the HIP default (null) stream, as the caller's own work
  hipError_t e;
  if ((e = c->p_ctr.ensure(2 * 8 * PREFIX_RANKS_MAX)) != hipSuccess) return c->hip_fail(e, "prefix counters");
  if ((e = c->p_dst.ensure(8ull * std::max<uint32_t>(n, 1))) != hipSuccess) return c->hip_fail(e, "prefix routes");
  c->work_begin(s);
  const PrefixSlots ps{n_ranks, cap_topics, cap_bytes};
  e = launch_prefix_route(d_blob, d_off, n, d_vpart_rank, n_vparts, ps, d_send, c->p_ctr.as<unsigned long long>(),
                          c->p_dst.as<uint64_t>(), s);
  c->work_end(s);
  return e == hipSuccess ? EGM_OK : c->hip_fail(e, "launch_prefix_route");
}

uint64_t egm_word_hash(const uint8_t* p, uint32_t len) { return word_hash(p, len); }
uint32_t egm_edge_bucket(uint32_t parent, uint32_t w, uint32_t mask) { return edge_bucket(parent, w, mask); }

}  // extern "C"
