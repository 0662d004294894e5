// egm_kernels.hip — gfx950 kernels for publish-time route lookup.
//
// Replaces, per batch of publish topics:
//   emqx_topic:words/1            apps/emqx/src/emqx_topic.erl:153-164   -> k_tokenise
//   emqx_trie:match/1 (+ do_match, match_compact, 'match_#', lookup_topic,
//   has_prefix)                   apps/emqx/src/emqx_trie.erl:100-114,190-270 -> k_walk / k_heavy
//   emqx_router:match_routes/1    apps/emqx/src/emqx_router.erl:129-141  -> mode EGM_MODE_ROUTES
//   emqx_broker:dispatch/2        apps/emqx/src/emqx_broker.erl:283-324  -> k_fanout_*
//
// The walk is an NFA frontier expansion over the word-level trie (egm_common.h):
// topics sorted into a locality order (a key from k_tokenise + a radix sort), then one
// wavefront per chunk of 64 of them, walking from an LDS work stack (pop up to
// 64 items, issue their reads together, compact children and emits back with
// __ballot / mbcnt), staging emits per topic and flushing them as pieces;
// k_compact assembles the CSR rows from the pieces.  Chunks with a topic
// deeper than the LDS stack allows are walked by k_heavy (one topic per wave,
// stack in HBM).
//
// This is pointer chasing over hashed edges — HBM / latency bound; no MFMA.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "egm_kernels.h"

namespace egm {

constexpr int MODE_TRIE = 0;
constexpr int MODE_ROUTES = 1;

constexpr int TOK_BLOCK = 256;
#ifndef EGM_TOK_LDS
#define EGM_TOK_LDS 16256   // staged topic bytes per tokenise block (A/B at C2: 24 KB -> 1.09 ms, 16 KB -> 0.92, 12 KB -> 1.12;
                            // 16 KB - 128 B keeps 4 blocks per CU beside the walk-order key table)
#endif
constexpr int TOK_LDS = EGM_TOK_LDS;
#ifndef EGM_TOK_WORDS
#define EGM_TOK_WORDS 2528   // words per tokenise block (5 B of LDS each): 32 000 B per block, 25 of LDS's 1 280-B
                             // allocation granules, so 5 blocks fit per CU (2 560 words took 26 granules: 4 blocks,
                             // as with round 5's 7 B per word) — C2 0.882 -> 0.773 ms, C3 2.57 -> 2.27 (r6av);
                             // 2048 made C3's segments of 128 depth-16 topics retry as two of 64
#endif
constexpr int TOK_WORDS = EGM_TOK_WORDS;
#ifndef EGM_TOK_U
#define EGM_TOK_U 2          // words per lane whose dictionary probes are in flight together
#endif
constexpr int TOK_U = EGM_TOK_U;
constexpr int SCAN_TILE = 2048;      // counts per scan tile (256 threads x 8)


// ------------------------------------------------------------ primitives ----
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t popc(uint64_t m) { return (uint32_t)__popcll(m); }

// Make one lane's LDS writes visible to the other lanes of the same wave.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t* total) {
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

__device__ __forceinline__ uint4 ld16(const void* p) { return *(const uint4*)p; }

// ------------------------------------------------------------ dictionary ----
__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t k) {
  uint32_t w = (k < 8) ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
  return (w >> (8 * (k & 3))) & 0xFFu;
}

// Byte-exact dictionary probe (linear probing over 32 B slots).
__device__ uint32_t dict_probe(const DevTable& tab, uint64_t h, const uint8_t* p, uint32_t len) {
  uint32_t i = (uint32_t)h & tab.dict_mask;
  for (;;) {
    const uint8_t* sp = (const uint8_t*)(tab.dict + i);
    const uint4 a = ld16(sp);       // {hash lo, hash hi, wid, len}
    const uint4 b = ld16(sp + 16);  // inline bytes: same 32 B slot, same round trip
    if (a.z == NONE) return WID_NONE;
    if (a.x == (uint32_t)h && a.y == (uint32_t)(h >> 32) && a.w == len) {
      bool eq = true;
      if (len <= 16) {
        for (uint32_t k = 0; k < len; ++k) eq &= byte_of(b, k) == p[k];
      } else {
        const uint8_t* q = tab.dict_blob + tab.dict_off[a.z];
        for (uint32_t k = 0; k < len; ++k) eq &= q[k] == p[k];
      }
      if (eq) return a.z;
    }
    i = (i + 1) & tab.dict_mask;
  }
}

// -------------------------------------------------------------- tokenise ----
// emqx_topic:words/1 (emqx_topic.erl:153-164) + wildcard/1 (:53-62) for a
// batch: one lane per topic.  The block's bytes are staged in LDS with
// coalesced 4-byte loads and scanned 4 bytes per LDS read; FNV-1a per word,
// then the byte-exact dictionary probe.
// Output: level count, TF_* flags and one word id per level at wid[off[t]+t+l].
// The topic's bytes start at byte `mis` of the aligned word array `wp`.
__device__ __forceinline__ void tokenise_one(const DevTable& tab, const uint32_t* wp, uint32_t mis, uint32_t len,
                                             uint32_t base, uint32_t* __restrict__ wid, uint32_t* lv_out,
                                             uint8_t* fl_out) {
  const uint8_t* p = (const uint8_t*)wp + mis;
  uint32_t l = 0, ws = 0;
  uint8_t fl = 0;
  for (uint32_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    const uint32_t wl = i - ws;
    uint32_t w;
    if (wl == 1 && p[ws] == '+') {
      w = WID_PLUS;
      fl |= TF_WILDCARD;
    } else if (wl == 1 && p[ws] == '#') {
      w = WID_HASH;
      fl |= TF_WILDCARD;
    } else {
      w = dict_probe(tab, word_hash(p + ws, wl), p + ws, wl);
    }
    wid[base + l] = w;
    ++l;
    ws = i + 1;
  }
  if (len > 0 && p[0] == '$') fl |= TF_DOLLAR;
  *lv_out = l;
  *fl_out = fl;
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* sw, uint32_t i) {
  return (sw[i >> 2] >> (8 * (i & 3u))) & 0xFFu;
}

// The 4 bytes at LDS byte offset i (any alignment; reads up to one word past).
__device__ __forceinline__ uint32_t lds_word(const uint32_t* sw, uint32_t i) {
  const uint32_t lo = sw[i >> 2], hi = sw[(i >> 2) + 1];
  return __builtin_amdgcn_alignbyte(hi, lo, i & 3u);
}

// Low n bytes of a word (n <= 4).
__device__ __forceinline__ uint32_t low_bytes(uint32_t v, uint32_t n) {
  return n >= 4 ? v : (v & ((1u << (8 * n)) - 1u));
}

// word_hash (egm_common.h) of the wl bytes at LDS offset st.
__device__ __forceinline__ uint64_t lds_word_hash(const uint32_t* sw, uint32_t st, uint32_t wl) {
  uint64_t h = FNV_BASIS;
  for (uint32_t k = 0; k < wl; k += 4) h = hash_chunk(h, low_bytes(lds_word(sw, st + k), wl - k));
  return word_hash_finish(h, wl);
}

// Mask (bit 7 of each byte) of the bytes of v equal to '/'.
__device__ __forceinline__ uint32_t slash_mask(uint32_t v) {
  const uint32_t x = v ^ 0x2F2F2F2Fu;
  return (x - 0x01010101u) & ~x & 0x80808080u;
}

// Keep the bytes [lo, hi) of a 4-byte word (0 <= lo <= hi <= 4) in a byte mask.
__device__ __forceinline__ uint32_t byte_range(uint32_t lo, uint32_t hi) {
  const uint32_t a = lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo));
  const uint32_t b = hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u);
  return a & b;
}

// Resolve a dictionary probe whose first slot {a, b} is already loaded; the
// candidate's bytes are in LDS at st.  Continues with the next slots (rare).
__device__ __forceinline__ uint32_t dict_resolve(const DevTable& tab, uint64_t h, uint4 a, uint4 b,
                                                 const uint32_t* sw, uint32_t st, uint32_t len) {
  uint32_t i = (uint32_t)h & tab.dict_mask;
  for (;;) {
    if (a.z == NONE) return WID_NONE;
    if (a.x == (uint32_t)h && a.y == (uint32_t)(h >> 32) && a.w == len) {
      bool eq = true;
      if (len <= 16) {
        const uint32_t bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (uint32_t k = 0; k < 16; k += 4)
          if (k < len) eq &= low_bytes(lds_word(sw, st + k), len - k) == low_bytes(bw[k >> 2], len - k);
      } else {
        const uint8_t* q = tab.dict_blob + tab.dict_off[a.z];
        for (uint32_t k = 0; k < len; ++k) eq &= q[k] == lds_byte(sw, st + k);
      }
      if (eq) return a.z;
    }
    i = (i + 1) & tab.dict_mask;
    const uint8_t* sp = (const uint8_t*)(tab.dict + i);
    a = ld16(sp);
    b = ld16(sp + 16);
  }
}

// ------------------------------------------------------------ walk order ----
// The walk's key of a topic: hashes of its 1-, 2-, 3- and 4-level word-id
// prefixes, b_l bits each (shape: b_l in nibble l, total <= 32 bits), most
// significant first; a level the topic lacks contributes 0.  Sorting by the
// key puts topics that share a prefix next to each other — colliding prefixes
// interleave, a group is never split — so the 64 lanes of a wave issue the
// same bucket reads (one request serves them all) and the L2 keeps what the
// neighbouring waves read.  Any order gives the same result sets.  k_tokenise
// computes the key beside the word ids, and with it the walk's record of the
// topic (the sort's value) and its first FIX_WORDS word ids at a fixed stride,
// so that a wave reads its sorted chunk's topics without an offsets lookup.
__device__ __forceinline__ uint32_t walk_key(const uint32_t* w4, uint32_t D, uint32_t shape) {
  uint64_t h = FNV_BASIS;
  uint32_t k = 0, used = 0;
#pragma unroll
  for (uint32_t l = 0; l < KEY_LEVELS; ++l) {
    const uint32_t bl = (shape >> (4 * l)) & 0xFu;
    h = mix64((h ^ w4[l]) * FNV_PRIME);
    const uint32_t b = (l < D && bl) ? (uint32_t)(h >> (64 - bl)) : 0u;
    k = bl ? ((k << bl) | b) : k;
    used += bl;
  }
  return used < 32 ? k << (32 - used) : k;
}

// the sort's value: topic | (levels | flags << 24 | words at the fixed stride << 31) << 32
__device__ __forceinline__ uint64_t sort_val(uint32_t t, uint32_t D, uint32_t f, bool fixed) {
  return (uint64_t)t | ((uint64_t)(min(D, 0xFFFFFFu) | ((f & 0x7Fu) << 24) | (fixed ? 0x80000000u : 0u)) << 32);
}

// emqx_topic:words/1 (emqx_topic.erl:153-164) + wildcard/1 (:53-62) for a
// block of TOK_BLOCK topics, in three passes over the block's bytes staged in
// LDS so that no lane waits on another's divergent work:
//   1. lane per topic: count '/' four bytes at a time -> levels, '$' flag;
//      block scan -> each topic's first word slot
//   2. lane per topic: record every word's (start, length, output index)
//   3. lane per word, two words per lane in flight: FNV-1a of its bytes, the
//      '+'/'#' words, the byte-exact dictionary probe -> wid[off[t] + t + l]
// The block's topics are taken in segments of S topics, S halved until the
// segment's bytes fit TOK_LDS and its words TOK_WORDS (C3's depth-16 topics
// of ~100 B: two segments of 128).  Only a single topic too long for LDS
// takes the lane-per-topic path from global memory.
__global__ __launch_bounds__(TOK_BLOCK) void k_tokenise(DevTable tab, const uint8_t* __restrict__ blob,
                                                        const uint32_t* __restrict__ off, uint32_t n,
                                                        uint32_t* __restrict__ wid, uint32_t* __restrict__ lv,
                                                        uint8_t* __restrict__ tfl, WalkOrderOut wo) {
  __shared__ __attribute__((aligned(16))) uint32_t sw[TOK_LDS / 4 + 1];   // +1: lds_word reads one word past
  __shared__ uint32_t wpos[TOK_WORDS];   // start | len << 16 (LDS byte index); then the word's id (sorted batch)
  __shared__ uint8_t wtop[TOK_WORDS];    // topic within the segment
  __shared__ uint32_t tg[TOK_BLOCK];     // wid index of the topic's word 0 (a word's is tg + its level)
  __shared__ uint32_t tex[TOK_BLOCK];    // the topic's first word in the segment (a word's level is i - tex)
  __shared__ uint32_t tflag[TOK_BLOCK];   // TF_* flags | levels << 8
  __shared__ uint32_t wsum[TOK_BLOCK / 64];
  const uint32_t blk0 = blockIdx.x * TOK_BLOCK;
  if (blk0 >= n) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // topics past the slot's count are padding (TF_SKIP); an overflowed slot is not matched at all
  const uint32_t n_live = wo.n_live ? (wo.n_live[2] ? 0u : min(wo.n_live[0], n)) : n;
  const uint32_t tend = min(blk0 + (uint32_t)TOK_BLOCK, n);
  uint32_t S = TOK_BLOCK;
  for (uint32_t t0 = blk0; t0 < tend;) {
    // block-uniform segment choice: every thread reads the same offsets
    uint32_t t1, sa, ea;
    for (;;) {
      t1 = min(t0 + S, tend);
      sa = off[t0] & ~3u;
      ea = (off[t1] + 3u) & ~3u;   // blob is readable up to a multiple of 4 (ABI)
      if ((ea - sa) <= (uint32_t)TOK_LDS || S == 1) break;
      S >>= 1;
    }
    const uint32_t t = t0 + tid;
    if ((ea - sa) > (uint32_t)TOK_LDS) {   // one topic longer than LDS: lane path from global memory
      if (tid == 0) {
        const uint32_t ts = off[t0], len = off[t0 + 1] - ts;
        uint32_t l;
        uint8_t fl;
        tokenise_one(tab, (const uint32_t*)(blob + (ts & ~3u)), ts & 3u, len, ts + t0, wid, &l, &fl);
        if (t0 >= n_live) fl |= TF_SKIP;
        lv[t0] = l;
        tfl[t0] = fl;
        if (wo.key) {
          wo.key[t0] = 0xFFFFFFFFu;   // sorted last
          wo.val[t0] = sort_val(t0, l, fl, false);
        }
      }
      t0 = t1;
      continue;
    }
    {
      const uint32_t nw = (ea - sa) >> 2;
      const uint32_t* src = (const uint32_t*)(blob + sa);
      for (uint32_t i = tid; i < nw; i += TOK_BLOCK) sw[i] = src[i];
    }
    __syncthreads();

    // ---- pass 1: levels per topic ----
    uint32_t ts = 0, len = 0, D = 0, fl = 0;
    if (t < t1) {
      ts = off[t] - sa;
      len = off[t + 1] - off[t];
      uint32_t c = 0;
      for (uint32_t q = ts & ~3u; q < ts + len; q += 4) {
        const uint32_t lo = q < ts ? ts - q : 0u, hi = min(4u, ts + len - q);
        c += popc((uint64_t)(slash_mask(sw[q >> 2]) & byte_range(lo, hi)));
      }
      D = c + 1;
      if (len > 0 && lds_byte(sw, ts) == '$') fl |= TF_DOLLAR;
      if (t >= n_live) fl |= TF_SKIP;
    }
    uint32_t wtot;
    uint32_t ex = wave_excl_scan(D, lane, &wtot);
    if (lane == 0) wsum[wv] = wtot;
    __syncthreads();
    uint32_t W = 0;
#pragma unroll
    for (int k = 0; k < TOK_BLOCK / 64; ++k) {
      if ((uint32_t)k < wv) ex += wsum[k];
      W += wsum[k];
    }
    __syncthreads();   // wsum and sw are rewritten by the next segment
    if (W > (uint32_t)TOK_WORDS) {
      if (S > 1) {     // too many words: retry the same topics in a smaller segment
        S >>= 1;
        continue;
      }
      if (tid == 0) {  // one topic with more words than LDS holds
        uint32_t l;
        uint8_t f;
        tokenise_one(tab, sw, ts, len, off[t] + t, wid, &l, &f);
        if (t >= n_live) f |= TF_SKIP;
        lv[t] = l;
        tfl[t] = f;
        if (wo.key) {
          wo.key[t] = 0xFFFFFFFFu;
          wo.val[t] = sort_val(t, l, f, false);
        }
      }
      __syncthreads();
      t0 = t1;
      continue;
    }
    tflag[tid] = fl | (min(D, 0xFFFFFFu) << 8);

    // ---- pass 2: word boundaries ----
    if (t < t1) {
      const uint32_t g = off[t] + t;   // wid index of the topic's first word
      uint32_t l = 0, ws = ts;
      for (uint32_t q = ts & ~3u; q < ts + len; q += 4) {
        const uint32_t lo = q < ts ? ts - q : 0u, hi = min(4u, ts + len - q);
        uint32_t m = slash_mask(sw[q >> 2]) & byte_range(lo, hi);
        while (m) {
          const uint32_t p = q + (__builtin_ctz(m) >> 3);
          m &= m - 1;
          wpos[ex + l] = ws | ((p - ws) << 16);
          wtop[ex + l] = (uint8_t)tid;
          ++l;
          ws = p + 1;
        }
      }
      wpos[ex + l] = ws | ((ts + len - ws) << 16);
      tex[tid] = ex;
      wtop[ex + l] = (uint8_t)tid;
      tg[tid] = g;
      lv[t] = D;
    }
    __syncthreads();

    // ---- pass 3: hash + dictionary probe, lane per word ----
    for (uint32_t i0 = tid; i0 < W; i0 += TOK_U * TOK_BLOCK) {
      uint32_t st[TOK_U], wl[TOK_U], res[TOK_U];
      uint64_t h[TOK_U];
      bool act[TOK_U], spec[TOK_U];
#pragma unroll
      for (int u = 0; u < TOK_U; ++u) {
        const uint32_t i = i0 + u * TOK_BLOCK;
        act[u] = i < W;
        const uint32_t pw = act[u] ? wpos[i] : 0u;
        st[u] = pw & 0xFFFFu;
        wl[u] = pw >> 16;
        h[u] = lds_word_hash(sw, st[u], wl[u]);
        spec[u] = false;
        res[u] = WID_NONE;
        if (wl[u] == 1) {
          const uint32_t c = lds_byte(sw, st[u]);
          if (c == '+' || c == '#') {
            spec[u] = true;
            res[u] = c == '+' ? WID_PLUS : WID_HASH;
          }
        }
      }
      uint4 a[TOK_U], b[TOK_U];
#pragma unroll
      for (int u = 0; u < TOK_U; ++u) {   // every first-slot read in flight (unconditional: see issue())
        const uint8_t* sp = (const uint8_t*)(tab.dict + ((act[u] && !spec[u]) ? ((uint32_t)h[u] & tab.dict_mask) : 0u));
        a[u] = ld16(sp);
        b[u] = ld16(sp + 16);
      }
#pragma unroll
      for (int u = 0; u < TOK_U; ++u) {
        if (!act[u]) continue;
        const uint32_t i = i0 + u * TOK_BLOCK;
        if (spec[u]) atomicOr(&tflag[wtop[i]], (uint32_t)TF_WILDCARD);
        else res[u] = dict_resolve(tab, h[u], a[u], b[u], sw, st[u], wl[u]);
        if (wo.key) {
          // sorted batch: a topic of <= FIX_WORDS levels is read only at the
          // fixed stride (its record's fixed bit), so wid[] is not written
          const uint32_t tt = wtop[i], l = i - tex[tt];
          wpos[i] = res[u];   // only this lane reads word i's position; the key reads the id back
          if ((tflag[tt] >> 8) <= FIX_WORDS) wo.wfix[(uint64_t)(t0 + tt) * FIX_WORDS + l] = res[u];
          else wid[tg[tt] + l] = res[u];
        } else {
          wid[tg[wtop[i]] + i - tex[wtop[i]]] = res[u];
        }
      }
    }
    __syncthreads();
    if (t < t1) {
      tfl[t] = (uint8_t)tflag[tid];
      if (wo.key) {
        uint32_t w4[KEY_LEVELS];
#pragma unroll
        for (uint32_t k = 0; k < KEY_LEVELS; ++k) w4[k] = k < D ? wpos[tex[tid] + k] : 0u;
        wo.key[t] = (tflag[tid] & TF_SKIP) ? 0xFFFFFFFFu : walk_key(w4, D, wo.shape);   // padding sorts last
        wo.val[t] = sort_val(t, D, tflag[tid] & 0xFFu, D <= FIX_WORDS);
      }
    }
    __syncthreads();   // tflag, wpos and sw are rewritten by the next segment
    t0 = t1;
  }
}

// -------------------------------------------------------------- NFA walk ----
// One wavefront walks one chunk of WALK_CHUNK topics at a time (a grid stride
// over the chunks, in walk order when the batch is sorted): topics are
// admitted into the LDS work stack 64 roots at a time as it drains.
//
// A work item is 16 B {node, meta, plus_child, word}:
//   meta = level[0:17) | slot[17:24) | transitions to take[24:28) | took '+' << 28
//   word = the topic's word id at `level`
// A state is finished when it is created, from the record that created it
// (the literal edge slot carries its child's record, the '+' child's record is
// one 16 B read): its 'match_#' emit and, at the topic's last level, its
// lookup_topic emit are staged at once, and only a state that still has a
// literal or '+' transition to take is pushed.  So a popped item costs exactly
// the reads of its own transitions — a bucket line and a 16-B record — plus
// the topic's next word (an L2-resident 4-B read), all issued together.
//
// This is match_compact/4's body (apps/emqx/src/emqx_trie.erl:251-266)
// without string keys:
//   'match_#'(Prefix)          -> the '#' fid of every state created
//   recurse Prefix/Word        -> literal child: bucket probe keyed (node, word)
//   recurse Prefix/'+'         -> '+' child: its record
//   lookup_topic(Topic, IsWc)  -> term fid at level == D if the path took a
//                                 '+' (TRIE mode) / always (ROUTES)
//   do_match/1's '$' rule      -> a '$' topic's root takes no '#'/'+'
//                                 (:208-215), and the single-word probe
//                                 lookup_topic(Prefix) -> term fid at D == 1
constexpr uint32_t ML_BITS = 17;
constexpr uint32_t MT_SHIFT = 17;
constexpr uint32_t MF_SHIFT = 24;
constexpr uint32_t MW_SHIFT = 28;
constexpr uint32_t M_CONT = 1u << 29;   // a literal probe continued: z = the next 64-B edge line to read
constexpr uint32_t LEVEL_MAX = (1u << ML_BITS) - 1;
#ifndef EGM_GUARD_BITS
#define EGM_GUARD_BITS 22   // loop guards: iterations a wave may spend in one loop before reporting a bug
#endif

#ifndef EGM_WALK_STACK
#define EGM_WALK_STACK 320   // items (16 B) per wave: chunks of up to DEEP_MIN levels
#endif
#ifndef EGM_WALK_STACK_DEEP
#define EGM_WALK_STACK_DEEP 504   // items per wave of the deep pass (deeper chunks: C3's wide frontiers; 640 until r5, 448 x 16 B until r6)
#endif
#ifndef EGM_WALK_DEEP_MIN
#define EGM_WALK_DEEP_MIN 12   // a chunk with a deeper topic is walked by the deep pass
#endif
#ifndef EGM_WALK_STAGE
#define EGM_WALK_STAGE 480   // staged emits per flush record, first pass (5 B each in LDS; >= 4 emits x 64 lanes;
                             // 320 until round 6: the first pass is VGPR-bound at 16 waves per CU, so LDS had
                             // room for longer records — fewer, longer runs for k_rec_burst; 448 / 480 / 512
                             // with stack 304: 8.49 / 8.39 / 8.38 ms per step, profiles/r6_walk_stage_ab.jsonl)
#endif
#ifndef EGM_WALK_STAGE_DEEP
#define EGM_WALK_STAGE_DEEP 320   // the deep pass's stage (LDS-bound: 448 would cost it a wave per CU)
#endif
#ifndef EGM_WALK_PAIRS
#define EGM_WALK_PAIRS 0     // A/B: the first pass pops two items per lane per iteration
#endif
#ifndef EGM_PROBE_CONT
#define EGM_PROBE_CONT 1     // a literal probe whose first line holds other keys is continued as a stack item
                             // (1: the first pass; 2: both passes; 0: off — A/B)
#endif
#ifndef EGM_PROBE4
#define EGM_PROBE4 0         // A/B: a literal probe reads all four slots of its bucket (two lines) at once
#endif
#ifndef EGM_PLUS_SKIP
#define EGM_PLUS_SKIP 1      // skip a literal child's '+' transition that would do nothing (A/B: 0)
#endif
#ifndef EGM_WALK_WORDS
#define EGM_WALK_WORDS 448   // staged topic word ids per wave (a chunk's topics, [topic][level])
#endif
#ifndef EGM_WALK_ITEM12
#define EGM_WALK_ITEM12 0        // the first pass keeps 12 B per stack item (A/B)
#endif
#ifndef EGM_WALK_ITEM12_DEEP
#define EGM_WALK_ITEM12_DEEP 1   // the deep pass keeps 12 B per stack item, the word re-read from the word stage:
                                 // 504 items in 10 240 B, 16 waves per CU instead of 14 at 16 B x 448 (C3 deep
                                 // walk 48.8 -> 45.4 ms, profiles/r6_walk_deep_item12_ab.jsonl)
#endif
#ifndef EGM_WALK_WORDS_DEEP
#define EGM_WALK_WORDS_DEEP 448   // the deep pass's word stage (sub-chunks of S topics, S * dmax <= it)
#endif
constexpr uint32_t WALK_STACK = EGM_WALK_STACK;
constexpr uint32_t WALK_STACK_DEEP = EGM_WALK_STACK_DEEP;
constexpr uint32_t DEEP_MIN = EGM_WALK_DEEP_MIN;
constexpr uint32_t WALK_STAGE = EGM_WALK_STAGE;
constexpr uint32_t WALK_STAGE_DEEP = EGM_WALK_STAGE_DEEP;
constexpr uint32_t WALK_STAGE_MAX = WALK_STAGE > WALK_STAGE_DEEP ? WALK_STAGE : WALK_STAGE_DEEP;   // record readers
constexpr uint32_t WALK_STAGE_MIN = WALK_STAGE < WALK_STAGE_DEEP ? WALK_STAGE : WALK_STAGE_DEEP;   // record sizing
constexpr uint32_t WALK_WORDS = EGM_WALK_WORDS;
constexpr uint32_t WALK_WORDS_DEEP = EGM_WALK_WORDS_DEEP;
// The pop bound (below) keeps room >= dmax after every iteration and a refill
// fills the stack to at most 64 items, so the stack cannot overflow while
// 64 + dmax <= the stack; the words of one topic must fit the word stage.
// A chunk with a deeper topic goes to k_heavy before any of it is walked.
__host__ __device__ constexpr uint32_t light_dmax(uint32_t stack, uint32_t words) {
  return (stack - 64) < words ? (stack - 64) : words;
}
static_assert(WALK_CHUNK == 64, "one topic per lane in the chunk prologue");
static_assert(WALK_STAGE_MIN >= 256, "a step stages up to 4 emits x 64 lanes");
static_assert(WALK_STAGE_MAX <= 0xFFFF, "a record's entry count and per-topic counts are 16-bit");
static_assert(light_dmax(WALK_STACK, WALK_WORDS) >= DEEP_MIN, "the first pass must take the chunks it does not hand on");
static_assert(light_dmax(WALK_STACK_DEEP, WALK_WORDS_DEEP) >= 16, "stack too small");

template <uint32_t STK, uint32_t STG, uint32_t WRD, bool N12>
struct alignas(16) WaveLds {
  static constexpr uint32_t STAGE = STG;
  uint4 stack[N12 ? 1 : STK];        // items {node, meta, plus_child, word}
  uint2 sxy[N12 ? STK : 1];          // 12-B items: {node, meta} ...
  uint32_t sz[N12 ? STK : 1];        // ... and plus_child; the word is words[slot][level]
  uint32_t stage_fid[STG];
  uint8_t stage_t[STG];              // topic in chunk of the emit
  uint32_t words[WRD + 2];           // the sub-chunk's word ids, [topic][level] (+2: the unclamped
                                     // reads of the words at level + 1 and + 2, unused past a leaf)
  uint32_t tinfo[WALK_CHUNK];        // D | tflags << 24 | words at the fixed stride << 31
  uint32_t cnt[WALK_CHUNK];          // ids per topic, whole chunk
  uint32_t fcnt[WALK_CHUNK];         // ids per topic in the current stage / its first slot in the record
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
// readfirstlane returns int: widen each half as unsigned (a sign-extended low
// half would set the high word of a pointer whose bit 31 is set)
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | (uint64_t)uni((uint32_t)v);
}

// The wave's current record segment (u32 offsets into MatchWork::rec) and
// the current chunk's record chain (all wave-uniform).
struct RecCursor {
  unsigned long long cur, end;     // free space [cur, end - REC_HDR) of the segment ({0, 0}: none yet)
  unsigned long long first;        // the chunk's first record
  uint32_t nrec;                   // the chunk's records so far
  uint32_t roff;                   // per lane: lane r holds the chunk's record r (offset / 4; r < REC_DIR)
};

#ifndef EGM_FLUSH_NT
#define EGM_FLUSH_NT 1   // flush stores with the nontemporal hint: the records do not displace table lines from L2
#endif
__device__ __forceinline__ void st_u32(uint32_t* p, uint32_t v) {
#if EGM_FLUSH_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Write the stage out as one flush record (round 5).  Each staged entry is
// ranked inside its topic by an LDS atomic on the topic's flush counter
// (ranks stay in registers); one wave scan of the 64 per-topic counts gives
// each topic's first slot, the entries move to their slots in the stage, and
// the record — header, the 64 counts as u16, the ids grouped by topic — goes
// out as one contiguous run of whole lines, lane l writing u32 l, l + 64, ...
// of it.  (Rounds 2-4 wrote each topic's entries into a fixed block of 96 ids
// by walk position: ~5 ids per topic per flush, a partial line in each of ~64
// blocks, 4.10 GB written per C2 walk for 1.99 GB of ids.)
template <class LDS>
__device__ __forceinline__ void flush_stage(LDS& L, uint32_t nstage, uint32_t lane, const MatchWork& w,
                                            RecCursor& rc) {
  constexpr uint32_t NQ = (LDS::STAGE + 63) / 64;
  uint32_t fv[NQ], pv[NQ];   // fid; topic | rank inside the flush << 8
#pragma unroll
  for (uint32_t r = 0; r < NQ; ++r) {
    const uint32_t i = lane + 64 * r;
    const bool act = i < nstage;
    const uint32_t ic = act ? i : 0u;
    const uint32_t tt = L.stage_t[ic];
    fv[r] = L.stage_fid[ic];
    pv[r] = act ? tt | (atomicAdd(&L.fcnt[tt], 1u) << 8) : 0xFFFFFFFFu;
  }
  wave_sync();
  const uint32_t fl = L.fcnt[lane];   // the chunk's topic `lane`: its entries in this flush
  uint32_t tot;
  const uint32_t gx = wave_excl_scan(fl, lane, &tot);
  L.fcnt[lane] = gx;
  // reserve the record: a new segment when the current one cannot hold it and a jump
  const uint32_t size = rec_size(nstage);
  if (rc.cur + size + REC_HDR > rc.end) {   // wave-uniform
    const unsigned long long grain =
        max((unsigned long long)w.rec_grain, (unsigned long long)(size + EGM_REC_ALIGN));   // (keeps the line alignment)
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(&w.stats->rec_cursor, grain);
    b = uni64(__shfl(b, 0, 64));
    if (rc.end && rc.cur + REC_HDR <= w.rec_cap && lane < REC_HDR)   // the old segment's tail: jump to the new one
      st_u32(w.rec + rc.cur + lane, lane == 0 ? REC_JUMP : lane == 2 ? (uint32_t)b : lane == 3 ? (uint32_t)(b >> 32) : 0u);
    rc.cur = b;
    rc.end = b + grain;
  }
  const unsigned long long base = rc.cur;
  rc.cur += size;
  if (rc.nrec == 0) rc.first = base;
  if (lane == rc.nrec) rc.roff = (uint32_t)(base >> 2);
  rc.nrec += 1;
  const bool ok = base + size <= w.rec_cap;
  if (!ok && lane == 0) atomicOr(&w.stats->overflow, 1u);
  wave_sync();
#pragma unroll
  for (uint32_t r = 0; r < NQ; ++r)
    if (pv[r] != 0xFFFFFFFFu) L.stage_fid[L.fcnt[pv[r] & 0xFFu] + (pv[r] >> 8)] = fv[r];
  wave_sync();
  if (ok) {
    // u32 j of the record: j < 4 the header, 4 <= j < 36 the counts of topics 2(j-4) and 2(j-4)+1, then the ids
    const uint32_t k2 = (lane >= REC_HDR && lane < REC_IDS) ? 2u * (lane - REC_HDR) : 0u;
    const uint32_t lo = (uint32_t)__shfl(fl, (int)k2, 64), hi = (uint32_t)__shfl(fl, (int)k2 + 1, 64);
    uint32_t* out = w.rec + base;
#pragma unroll 1
    for (uint32_t j = lane; j < size; j += 64) {
      uint32_t v;
      if (j < REC_HDR) v = j == 0 ? (nstage | REC_TAG) : 0u;
      else if (j < REC_IDS) v = lo | (hi << 16);
      else v = j - REC_IDS < nstage ? L.stage_fid[j - REC_IDS] : 0u;
#ifdef EGM_AB_NO_ID_STORES   // measurement only (tools/build_variant.py): the walk without its id stores
      if (v != 0x7FFFFFF1u) continue;
#endif
      st_u32(out + j, v);
    }
  }
  wave_sync();
  L.cnt[lane] += fl;
  L.fcnt[lane] = 0;
  wave_sync();
}

// Slot search from slot k0 of bucket b on (rare: both first slots hold other keys).
__device__ __forceinline__ bool edge_probe_from(const DevTable& tab, uint32_t b, int k0, uint32_t node, uint32_t w,
                                                uint4* lo_out, uint4* hi_out) {
  for (;;) {
    const EdgeSlot* bp = tab.edges + (size_t)b * EDGE_BUCKET;
    for (int k = k0; k < EDGE_BUCKET; ++k) {
      const uint4 lo = ld16(bp + k);
      const uint4 hi = ld16((const uint8_t*)(bp + k) + 16);
      if (lo.x == node && lo.y == w) {
        *lo_out = lo;
        *hi_out = hi;
        return true;
      }
      if (lo.x == NONE) return false;
    }
    k0 = 0;
    b = (b + 1) & tab.edge_mask;
  }
}

// Staged word ids (round 4): while the dictionary's ids fit 27 bits, the walk
// stages a topic's words in LDS as id | sig_index(id) << 27, so a pop gets
// the next word's literal-child signature bit with two VALU instead of
// re-hashing the word (fmix64: ~13 VALU, five of them quarter-rate
// multiplies, on every pop).  The reserved ids (WID_NONE/PLUS/HASH, >=
// WID_MAX) keep their top bits (31), which no packed id has (< 28).
#ifndef EGM_WORD_SIG
#define EGM_WORD_SIG 1
#endif
constexpr uint32_t WP_SHIFT = 27;
__device__ __forceinline__ uint32_t word_pack(uint32_t w) {
  return w >= WID_MAX ? w : (w | (sig_index(w) << WP_SHIFT));
}
__device__ __forceinline__ uint32_t word_plain(uint32_t p) { return (p >> WP_SHIFT) == 31u ? p : (p & ((1u << WP_SHIFT) - 1u)); }
__device__ __forceinline__ uint32_t word_sig(uint32_t p) {
  const uint32_t k = p >> WP_SHIFT;
  return k < SIG_BITS ? (1u << (SIG_SHIFT + k)) : 0u;
}

// One popped item between issuing its reads and consuming them.
struct Pend {
  uint4 it;                 // the item
  uint32_t D, nw, nsig;     // its topic's depth, the word at level + 1 and its signature bit
  uint32_t nsig2;           // the signature bit of the word at level + 2 (the literal child's '+' child)
  bool act, lit, plus, d1;  // d1: a one-word '$' topic (do_match/1's lookup_topic probe)
  uint4 prec, l0, h0, l1, h1;
  uint32_t line;            // the 64-B edge line read (its two slots are l0/h0, l1/h1)
#if EGM_PROBE4
  uint4 l2, h2, l3, h3;     // A/B: the bucket's second line (slots 2-3) read in the same round
#endif
};

// Branch-free on purpose: every lane issues its loads unconditionally (an
// idle lane reads node 0 / bucket 0, lines every wave keeps hot).  A load
// inside an `if` makes LLVM merge its result at the end of the block, and
// the copy it inserts there waits for the load.  The next level's word comes
// from the LDS word stage (k_walk: `words` = the topic's staged words) or
// from HBM (k_heavy: `words` = null, `wid` + `gbase`).
template <bool CONT>
__device__ __forceinline__ void issue(const DevTable& tab, const uint32_t* words, const uint32_t* __restrict__ wid,
                                      uint32_t gbase, Pend& p) {
  const uint32_t meta = p.it.y;
  const uint32_t fl = (meta >> MF_SHIFT) & 0xFu;
  p.plus = p.act && (fl & F_PLUS);
  p.lit = p.act && (fl & F_LIT) && p.it.w < WID_MAX;
  // the 64-B edge line to read: a bucket's first (two slots), or where a
  // continued probe goes on (M_CONT: its z; such an item takes no '+')
  const uint32_t line = (CONT && (meta & M_CONT)) ? p.it.z : (EDGE_BUCKET / 2) * edge_bucket(p.it.x, p.it.w, tab.edge_mask);
  p.line = line;
  p.prec = ld16(tab.nodes + (p.plus ? p.it.z : 0u));
  const uint8_t* bp = (const uint8_t*)tab.edges + (size_t)(p.lit ? line : 0u) * 64;
  p.l0 = ld16(bp);   // the bucket's first two slots: one 64-B line
  p.h0 = ld16(bp + 16);
  p.l1 = ld16(bp + 32);
  p.h1 = ld16(bp + 48);
#if EGM_PROBE4
  p.l2 = ld16(bp + 64);
  p.h2 = ld16(bp + 80);
  p.l3 = ld16(bp + 96);
  p.h3 = ld16(bp + 112);
#endif
  // the next level's word (used only if level + 1 < D).  From the LDS stage
  // it is read unclamped, so the read does not wait for the topic's depth
  // (a leaf reads the next topic's word 0, or the pad word past the stage).
  uint32_t w2;
  if (words) {
    const uint32_t raw = words[(meta & LEVEL_MAX) + 1];
    const uint32_t raw2 = words[(meta & LEVEL_MAX) + 2];
#if EGM_WORD_SIG
    if (tab.sig_packed) {
      p.nw = word_plain(raw);
      p.nsig = word_sig(raw);
      p.nsig2 = word_sig(raw2);
      return;
    }
#endif
    p.nw = raw;
    w2 = raw2;
  } else {
    p.nw = wid[p.act ? gbase + min((meta & LEVEL_MAX) + 1, p.D - 1) : 0u];
    w2 = wid[p.act ? gbase + min((meta & LEVEL_MAX) + 2, p.D - 1) : 0u];
  }
  p.nsig = p.nw < WID_MAX ? sig_bit(p.nw) : 0u;
  p.nsig2 = w2 < WID_MAX ? sig_bit(w2) : 0u;
}

// Children and emits of one popped item.
struct Out {
  uint32_t f0, f1, f2, f3;  // literal child: '#', terminal; '+' child: '#', terminal
  bool e0, e1, e2, e3;
  uint4 c0, c1;             // children to push
  bool p0, p1;
  bool slow;                // the literal probe needed another bucket read (instrumentation)
  uint32_t created;         // states created (SURVEY §8d V_t)
};

// Straight-line on purpose: every field is computed unconditionally and
// selected by the lane's flags (conditionally assigned fields became phis
// whose copies cost a score of VGPRs).
template <bool CONT>
__device__ __forceinline__ void finish(const DevTable& tab, int mode, const Pend& p, Out& o) {
  const uint32_t meta = p.it.y;
  const uint32_t level = meta & LEVEL_MAX;
  const uint32_t wc = (meta >> MW_SHIFT) & 1u;
  const uint32_t D = p.D;
  const bool leaf = level + 1 == D;
  const uint32_t nw = p.nw;
  const uint32_t base_meta = (level + 1) | (meta & (0x7Fu << MT_SHIFT));
  // the literal probe of a child is only worth a read if its signature has
  // the next word's bit (egm_common.h)
  const uint32_t nsig = p.nsig;
  // literal child: pick the matching slot's fields with masks, not a select
  // of the two loaded slots (LLVM folds that into a phi of addresses into the
  // per-item array and keeps the array in scratch)
  const uint32_t node = p.it.x;
  const bool m0 = p.l0.x == node && p.l0.y == p.it.w;
  const bool z0 = p.l0.x == NONE;
  const bool m1 = !m0 && !z0 && p.l1.x == node && p.l1.y == p.it.w;
  const bool z1 = p.l1.x == NONE;
  const uint32_t s1 = m1 ? 0xFFFFFFFFu : 0u;
  uint32_t cz = (p.l0.z & ~s1) | (p.l1.z & s1), cw = (p.l0.w & ~s1) | (p.l1.w & s1);
  uint32_t hx = (p.h0.x & ~s1) | (p.h1.x & s1), hy = (p.h0.y & ~s1) | (p.h1.y & s1);
  uint32_t hz = (p.h0.z & ~s1) | (p.h1.z & s1), hw = (p.h0.w & ~s1) | (p.h1.w & s1);
  bool found = p.lit && (m0 || m1);
#if EGM_PROBE4
  const bool q = !m0 && !z0 && !m1 && !z1;   // slots 2-3 (already loaded) are next
  const bool m2 = q && p.l2.x == node && p.l2.y == p.it.w, z2 = p.l2.x == NONE;
  const bool m3 = q && !m2 && !z2 && p.l3.x == node && p.l3.y == p.it.w, z3 = p.l3.x == NONE;
  {
    const uint32_t s2 = m2 ? 0xFFFFFFFFu : 0u, s3 = m3 ? 0xFFFFFFFFu : 0u, k = s2 | s3;
    cz = (cz & ~k) | (p.l2.z & s2) | (p.l3.z & s3);
    cw = (cw & ~k) | (p.l2.w & s2) | (p.l3.w & s3);
    hx = (hx & ~k) | (p.h2.x & s2) | (p.h3.x & s3);
    hy = (hy & ~k) | (p.h2.y & s2) | (p.h3.y & s3);
    hz = (hz & ~k) | (p.h2.z & s2) | (p.h3.z & s3);
    hw = (hw & ~k) | (p.h2.w & s2) | (p.h3.w & s3);
  }
  found = found || (p.lit && (m2 || m3));
  const bool slow = p.lit && q && !m2 && !z2 && !m3 && !z3;
  constexpr int K0 = 4;
#else
  const bool slow = p.lit && !m0 && !z0 && !m1 && !z1;
  constexpr int K0 = 2;
#endif
  o.slow = slow;
  if (!CONT && slow) {   // the slots read hold other keys: keep probing
    uint4 lo, hi;
    found = edge_probe_from(tab, edge_bucket(node, p.it.w, tab.edge_mask), K0, node, p.it.w, &lo, &hi);
    cz = lo.z;
    cw = lo.w;
    hx = hi.x;
    hy = hi.y;
    hz = hi.z;
    hw = hi.w;
  }
  cw = found ? cw : 0u;
  o.e0 = (cw & F_HASH) != 0;
  o.f0 = hy;
  o.e1 = leaf && (cw & F_TERM) && (mode == MODE_ROUTES || wc || p.d1);
  o.f1 = hz;
  // the literal child's '+' child (flags from the slot) lands at level + 2
  // when the child is popped: if it would emit nothing and push nothing
  // there, the child does not take that transition — no record read, and no
  // pop at all for a child left with none — and it is counted as created
  // here (SURVEY §8d V_t counts it)
  const uint32_t pfl = found ? hw : 0u;
  const bool leaf2 = level + 2 == D;
#if EGM_PLUS_SKIP
  const bool puse = (pfl & F_HASH) || (leaf2 ? (pfl & F_TERM) != 0
                                            : ((pfl & F_PLUS) || ((pfl & p.nsig2) && (pfl & F_LIT))));
#else
  const bool puse = true;
#endif
  const bool pskip = !leaf && (cw & F_PLUS) && !puse;
  const uint32_t go0 = (puse ? (cw & F_PLUS) : 0u) | ((cw & nsig) ? (cw & F_LIT) : 0u);
  o.p0 = !leaf && go0;
  o.c0 = make_uint4(cz, base_meta | (go0 << MF_SHIFT) | (wc << MW_SHIFT), hx, nw);
  if (CONT && slow) {
    // both slots of the line hold other keys: rather than a second dependent
    // read here, which the whole wave would wait for (82 % of C2's
    // iterations had such a lane, round 6), the probe goes back on the stack
    // as an item that reads the next line (same level, literal transition
    // only) and is popped with the next iteration's items
    const uint32_t nl = (p.line + 1) & ((EDGE_BUCKET / 2) * (tab.edge_mask + 1u) - 1u);
    o.p0 = true;
    o.c0 = make_uint4(node, (meta & ~(0xFu << MF_SHIFT)) | (F_LIT << MF_SHIFT) | M_CONT, nl, p.it.w);
  }
  // '+' child
  const uint32_t pf = p.plus ? p.prec.w : 0u;
  o.e2 = (pf & F_HASH) != 0;
  o.f2 = p.prec.y;
  o.e3 = leaf && (pf & F_TERM);
  o.f3 = p.prec.z;
  const uint32_t go1 = (pf & F_PLUS) | ((pf & nsig) ? (pf & F_LIT) : 0u);
  o.p1 = !leaf && go1;
  o.c1 = make_uint4(p.it.z, base_meta | (go1 << MF_SHIFT) | (1u << MW_SHIFT), p.prec.x, nw);
  o.created = (found ? 1u : 0u) + (p.plus ? 1u : 0u) + (pskip ? 1u : 0u);
}

// lookup_routes(Topic) of a wildcard topic in ROUTES mode (emqx_router.erl:
// 129-134): the topic's words walked as a literal key, '+'/'#' words taking
// the '+'/'#' edges.  Rare (MQTT publishes never carry wildcards): one lane,
// one dependent read per level.
__device__ bool exact_walk(const DevTable& tab, const uint32_t* __restrict__ words, uint32_t D, uint32_t* fid) {
  uint32_t node = 0;
  for (uint32_t l = 0; l < D; ++l) {
    const uint32_t wd = words[l];
    uint32_t child = NONE;
    if (wd == WID_PLUS) child = tab.nodes[node].plus_child;
    else if (wd == WID_HASH) child = tab.hash_child[node];
    else if (wd < WID_MAX) {
      uint4 lo, hi;
      if (edge_probe_from(tab, edge_bucket(node, wd, tab.edge_mask), 0, node, wd, &lo, &hi)) child = lo.z;
    }
    if (child == NONE) return false;
    node = child;
  }
  const NodeRec r = tab.nodes[node];
  *fid = r.term_fid;
  return (r.flags & F_TERM) != 0;
}

// The root state of a topic: its '#' emit (never for a '$' topic) and the
// transitions it has to take (s0: the signature bit of its first word).
__device__ __forceinline__ uint32_t root_flags(uint4 root, bool dollar, uint32_t s0) {
  return (dollar ? 0u : (root.w & F_PLUS)) | ((root.w & s0) ? (root.w & F_LIT) : 0u);
}

// A topic's word ids: at the fixed stride of the sorted batch, or in wid[].
__device__ __forceinline__ const uint32_t* topic_words(const MatchWork& w, uint32_t tinfo, uint32_t gbase) {
  return (tinfo >> 31) ? w.wfix + (uint64_t)gbase * FIX_WORDS : w.wid + gbase;
}

// One wave walks one chunk of 64 topics at a time (a grid stride over the
// chunks).  The chunk's words are staged in LDS ([topic][level]; deep topics
// in sub-chunks of S topics with S * dmax <= WALK_WORDS), topics are admitted
// 64 roots at a time while the stack is short, and the wave pops up to 64
// items per iteration.
//
// Two passes: the first (DEEP = false, a 320-item stack, 17 waves per CU)
// walks the chunks of up to DEEP_MIN levels and hands deeper ones to the
// second (DEEP = true: a 504-item stack of 12-B items, 16 waves per CU), whose wider stack
// keeps the wave's pops full on deep, wide frontiers (C3: lane occupancy 0.39
// -> 0.80) where the first pass's room bound would narrow it; a chunk deeper
// than the deep pass takes goes to k_heavy.
#ifdef EGM_WALK_WPE   // A/B: ask the compiler for this many waves per SIMD (caps VGPRs)
#define EGM_WALK_ATTR __attribute__((amdgpu_waves_per_eu(EGM_WALK_WPE)))
#else
#define EGM_WALK_ATTR
#endif
// Hand the first n (wave-uniform) of lane-held chunk ids to the deep pass.
__device__ __forceinline__ void deep_flush(const MatchWork& w, uint32_t c, uint32_t n, uint32_t lane) {
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(&w.stats->n_deep, n);
  base = uni(__shfl(base, 0, 64));
  if (lane < n) w.deep[base + lane] = c;
}

template <bool DEEP>
__global__ __launch_bounds__(64) EGM_WALK_ATTR void k_walk(DevTable tab, const uint32_t* __restrict__ off, uint32_t n,
                                                           int mode, MatchWork w) {
  constexpr uint32_t STK = DEEP ? WALK_STACK_DEEP : WALK_STACK;
  // probe continuations in the first pass only: the deep pass (C3) measured
  // 53.8 -> 55.2 ms with them, the first pass (C2) 8.20 -> 6.23 ms (round 6)
  constexpr bool PROBE_CONT = EGM_PROBE_CONT != 0 && (!DEEP || EGM_PROBE_CONT > 1);
  constexpr uint32_t STG = DEEP ? WALK_STAGE_DEEP : WALK_STAGE;
  constexpr uint32_t WRD = DEEP ? WALK_WORDS_DEEP : WALK_WORDS;
  // (a continued probe keeps its line in z and its word is the one at its level: it fits 12 B too)
  constexpr bool N12 = DEEP ? EGM_WALK_ITEM12_DEEP != 0 : EGM_WALK_ITEM12 != 0;
  __shared__ WaveLds<STK, STG, WRD, N12> L;
  auto st_put = [&](uint32_t i, const uint4& v) {
    if constexpr (N12) {
      L.sxy[i] = make_uint2(v.x, v.y);
      L.sz[i] = v.z;
    } else {
      L.stack[i] = v;
    }
  };
  auto st_get = [&](uint32_t i) -> uint4 {
    if constexpr (N12) {
      const uint2 a = L.sxy[i];
      return make_uint4(a.x, a.y, L.sz[i], 0u);
    } else {
      return L.stack[i];
    }
  };
  const uint32_t lane = threadIdx.x;
  // the first pass walks every chunk, the deep pass the chunks the first handed on
  const uint32_t ct = w.ct;   // topics per chunk (lanes >= ct hold none)
  const uint32_t nchunks = DEEP ? uni(*(volatile unsigned int*)&w.stats->n_deep) : (n + ct - 1) / ct;
  uint4 root = ld16(tab.nodes);   // wave-uniform: keep it in SGPRs
  root.x = uni(root.x);
  root.y = uni(root.y);
  root.z = uni(root.z);
  root.w = uni(root.w);
  uint32_t created = 0;
  unsigned long long iters = 0, popped = 0, bounded = 0, lit_probes = 0, plus_reads = 0;
  uint32_t slow_lanes = 0, slow_iters = 0;
  RecCursor rc{0, 0, 0, 0, 0};
  const uint32_t guard_lim = (w.debug & DEBUG_FORCE_GUARD) ? 2u : (1u << EGM_GUARD_BITS);
  // sorted batch: the record of the chunk's j-th topic in walk order, loaded
  // one chunk ahead (a grid stride: the wave's next chunk is c + gridDim.x)
  const uint64_t* ord = w.order;
  uint64_t rec = (ord && !DEEP) ? ord[min(blockIdx.x * ct + lane, n - 1)] : 0ull;
  uint32_t deep_c = 0, n_pend = 0;   // chunks for the deep pass not yet handed on
  for (uint32_t ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const uint32_t c = DEEP ? uni(w.deep[ci]) : ci;
    const uint32_t t0 = c * ct;
    const uint32_t nt = min(ct, n - t0);
    // ---- topic info (lane j: the chunk's j-th topic in walk order) ----
    uint32_t D = 0, f = 0, my_t = 0;
    bool fixed = false;
    if (ord) {
      const uint64_t r = DEEP ? ord[min(t0 + lane, n - 1)] : rec;
      if (!DEEP) rec = ord[min((uint64_t)(c + gridDim.x) * ct + lane, (uint64_t)n - 1)];   // the next chunk's, in flight now
      if (lane < nt) {
        my_t = (uint32_t)r;
        D = (uint32_t)(r >> 32) & 0xFFFFFFu;
        f = (uint32_t)(r >> 56) & 0x7Fu;
        fixed = (r >> 63) != 0;
      }
    } else if (lane < nt) {
      my_t = t0 + lane;
      D = w.lv[my_t];
      f = w.tfl[my_t];
    }
    L.tinfo[lane] = D | (f << 24) | (fixed ? 0x80000000u : 0u);
    L.cnt[lane] = 0;
    L.fcnt[lane] = 0;
    uint32_t dmax = D;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) dmax = max(dmax, (uint32_t)__shfl_xor(dmax, d, 64));
    dmax = uni(dmax);
    if (dmax > light_dmax(WALK_STACK_DEEP, WALK_WORDS_DEEP) || (w.debug & DEBUG_FORCE_HEAVY)) {   // the whole chunk goes to k_heavy
      if (lane == 0) {
        const uint32_t d = atomicAdd(&w.stats->n_deferred, 1u);
        w.deferred[d] = c;
        w.chunks[c] = make_uint4(0, 0, 0, CHUNK_HEAVY);
      }
      continue;
    }
    if (!DEEP && dmax > DEEP_MIN) {   // to the deep pass: lane k holds the wave's k-th such chunk,
      deep_c = lane == n_pend ? c : deep_c;   // handed on 64 at a time (one atomic per 64: a
      if (++n_pend == 64) {                   // per-chunk atomic on one counter serialised a C3 batch)
        deep_flush(w, deep_c, n_pend, lane);
        n_pend = 0;
      }
      continue;
    }
    // lane j's register: a wid[] index (off[t] + t) or its topic (fixed stride);
    // only words at a variable offset need off[] (read by other lanes with a shuffle)
    const uint32_t gb = lane < nt ? (fixed ? my_t : off[my_t] + my_t) : 0u;
    uint32_t S = WALK_CHUNK;
    while (S > 1 && S * dmax > WRD) S >>= 1;
    uint32_t nstage = 0;
    rc.nrec = 0;
    const uint32_t flim = min(w.flush_lim, STG);   // this pass's stage (the host's limit is the larger one's)
    wave_sync();
    for (uint32_t sub = 0; sub < nt; sub += S) {
      const uint32_t end = min(sub + S, nt);
      const uint32_t gsub = __shfl(gb, (int)min(sub + lane, (uint32_t)WALK_CHUNK - 1), 64);
      if (lane < end - sub) {   // stage the sub-chunk's words: topic j's word 0 at LDS (j % S) * dmax
        const uint32_t j = sub + lane, Dj = L.tinfo[j] & 0xFFFFFFu;
        const uint32_t* src = topic_words(w, L.tinfo[j], gsub);
        uint32_t* dst = L.words + lane * dmax;
        const bool pk = EGM_WORD_SIG && tab.sig_packed;
        uint32_t i = 0;
        for (; i + 4 <= Dj; i += 4) {
          const uint32_t a0 = src[i], a1 = src[i + 1], a2 = src[i + 2], a3 = src[i + 3];
          dst[i] = pk ? word_pack(a0) : a0;
          dst[i + 1] = pk ? word_pack(a1) : a1;
          dst[i + 2] = pk ? word_pack(a2) : a2;
          dst[i + 3] = pk ? word_pack(a3) : a3;
        }
        for (; i < Dj; ++i) dst[i] = pk ? word_pack(src[i]) : src[i];
      }
      wave_sync();
      uint32_t next = sub, sp = 0;
      uint32_t guard = 0;   // every loop of the kernel is bounded: a bug reports, it never hangs the GPU
      for (;;) {
        if (++guard > guard_lim) {
          if (lane == 0) atomicOr(&w.stats->guard, GUARD_LOOP);
          break;
        }
        // ---- admit new topics while the stack is short: their root '#'
        // emit, their root item (a wildcard topic in ROUTES mode: one exact
        // lookup, no item) ----
        if (sp < 64u && next < end) {
          const uint32_t k = min(64u - sp, end - next);
          if (nstage && nstage + 64u > flim) {
            flush_stage(L, nstage, lane, w, rc);
            nstage = 0;
          }
          bool has = false, em = false;
          uint32_t fid = NONE;
          uint4 it = make_uint4(0, 0, 0, 0);
          const uint32_t j = next + lane;
          const uint32_t gj = __shfl(gb, (int)min(j, (uint32_t)WALK_CHUNK - 1), 64);
          if (lane < k) {
            const uint32_t ti = L.tinfo[j], Dj = ti & 0xFFFFFFu, tf = (ti >> 24) & 0x7Fu;
            if (tf & (TF_WILDCARD | TF_SKIP)) {   // padding: no walk, no ids
              if (mode == MODE_ROUTES && !(tf & TF_SKIP)) em = exact_walk(tab, topic_words(w, ti, gj), Dj, &fid);
            } else {
              const bool dollar = (tf & TF_DOLLAR) != 0;
              em = (root.w & F_HASH) && !dollar;   // filter '#': never for a '$' topic
              fid = root.y;
              created += 1;
              const uint32_t w0r = L.words[(j & (S - 1)) * dmax];
              const bool pk = EGM_WORD_SIG && tab.sig_packed;
              const uint32_t w0 = pk ? word_plain(w0r) : w0r;
              const uint32_t rf = root_flags(root, dollar, pk ? word_sig(w0r) : (w0 < WID_MAX ? sig_bit(w0) : 0u));
              has = rf != 0;
              it = make_uint4(0, (j << MT_SHIFT) | (rf << MF_SHIFT), root.x, w0);
            }
          }
          const uint64_t b = __ballot(has);
          if (has) st_put(sp + mbcnt(b), it);
          sp += popc(b);
          const uint64_t be = __ballot(em);
          if (em) {
            const uint32_t q = nstage + mbcnt(be);
            L.stage_fid[q] = fid;
            L.stage_t[q] = (uint8_t)j;
          }
          nstage += popc(be);
          next += k;
          wave_sync();
        }
        if (sp == 0) {
          if (next >= end) break;
          continue;
        }
        // ---- pop up to 64 items and issue all their reads ----
        // An item pushes at most two children (net +1), so popping k <= room -
        // dmax items keeps room >= dmax afterwards; with room <= dmax the wave
        // pops one item at a time, a plain DFS, whose stack grows by at most
        // one pending sibling per level below the top item.  So the stack
        // never overflows: a deep, wide frontier (C3: depth 16, '+' p=.35)
        // narrows the wave instead.
        const uint32_t room = STK - sp;
        const uint32_t lim = room > dmax ? room - dmax : 1u;
        // EGM_WALK_PAIRS (A/B): the first pass pops up to 128 items per
        // iteration, two per lane — twice the reads in flight per wave and
        // the iteration's fixed work shared by two items (same pop bound)
        constexpr bool PAIRS = EGM_WALK_PAIRS && !DEEP;
        const uint32_t want = min(PAIRS ? 128u : 64u, sp), take = min(want, lim), bi = sp - take;
        const uint32_t take_a = min(take, 64u), take_b = take - take_a;
        bounded += take < want ? 1u : 0u;
        iters += 1;
        popped += take;
        Pend p, pb;
        p.act = lane < take_a;
        p.it = st_get(min(bi + lane, STK - 1));   // unconditional: see issue()
        if (PAIRS) {
          pb.act = lane < take_b;
          pb.it = st_get(min(bi + 64 + lane, STK - 1));
        }
        sp = bi;
        const uint32_t tt = (p.it.y >> MT_SHIFT) & 0x7Fu;
        const uint32_t ti = L.tinfo[tt];
        p.D = ti & 0xFFFFFFu;
        p.d1 = p.D == 1 && ((ti >> 24) & TF_DOLLAR);   // TF_DOLLAR < 0x80: the fixed-stride bit is not read
        if constexpr (N12) {   // the item's word: its topic's staged word at its level
          const uint32_t raw = L.words[(tt & (S - 1)) * dmax + min(p.it.y & LEVEL_MAX, dmax - 1)];
          p.it.w = (EGM_WORD_SIG && tab.sig_packed) ? word_plain(raw) : raw;
        }
        issue<PROBE_CONT>(tab, L.words + (tt & (S - 1)) * dmax, nullptr, 0, p);
        uint32_t ttb = 0;
        if (PAIRS) {
          ttb = (pb.it.y >> MT_SHIFT) & 0x7Fu;
          const uint32_t tib = L.tinfo[ttb];
          pb.D = tib & 0xFFFFFFu;
          pb.d1 = pb.D == 1 && ((tib >> 24) & TF_DOLLAR);
          issue<PROBE_CONT>(tab, L.words + (ttb & (S - 1)) * dmax, nullptr, 0, pb);
          lit_probes += popc(__ballot(pb.lit));
          plus_reads += popc(__ballot(pb.plus));
        }
        lit_probes += popc(__ballot(p.lit));
        plus_reads += popc(__ballot(p.plus));
        wave_sync();
        // ---- consume: children -> stack, emits -> stage ----
        auto consume = [&](const Pend& q, uint32_t qt) -> bool {
          Out o;
          finish<PROBE_CONT>(tab, mode, q, o);
          created += o.created;
          {
            const uint32_t ns = popc(__ballot(o.slow));
            slow_lanes += ns;
            slow_iters += ns ? 1u : 0u;
          }
          const uint64_t c0b = __ballot(o.p0), c1b = __ballot(o.p1);
          const uint32_t m0 = popc(c0b), nc = m0 + popc(c1b);
          if (sp + nc > STK) {   // guard only: the pop bound keeps sp + pushes <= STK
            if (lane == 0) atomicOr(&w.stats->guard, GUARD_STACK);
            return false;
          }
          if (o.p0) st_put(sp + mbcnt(c0b), o.c0);
          if (o.p1) st_put(sp + m0 + mbcnt(c1b), o.c1);
          sp += nc;
          const uint64_t b0 = __ballot(o.e0), b1 = __ballot(o.e1), b2 = __ballot(o.e2), b3 = __ballot(o.e3);
          const uint32_t n0 = popc(b0), n1 = n0 + popc(b1), n2 = n1 + popc(b2), ne = n2 + popc(b3);
          if (nstage && nstage + ne > flim) {   // (flim <= WALK_STAGE: the stage never overfills)
            wave_sync();
            flush_stage(L, nstage, lane, w, rc);
            nstage = 0;
          }
          const uint8_t st = (uint8_t)qt;
          if (o.e0) {
            const uint32_t x = nstage + mbcnt(b0);
            L.stage_fid[x] = o.f0;
            L.stage_t[x] = st;
          }
          if (o.e1) {
            const uint32_t x = nstage + n0 + mbcnt(b1);
            L.stage_fid[x] = o.f1;
            L.stage_t[x] = st;
          }
          if (o.e2) {
            const uint32_t x = nstage + n1 + mbcnt(b2);
            L.stage_fid[x] = o.f2;
            L.stage_t[x] = st;
          }
          if (o.e3) {
            const uint32_t x = nstage + n2 + mbcnt(b3);
            L.stage_fid[x] = o.f3;
            L.stage_t[x] = st;
          }
          nstage += ne;
          return true;
        };
        if (!consume(p, tt)) break;
        if (PAIRS && take_b) {
          if (!consume(pb, ttb)) break;
        }
        wave_sync();
      }
    }
    if (nstage) flush_stage(L, nstage, lane, w, rc);
    if (lane < nt) w.cnt[w.walk_rows ? t0 + lane : my_t] = L.cnt[lane];
    if (lane == 0) w.chunks[c] = make_uint4((uint32_t)rc.first, (uint32_t)(rc.first >> 32), rc.nrec, CHUNK_WALKED);
    if (lane < min(rc.nrec, REC_DIR)) w.dir[(uint64_t)c * REC_DIR + lane] = rc.roff;   // the chunk's directory
    wave_sync();
  }
  if (!DEEP && n_pend) deep_flush(w, deep_c, n_pend, lane);
  unsigned long long v = created;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if (lane == 0 && (iters || v)) {   // a wave that walked nothing adds nothing (same-address atomics serialise)
    if (v) atomicAdd(&w.stats->visited, v);
    atomicAdd(&w.stats->iters, iters);
    atomicAdd(&w.stats->popped, popped);
    if (bounded) atomicAdd(&w.stats->bounded, bounded);
    atomicAdd(&w.stats->lit_probes, lit_probes);
    atomicAdd(&w.stats->plus_reads, plus_reads);
    if (slow_lanes) {
      atomicAdd(&w.stats->slow_lanes, slow_lanes);
      atomicAdd(&w.stats->slow_iters, slow_iters);
    }
  }
}

// ----------------------------------------------------------------- heavy ----
// Topics of deferred chunks (a topic deeper than the walk's deep pass takes, or every chunk
// under DEBUG_FORCE_HEAVY): one wave per topic, the same states and pop bound
// as k_walk, but the stack lives in HBM — heavy_cap items per wave, sized by
// the host to at least the batch's deepest possible topic + 192, so by the
// pop-bound argument no legal topic (<= 65 535 bytes, emqx_topic.erl:45,
// 99-100) can overflow it.  Two passes: count, then fill at a reserved offset
// (one piece per topic).
__device__ __forceinline__ void heavy_fence() {
  // the wave's own stack stores must have reached L2 before its next loads of them
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// Stack reads bypass the CU's L1 (a nontemporal load is served by L2): the
// L1 may still hold a line of the stack from before the wave's own stores to it.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_l2(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__global__ __launch_bounds__(64) void k_heavy(DevTable tab, const uint32_t* __restrict__ off, uint32_t n, int mode,
                                              MatchWork w) {
  const uint32_t lane = threadIdx.x;
  uint4 root = ld16(tab.nodes);
  root.x = uni(root.x);
  root.y = uni(root.y);
  root.z = uni(root.z);
  root.w = uni(root.w);
  const uint32_t ct = w.ct, total = w.stats->n_deferred * ct;
  uint4* stk = w.heavy_stack + (uint64_t)blockIdx.x * w.heavy_cap;
  const uint32_t cap = w.heavy_cap;
  const uint32_t guard_lim = (w.debug & DEBUG_FORCE_GUARD) ? 2u : (1u << EGM_GUARD_BITS);
  unsigned long long created = 0;
  for (;;) {
    uint32_t idx = 0;
    if (lane == 0) idx = atomicAdd(&w.stats->heavy_next, 1u);
    idx = uni(__shfl(idx, 0, 64));
    if (idx >= total) break;
    const uint32_t pos = w.deferred[idx / ct] * ct + idx % ct;   // in walk order
    if (pos >= n) continue;
    const uint64_t rec = w.order ? w.order[pos] : (uint64_t)pos;
    const uint32_t t = uni((uint32_t)rec);
    const uint32_t row = w.walk_rows ? pos : t;   // every id of a heavy topic is in its piece
    // a sorted batch keeps a short topic's words only at the fixed stride (k_tokenise)
    const bool fixed = w.order && (rec >> 63);
    const uint32_t* words = fixed ? w.wfix : w.wid;
    const uint32_t D = uni(w.lv[t]), tf = uni(w.tfl[t]), tb = uni(fixed ? t * FIX_WORDS : off[t] + t);
    if (tf & (TF_WILDCARD | TF_SKIP)) {   // no trie walk: TRIE mode matches nothing, ROUTES mode one exact lookup
      uint32_t fid = NONE;
      const bool em = mode == MODE_ROUTES && !(tf & TF_SKIP) && exact_walk(tab, words + tb, D, &fid);
      if (lane == 0) {
        if (em) {
          const unsigned long long base = atomicAdd(&w.stats->cursor, 1ull);
          const unsigned long long p = atomicAdd(&w.stats->pieces, 1ull);
          if (base < w.ids_cap && p < w.pieces_cap) {
            w.ids_tmp[base] = fid;
            w.pieces[p] = make_uint4(row, 1, (uint32_t)base, 0);
          } else {
            atomicOr(&w.stats->overflow, 1u);
          }
        }
        w.cnt[row] = em ? 1u : 0u;
        w.tfl[t] = (uint8_t)(tf | TF_HEAVY);
      }
      continue;
    }
    if (D + 192u > cap) {   // cannot happen for a legal topic (the host sizes cap from the batch)
      if (lane == 0) {
        atomicAdd(&w.stats->errors, 1u);
        w.cnt[row] = 0;
        w.tfl[t] = (uint8_t)(tf | TF_HEAVY | TF_ERROR);
      }
      continue;
    }
    const bool dollar = (tf & TF_DOLLAR) != 0;
    const uint32_t w0 = uni(words[tb]);
    const uint32_t rfl = root_flags(root, dollar, w0 < WID_MAX ? sig_bit(w0) : 0u);
    const bool rem = (root.w & F_HASH) && !dollar;
    unsigned long long base = 0;
    uint32_t count = 0;
    bool fits = true;
    for (int pass = 0; pass < 2; ++pass) {
      uint32_t sp = 0, k = 0;
      if (rem) {
        if (pass == 1 && fits && lane == 0) w.ids_tmp[base] = root.y;
        k = 1;
      }
      if (rfl) {
        if (lane == 0) stk[0] = make_uint4(0, rfl << MF_SHIFT, root.x, w0);
        sp = 1;
      }
      if (pass == 0 && lane == 0) created += 1;
      heavy_fence();
      uint32_t guard = 0;
      while (sp) {
        if (++guard > guard_lim) {
          if (lane == 0) atomicOr(&w.stats->guard, GUARD_LOOP);
          break;
        }
        const uint32_t room = cap - sp;
        const uint32_t lim = room > D ? room - D : 1u;
        const uint32_t take = min(min(64u, sp), lim), bi = sp - take;
        Pend p;
        p.act = lane < take;
        p.it = ld16_l2(stk + (p.act ? bi + lane : 0u));
        p.D = D;
        p.d1 = D == 1 && (tf & TF_DOLLAR);
        issue<false>(tab, nullptr, words, tb, p);
        sp = bi;
        Out o;
        finish<false>(tab, mode, p, o);
        if (pass == 0) created += o.created;
        const uint64_t c0b = __ballot(o.p0), c1b = __ballot(o.p1);
        const uint32_t m0 = popc(c0b);
        if (sp + m0 + popc(c1b) > cap) {   // guard only: the pop bound keeps sp + pushes <= cap
          count = 0;
          fits = false;
          if (lane == 0) atomicOr(&w.stats->guard, GUARD_STACK);
          break;
        }
        heavy_fence();   // every lane's pop load is done before the pushes overwrite those entries
        if (o.p0) stk[sp + mbcnt(c0b)] = o.c0;
        if (o.p1) stk[sp + m0 + mbcnt(c1b)] = o.c1;
        sp += m0 + popc(c1b);
        const uint64_t b0 = __ballot(o.e0), b1 = __ballot(o.e1), b2 = __ballot(o.e2), b3 = __ballot(o.e3);
        const uint32_t n0 = popc(b0), n1 = popc(b1), n2 = popc(b2);
        if (pass == 1 && fits) {
          if (o.e0) w.ids_tmp[base + k + mbcnt(b0)] = o.f0;
          if (o.e1) w.ids_tmp[base + k + n0 + mbcnt(b1)] = o.f1;
          if (o.e2) w.ids_tmp[base + k + n0 + n1 + mbcnt(b2)] = o.f2;
          if (o.e3) w.ids_tmp[base + k + n0 + n1 + n2 + mbcnt(b3)] = o.f3;
        }
        k += n0 + n1 + n2 + popc(b3);
        heavy_fence();
      }
      if (pass == 0) {
        count = k;
        unsigned long long pb = 0;
        if (lane == 0 && count) {
          base = atomicAdd(&w.stats->cursor, (unsigned long long)count);
          pb = atomicAdd(&w.stats->pieces, 1ull);
        }
        base = __shfl(base, 0, 64);
        pb = __shfl(pb, 0, 64);
        fits = count == 0 || (base + count <= w.ids_cap && pb < w.pieces_cap);
        if (lane == 0) {
          if (!fits) atomicOr(&w.stats->overflow, 1u);
          w.cnt[row] = count;
          if (count && fits) w.pieces[pb] = make_uint4(row, count, (uint32_t)base, 0);
          w.tfl[t] = (uint8_t)(tf | TF_HEAVY);
        }
        if (!count || !fits) break;
      }
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) created += __shfl_xor(created, d, 64);
  if (lane == 0 && created) atomicAdd(&w.stats->visited, created);
}

// ------------------------------------------------------------------ scan ----
// counts u32[n] -> row_ptr u64[n+1] (exclusive), three launches.
__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t* __restrict__ cnt, uint32_t n,
                                                     uint64_t* __restrict__ tile_sums) {
  __shared__ uint64_t part[4];
  const uint32_t i0 = blockIdx.x * SCAN_TILE + threadIdx.x * 8;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (i0 + k < n) s += cnt[i0 + k];
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_down(s, d, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(1024) void k_scan_top(uint64_t* __restrict__ tile_sums, uint32_t ntiles) {
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry_s;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < ntiles; b0 += 1024) {
    const uint32_t i = b0 + threadIdx.x;
    const uint64_t v = i < ntiles ? tile_sums[i] : 0;
    uint64_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
      uint64_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t pre = carry_s;
    for (uint32_t k = 0; k < wv; ++k) pre += wsum[k];
    if (i < ntiles) tile_sums[i] = pre + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry_s = pre + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_sums[ntiles] = carry_s;
}

__global__ __launch_bounds__(256) void k_scan_apply(const uint32_t* __restrict__ cnt, uint32_t n,
                                                    const uint64_t* __restrict__ tile_sums, uint32_t ntiles,
                                                    uint64_t* __restrict__ row_ptr, uint64_t* __restrict__ copy) {
  __shared__ uint64_t wsum[4];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t i0 = blockIdx.x * SCAN_TILE + threadIdx.x * 8;
  uint32_t v[8];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = (i0 + k < n) ? cnt[i0 + k] : 0u;
    s += v[k];
  }
  uint64_t x = s;
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint64_t pre = tile_sums[blockIdx.x];
  for (uint32_t k = 0; k < wv; ++k) pre += wsum[k];
  pre += x - s;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (i0 + k < n) {
      row_ptr[i0 + k] = pre;
      if (copy) copy[i0 + k] = pre;
    }
    pre += v[k];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) row_ptr[n] = tile_sums[ntiles];
}

// Small arrays (n <= SCAN_SMALL): the whole scan in one launch of one block
// — a small batch's scan is three launches' fixed cost otherwise (round 6:
// 3 x 4.5 us of a 4096-topic batch's ~330 us).
constexpr uint32_t SCAN_SMALL = 65536;
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t* __restrict__ cnt, uint32_t n,
                                                     uint64_t* __restrict__ row_ptr, uint64_t* __restrict__ copy) {
  __shared__ uint64_t wsum[16];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t per = (n + 1023) / 1024, i0 = threadIdx.x * per;
  uint64_t s = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (i0 + k < n) s += cnt[i0 + k];
  uint64_t x = s;
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint64_t pre = x - s;
  for (uint32_t k = 0; k < wv; ++k) pre += wsum[k];
  for (uint32_t k = 0; k < per; ++k) {
    if (i0 + k < n) {
      row_ptr[i0 + k] = pre;
      if (copy) copy[i0 + k] = pre;
      pre += cnt[i0 + k];
    }
  }
  if (threadIdx.x == 1023) row_ptr[n] = pre;   // the last thread's running sum: the total
}

// Spilled pieces -> CSR rows, no atomics.  One wave per window of 64 pieces:
// a wave scan lays the window's ids out as one run [0, tot), and the lanes
// copy that run with consecutive lanes on consecutive ids (a binary search
// over the window's 64 scan values finds each id's piece).  Unused slab slots
// (count 0) are skipped.  Pieces hold the ids past a topic's fixed block (and
// every id of a heavy topic): a few percent of the batch at C2.
#ifndef EGM_COMPACT_WAVES
#define EGM_COMPACT_WAVES 4
#endif
#ifndef EGM_COMPACT_BLOCKS
#define EGM_COMPACT_BLOCKS 65536   // grid cap
#endif
constexpr int COMPACT_WAVES = EGM_COMPACT_WAVES;
constexpr int COMPACT_IPL = 8;   // ids per lane per copy round in flight

// The copy of one window of up to 64 runs (src, dst, count) laid out in LDS.
__device__ __forceinline__ void copy_runs(const uint32_t* __restrict__ src_base, uint32_t* __restrict__ ids,
                                          const uint32_t* s_scan, const uint64_t* s_src, const uint64_t* s_dst,
                                          uint32_t tot, uint32_t lane) {
  for (uint32_t q0 = lane; q0 < tot; q0 += 64 * COMPACT_IPL) {
    uint32_t v[COMPACT_IPL];
    uint64_t d[COMPACT_IPL];
#pragma unroll
    for (int r = 0; r < COMPACT_IPL; ++r) {
      const uint32_t q = min(q0 + 64u * r, tot - 1);
      uint32_t k = 0;
#pragma unroll
      for (uint32_t step = 32; step >= 1; step >>= 1)
        if (s_scan[k + step] <= q) k += step;
      const uint32_t o = q - s_scan[k];
      d[r] = s_dst[k] + o;
      v[r] = src_base[s_src[k] + o];
    }
#pragma unroll
    for (int r = 0; r < COMPACT_IPL; ++r)
      if (q0 + 64u * r < tot) ids[d[r]] = v[r];   // plain stores: nontemporal ones measured 2x slower here
  }
}

__device__ __forceinline__ bool compact_checks(const uint64_t* row_ptr, uint32_t n, uint64_t ids_cap,
                                               MatchStats* stats) {
  const uint64_t total = row_ptr[n];
  if (blockIdx.x == 0 && threadIdx.x == 0) stats->total_ids = total;
  if (stats->overflow || stats->guard) return false;   // a guard trip: no rows are assembled
  if (total > ids_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&stats->overflow, 2u);
    return false;
  }
  return true;
}

__global__ __launch_bounds__(64 * COMPACT_WAVES) void k_compact(const uint4* __restrict__ pieces,
                                                                const uint32_t* __restrict__ ids_tmp, uint32_t n,
                                                                const uint64_t* __restrict__ row_ptr,
                                                                uint32_t* __restrict__ ids, uint64_t ids_cap,
                                                                uint64_t pieces_cap, MatchStats* stats) {
  __shared__ uint32_t s_scan[COMPACT_WAVES][64];
  __shared__ uint64_t s_src[COMPACT_WAVES][64];
  __shared__ uint64_t s_dst[COMPACT_WAVES][64];
  if (!compact_checks(row_ptr, n, ids_cap, stats)) return;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t np = min((uint64_t)stats->pieces, pieces_cap);
  if (np == 0) return;
  const uint64_t nwin = (np + 63) / 64, nw = (uint64_t)gridDim.x * COMPACT_WAVES;
  const uint64_t per = (nwin + nw - 1) / nw, me = (uint64_t)blockIdx.x * COMPACT_WAVES + wave;
  const uint64_t wend = min(nwin, (me + 1) * per) * 64;
  uint64_t w0 = me * per * 64;
  uint4 pc = pieces[min(w0 + lane, np - 1)];   // unconditional (a load under a branch is waited for at once)
  for (; w0 < wend; w0 += 64) {
    const uint64_t i = w0 + lane;
    const uint32_t c = i < np ? pc.y : 0u;
    const uint64_t rp = row_ptr[c ? pc.x : 0u];
    uint32_t tot;
    const uint32_t ex = wave_excl_scan(c, lane, &tot);
    s_scan[wave][lane] = ex;
    s_src[wave][lane] = pc.z;
    s_dst[wave][lane] = rp + pc.w;
    wave_sync();
    pc = pieces[min(i + 64, np - 1)];   // the next window's piece, in flight during the copy
    copy_runs(ids_tmp, ids, s_scan[wave], s_src[wave], s_dst[wave], tot, lane);
    wave_sync();
  }
}

// Flush records -> CSR rows (round 5): one wave per chunk (a grid stride).
// Lane j takes the chunk's j-th topic: its row (the walk position in
// walk-order rows, else the input topic from the sorted record) and that row's
// start from the scan.  The chunk's records come from its directory (the
// walk's record offsets, REC_DIR of them; a longer chunk continues along the
// chain).  Each record is placed by scanning its 64 counts into the topics'
// slots and storing every id at row start + the topic's running offset (its
// owner found by a 6-step LDS search).  In walk-order rows a chunk's rows are
// one contiguous run (and topic[k] is written here); in input order each
// topic's piece of a record goes to a scattered row.  Chunks walked by k_heavy
// are skipped (their ids arrive as pieces, k_compact).
//
// k_rec_rows (A/B, EGM_REC_ROWS=0) places one record at a time with the next
// one's loads in flight; k_rec_burst (the default) loads REC_BURST records at
// once.  Measured at C2 (r5, rocprof): 1.93 / 1.65 ms.  Two forms that
// assemble the chunk in LDS first and store whole lines were slower: a 16 KB
// LDS window per wave (4.2 ms: 9 waves per CU, a round trip per record) and
// an in-order gather through an LDS table of the chunk's records (1.52 ms +
// 0.37 ms for chunks of more than 16 records).  Stores of records as one
// contiguous run (measurement only) take 0.93 ms and no stores 0.46 ms: the
// runs of ~5 ids per topic and record are what costs.
constexpr int REC_WAVES = 4;
constexpr uint32_t REC_IPL = (WALK_STAGE_MAX + 63) / 64;   // a record's ids, all loaded in one round
struct RecLoad {
  uint64_t off;
  uint32_t hdr, cr;
  uint32_t v[REC_IPL];
};
__global__ __launch_bounds__(64 * REC_WAVES) void k_rec_rows(const uint32_t* __restrict__ rec, uint64_t rec_cap,
                                                             const uint4* __restrict__ chunks,
                                                             const uint32_t* __restrict__ dir,
                                                             const uint64_t* __restrict__ order, uint32_t n,
                                                             const uint64_t* __restrict__ row_ptr,
                                                             uint32_t* __restrict__ topic, uint32_t* __restrict__ ids,
                                                             uint64_t ids_cap, MatchStats* stats, uint32_t ct) {
  __shared__ uint32_t s_ex[REC_WAVES][64];
  __shared__ uint64_t s_dst[REC_WAVES][64];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool ok = compact_checks(row_ptr, n, ids_cap, stats);
  const uint32_t nchunks = (n + ct - 1) / ct;
  // every load of one record (out of the slab: header 0, which fails the tag check)
  auto issue = [&](uint64_t o, RecLoad& L) {
    const bool in = o + REC_IDS <= rec_cap;
    const uint64_t oc = in ? o : 0ull;
    L.off = o;
    L.hdr = in ? rec[oc] : 0u;
    L.cr = ((const uint16_t*)(rec + oc + REC_HDR))[lane];
#pragma unroll
    for (uint32_t k = 0; k < REC_IPL; ++k) L.v[k] = rec[min(oc + REC_IDS + lane + 64u * k, rec_cap - 1)];
  };
  for (uint32_t c = blockIdx.x * REC_WAVES + wave; c < nchunks; c += gridDim.x * REC_WAVES) {
    const uint32_t t = c * ct + lane;
    const bool act = lane < ct && t < n;
    const uint32_t my_t = act ? (order ? (uint32_t)order[t] : t) : 0u;
    if (topic && act) topic[t] = my_t;   // written even when the rows are not (overflow): the map is the order
    const uint4 ch = chunks[c];
    if (!ok || !(ch.w & CHUNK_WALKED) || ch.z == 0) continue;
    const uint32_t nrec = ch.z;
    uint64_t dst = act ? row_ptr[topic ? t : my_t] : 0ull;
    const uint32_t roff = lane < min(nrec, REC_DIR) ? dir[(uint64_t)c * REC_DIR + lane] : 0u;
    RecLoad A, B;
    issue((uint64_t)ch.x | ((uint64_t)ch.y << 32), A);
    for (uint32_t r = 0; r < nrec; ++r) {
      const bool next_dir = r + 1 < nrec && r + 1 < REC_DIR;
      if (next_dir) issue((uint64_t)(uint32_t)__shfl((int)roff, (int)(r + 1), 64) << 2, B);   // in flight now
      uint32_t tot;
      const uint32_t ex = wave_excl_scan(A.cr, lane, &tot);
      if ((A.hdr & 0xFFFF0000u) != REC_TAG || (A.hdr & 0xFFFFu) != tot || tot > WALK_STAGE_MAX) {
        if (lane == 0) atomicOr(&stats->guard, GUARD_STACK);   // a broken directory or chain: a bug, reported
        break;
      }
      s_ex[wave][lane] = ex;
      s_dst[wave][lane] = dst;
      dst += A.cr;
      wave_sync();
#ifdef EGM_AB_REC_STORE   // measurement only: 0 = no id stores
#pragma unroll
      for (uint32_t k = 0; k < REC_IPL; ++k)
        if (A.v[k] == 0x7FFFFFF1u) ids[0] = A.v[k];
#else
#pragma unroll
      for (uint32_t k = 0; k < REC_IPL; ++k) {
        const uint32_t q = lane + 64u * k;
        if (q < tot) {
          uint32_t o = 0;
#pragma unroll
          for (uint32_t step = 32; step >= 1; step >>= 1)
            if (s_ex[wave][o + step] <= q) o += step;
          ids[s_dst[wave][o] + (q - s_ex[wave][o])] = A.v[k];
        }
      }
#endif
      wave_sync();
      if (r + 1 < nrec && !next_dir) {   // past the directory: the chain (rare: a chunk of > REC_DIR records)
        uint64_t o = A.off + rec_size(tot);
        if (o + REC_HDR <= rec_cap && (rec[o] & 0xFFFF0000u) == REC_JUMP)   // wave-uniform
          o = (uint64_t)rec[o + 2] | ((uint64_t)rec[o + 3] << 32);
        issue(o, B);
      }
      A = B;
    }
  }
}

// The burst form of k_rec_rows (round 5): the chunk's records are loaded
// REC_BURST at a time from the directory, all in one round, then placed one
// after the other — so a chunk's output lines are written within a short
// burst and are completed in L2 instead of being evicted half written (the
// direct form keeps each chunk open for ~11 dependent rounds: 4.1 GB written
// per C2 batch for 1.99 GB of ids, PMC r5g).
#ifndef EGM_REC_BURST
#define EGM_REC_BURST 7   // a C2 chunk's ids come in ~7 records of 480 (burst 8 at 8 ids per lane spills 44 B)
#endif
#ifndef EGM_REC_BITMAP
#define EGM_REC_BITMAP 1   // ids placed through a bitmap of run starts (A/B: 0, the LDS search)
#endif
#ifndef EGM_REC_WPE
#define EGM_REC_WPE 4      // waves per SIMD k_rec_burst is compiled for (caps its VGPRs at 128)
#endif
constexpr uint32_t REC_BURST = EGM_REC_BURST;
__global__ __launch_bounds__(64 * REC_WAVES) __attribute__((amdgpu_waves_per_eu(EGM_REC_WPE))) void k_rec_burst(const uint32_t* __restrict__ rec, uint64_t rec_cap,
                                                              const uint4* __restrict__ chunks,
                                                              const uint32_t* __restrict__ dir,
                                                              const uint64_t* __restrict__ order, uint32_t n,
                                                              const uint64_t* __restrict__ row_ptr,
                                                              uint32_t* __restrict__ topic, uint32_t* __restrict__ ids,
                                                              uint64_t ids_cap, MatchStats* stats, uint32_t ct) {
#if EGM_REC_BITMAP
  __shared__ uint64_t s_bm[REC_WAVES][REC_IPL];   // the record's run starts (bit q: an id position where a topic's run begins)
  __shared__ uint64_t s_dst[REC_WAVES][64];       // the r-th run: its topic's next id in HBM minus the run's start
#else
  __shared__ uint32_t s_ex[REC_WAVES][64];
  __shared__ uint64_t s_dst[REC_WAVES][64];
#endif
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool ok = compact_checks(row_ptr, n, ids_cap, stats);
#if EGM_REC_BITMAP
  if (lane < REC_IPL) s_bm[wave][lane] = 0ull;
  wave_sync();
  const uint64_t lmask = (2ull << lane) - 1ull;   // positions <= lane of a 64-position word (lane 63: all)
#endif
  const uint32_t nchunks = (n + ct - 1) / ct;
  for (uint32_t c = blockIdx.x * REC_WAVES + wave; c < nchunks; c += gridDim.x * REC_WAVES) {
    const uint32_t t = c * ct + lane;
    const bool act = lane < ct && t < n;
    const uint32_t my_t = act ? (order ? (uint32_t)order[t] : t) : 0u;
    if (topic && act) topic[t] = my_t;   // written even when the rows are not (overflow): the map is the order
    const uint4 ch = chunks[c];
    const uint32_t nrec = ch.z;
    if (!ok || !(ch.w & CHUNK_WALKED) || nrec == 0) continue;
    uint64_t dst = act ? row_ptr[topic ? t : my_t] : 0ull;
    const uint32_t roff = lane < min(nrec, REC_DIR) ? dir[(uint64_t)c * REC_DIR + lane] : 0u;
    uint64_t chain = 0;   // past the directory: the next record along the chain
    bool broken = false;
    for (uint32_t r0 = 0; r0 < nrec && !broken; r0 += REC_BURST) {
      const uint32_t nb = min(REC_BURST, nrec - r0);
      uint32_t hdr[REC_BURST], cr[REC_BURST], v[REC_BURST][REC_IPL];
      uint64_t off[REC_BURST];
      const bool from_dir = r0 + nb <= REC_DIR;   // wave-uniform
      // every slot's loads issued unconditionally (a slot past the burst re-reads its
      // first record): a load under a branch is waited for at the branch's end
#pragma unroll
      for (uint32_t b = 0; b < REC_BURST; ++b) {
        // the record's offset and header are wave-uniform: scalar registers and a scalar load
        const uint32_t rb = from_dir ? r0 + (b < nb ? b : 0u) : 0u;
        const uint64_t o = (uint64_t)uni((uint32_t)__shfl((int)roff, (int)min(rb, REC_DIR - 1), 64)) << 2;
        const bool in = o + REC_IDS <= rec_cap;
        const uint64_t oc = in ? o : 0ull;
        off[b] = o;
        hdr[b] = in ? uni(rec[oc]) : 0u;
        cr[b] = ((const uint16_t*)(rec + oc + REC_HDR))[lane];
#pragma unroll
        for (uint32_t k = 0; k < REC_IPL; ++k) v[b][k] = rec[min(oc + REC_IDS + lane + 64u * k, rec_cap - 1)];
      }
#pragma unroll
      for (uint32_t b = 0; b < REC_BURST; ++b) {
        if (b >= nb) break;
        if (!from_dir) {   // (rare: a chunk of more than REC_DIR records) one record at a time along the chain
          uint64_t o = r0 + b < REC_DIR ? ((uint64_t)(uint32_t)__shfl((int)roff, (int)(r0 + b), 64) << 2) : chain;
          if (o + REC_HDR <= rec_cap && (rec[o] & 0xFFFF0000u) == REC_JUMP)   // wave-uniform
            o = (uint64_t)rec[o + 2] | ((uint64_t)rec[o + 3] << 32);
          const bool in = o + REC_IDS <= rec_cap;
          const uint64_t oc = in ? o : 0ull;
          off[b] = o;
          hdr[b] = in ? rec[oc] : 0u;
          cr[b] = ((const uint16_t*)(rec + oc + REC_HDR))[lane];
#pragma unroll
          for (uint32_t k = 0; k < REC_IPL; ++k) v[b][k] = rec[min(oc + REC_IDS + lane + 64u * k, rec_cap - 1)];
        }
        uint32_t tot;
        const uint32_t ex = wave_excl_scan(cr[b], lane, &tot);
        if ((hdr[b] & 0xFFFF0000u) != REC_TAG || (hdr[b] & 0xFFFFu) != tot || tot > WALK_STAGE_MAX) {
          if (lane == 0) atomicOr(&stats->guard, GUARD_STACK);   // a broken directory or chain: a bug, reported
          broken = true;
          break;
        }
        chain = off[b] + rec_size(tot);
#if EGM_REC_BITMAP
        // round 6: each non-empty topic marks where its run starts; an id's run
        // is then the count of starts at or before it (popcounts of the bitmap)
        // instead of a 6-step LDS search per id (k_rec_burst's VALU: 407M per C2 batch)
        {
          const bool ne = cr[b] != 0;
          const uint64_t bal = __ballot(ne);
          if (ne) {
            s_dst[wave][mbcnt(bal)] = dst - ex;   // mod 2^64: id q of the run goes to (dst - ex) + q
            atomicOr((unsigned long long*)&s_bm[wave][ex >> 6], 1ull << (ex & 63u));
          }
          dst += cr[b];
          wave_sync();
          uint64_t wk[REC_IPL];
#pragma unroll
          for (uint32_t k = 0; k < REC_IPL; ++k) wk[k] = uni64(s_bm[wave][k]);
          if (lane < REC_IPL) s_bm[wave][lane] = 0ull;   // for the next record (a wave's LDS operations stay in order)
          uint32_t pre = 0;
#pragma unroll
          for (uint32_t k = 0; k < REC_IPL; ++k) {
            const uint32_t q = lane + 64u * k;
            const uint32_t r = pre + popc(wk[k] & lmask);   // runs that start at or before q (>= 1 below tot)
            pre += popc(wk[k]);
            if (q < tot) ids[s_dst[wave][r - 1] + q] = v[b][k];
          }
          wave_sync();
        }
#else
        s_ex[wave][lane] = ex;
        s_dst[wave][lane] = dst;
        dst += cr[b];
        wave_sync();
#pragma unroll
        for (uint32_t k = 0; k < REC_IPL; ++k) {
          const uint32_t q = lane + 64u * k;
          if (q < tot) {
            uint32_t o = 0;
#pragma unroll
            for (uint32_t step = 32; step >= 1; step >>= 1)
              if (s_ex[wave][o + step] <= q) o += step;
            ids[s_dst[wave][o] + (q - s_ex[wave][o])] = v[b][k];
          }
        }
        wave_sync();
#endif
      }
    }
  }
}

// ------------------------------------------------------------- launchers ----
// One wave per block; a grid stride over the chunks beyond 32 waves per CU.
int walk_grid_blocks(uint32_t n) {
  const uint32_t ct = walk_chunk_topics(n), chunks = (n + ct - 1) / ct;
  uint32_t blocks = chunks < 256u * 32u ? chunks : 256u * 32u;
  blocks = (blocks + 7) & ~7u;   // a multiple of the 8 XCDs
  return blocks ? (int)blocks : 1;
}

// The deep pass: a grid stride over the chunks handed to it, exactly as many
// waves as are resident together (its LDS stack sets that: 16 per CU at 504
// 12-B items, 14 at round 5's 448 16-B items).  A wave that does not fit would start only when another ends, with
// a whole share of chunks still to walk: C3 measured 59 ms at 10 waves per CU
// and 640 items, 80 ms when an 11th was asked for, 53 ms at 14 waves of 448
// items (r5 A/B).  EGM_DEEP_WAVES forces a count (A/B).
#ifndef EGM_DEEP_WAVES
#define EGM_DEEP_WAVES 0   // 0: the occupancy the runtime reports for k_walk<true>
#endif
// The runtime's figure is capped by what the LDS holds at a 1280-B allocation
// granule (160 KB / 128): round 6 measured the deep pass with waves of 11 600 B
// (the runtime said 14 per CU, 12 fit) at 65.6 ms against 48.8 ms at 11 344 B
// (14 fit), and 10 320 B (said 15, 14 fit) at 63.3 ms — the waves that did not
// fit ran as a tail (gpurun_out r6am, r6an).
constexpr int LDS_PER_CU = 160 * 1024;
constexpr int LDS_GRANULE = 1280;
static uint32_t deep_waves_per_cu() {
  static const uint32_t v = [] {
    int nb = EGM_DEEP_WAVES;
    if (nb <= 0 &&
        (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_walk<true>, 64, 0) != hipSuccess || nb <= 0))
      nb = 8;
    hipFuncAttributes fa;
    if (EGM_DEEP_WAVES <= 0 && hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_walk<true>)) == hipSuccess &&
        fa.sharedSizeBytes > 0) {
      const int per = (int)((fa.sharedSizeBytes + LDS_GRANULE - 1) / LDS_GRANULE) * LDS_GRANULE;
      nb = std::max(1, std::min(nb, LDS_PER_CU / per));
    }
    return (uint32_t)std::min(nb, 32);
  }();
  return v;
}

int deep_grid_blocks(uint32_t n) {
  const uint32_t ct = walk_chunk_topics(n), chunks = (n + ct - 1) / ct;
  const uint32_t per = 256u * deep_waves_per_cu();
  uint32_t blocks = chunks < per ? chunks : per;
  blocks = (blocks + 7) & ~7u;
  return blocks ? (int)blocks : 1;
}

uint32_t heavy_stack_items(uint64_t max_levels) { return (uint32_t)(max_levels + 256); }

uint32_t walk_stage() { return WALK_STAGE_MAX; }
uint32_t walk_stage_min() { return WALK_STAGE_MIN; }

size_t scan_tiles(uint32_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

static void scan_counts(const uint32_t* cnt, uint32_t n, uint64_t* tile_sums, uint64_t* row_ptr,
                        hipStream_t s, uint64_t* copy = nullptr) {
  if (n <= SCAN_SMALL) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, s, cnt, n, row_ptr, copy);
    return;
  }
  const uint32_t ntiles = (uint32_t)scan_tiles(n);
  if (ntiles) hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(256), 0, s, cnt, n, tile_sums);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, tile_sums, ntiles);
  hipLaunchKernelGGL(k_scan_apply, dim3(ntiles ? ntiles : 1), dim3(256), 0, s, cnt, n, tile_sums, ntiles, row_ptr,
                     copy);
}

// EGM_TRACE_KERNELS=1: synchronise after every kernel of a batch and name it
// on stderr (diagnostics: which kernel of a batch does not return).
static bool trace_kernels() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("EGM_TRACE_KERNELS");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}
static void trace(hipStream_t s, const char* what) {
  if (!trace_kernels()) return;
  fprintf(stderr, "[egm] %s ...", what);
  const hipError_t e = hipStreamSynchronize(s);
  fprintf(stderr, " %s\n", hipGetErrorString(e));
}

uint32_t walk_key_bits(uint32_t shape) {
  uint32_t b = 0;
  for (uint32_t l = 0; l < KEY_LEVELS; ++l) b += (shape >> (4 * l)) & 0xFu;
  return b;
}

// ------------------------------------------------------- walk-order sort ----
// LSD radix sort of the batch's (32-bit key, 8-B record) pairs by the key's
// `kbits` high bits, 8 bits per pass, hand-written for gfx950 (round 6; rounds
// 2-5 called hipCUB's onesweep).  The order only buys the walk locality — the
// reference's results are order-free sets (apps/emqx/test/emqx_trie_SUITE.erl:
// 82,101,118) — but the sort is stable and deterministic, so a batch always
// walks in the same order.
//
//   k_sort_hist   one read of the keys: every pass's 256-bin histogram (LDS
//                 counts, one global add per bin and block); also zeroes the
//                 passes' look-back words.
//   k_sort_pass   per pass, one kernel: a block takes a ticket (its tile of
//                 SORT_TILE pairs, in dispatch order), ranks its pairs by digit
//                 with wave ballots (8 per row of 64: the lanes holding the same
//                 digit; stable: rows in input order, waves in input order),
//                 publishes its per-digit totals and finds each digit's global
//                 start by a decoupled look-back over the preceding tiles'
//                 words {flag:2 | count:30} (agent-scope loads and stores: the
//                 tiles run on all eight XCDs), then places the pairs sorted in
//                 LDS and writes each digit's run contiguously.
// Bytes per pair and pass: 12 read + 12 written (the last pass writes only the
// records), + 4 read once for the histograms.
constexpr int SORT_THREADS = 256;
#ifndef EGM_SORT_ITEMS
#define EGM_SORT_ITEMS 15                                       // pairs per thread: 3840 per tile, 51 KB LDS -> 3 blocks/CU
#endif
#ifndef EGM_SORT_TICKET
#define EGM_SORT_TICKET 1                                       // 0 (A/B): tile = blockIdx (in-order dispatch assumed)
#endif
constexpr int SORT_ITEMS = EGM_SORT_ITEMS;
constexpr uint32_t SORT_TILE = SORT_THREADS * SORT_ITEMS;
constexpr uint32_t SORT_MAX_PASSES = 4;
constexpr uint32_t SORT_HIST_BLOCKS = 1024;
constexpr uint32_t SORT_AGG = 1u << 30, SORT_PFX = 2u << 30, SORT_CNT = SORT_AGG - 1u;
constexpr size_t SORT_HEAD = 8192;                              // tickets[4] + hist[4][256], rounded
constexpr uint32_t SORT_SPIN_LIMIT = 1u << 20;                  // look-back polls before a guard trip
#ifndef EGM_SORT_LB
#define EGM_SORT_LB 8                                           // look-back words in flight per digit
#endif
constexpr int SORT_LB = EGM_SORT_LB;

static inline uint32_t sort_passes(uint32_t kbits) { return (kbits + 7) / 8; }
static inline uint32_t sort_tiles(uint32_t n) { return (n + SORT_TILE - 1) / SORT_TILE; }
static inline size_t sort_vals_bytes(uint32_t n) { return ((size_t)n * 8 + 255) & ~(size_t)255; }

size_t walk_sort_temp_bytes(uint32_t n, uint32_t shape) {
  const uint32_t kbits = min(walk_key_bits(shape), 32u);
  if (!kbits) return 0;
  return SORT_HEAD + sort_vals_bytes(n) + (size_t)sort_passes(kbits) * sort_tiles(n) * 256 * 4;
}

__global__ __launch_bounds__(256) void k_sort_hist(const uint32_t* __restrict__ key, uint32_t n, uint32_t begin,
                                                  uint32_t npass, uint32_t* __restrict__ hist,
                                                  uint32_t* __restrict__ status, uint64_t status_words) {
  // one copy of the histograms per wave: LDS atomics of one wave only contend
  // with each other (the walk key's top digit is Zipf-skewed)
  __shared__ uint32_t h[4][SORT_MAX_PASSES * 256];
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  for (uint32_t i = tid; i < 4 * SORT_MAX_PASSES * 256; i += 256) (&h[0][0])[i] = 0;
  const uint64_t g0 = (uint64_t)blockIdx.x * 256 + tid, gs = (uint64_t)gridDim.x * 256;
  for (uint64_t i = g0; i < status_words; i += gs) status[i] = 0;
  __syncthreads();
  uint32_t* hw = h[wv];
  auto count = [&](uint32_t k) {
    for (uint32_t p = 0; p < npass; ++p) atomicAdd(&hw[p * 256 + ((k >> (begin + 8 * p)) & 0xFFu)], 1u);
  };
  const uint32_t n4 = n / 4;
  constexpr int HU = 8;   // loads in flight per thread (the loop is latency-bound otherwise)
  for (uint64_t i0 = g0; i0 < n4; i0 += gs * HU) {
    uint4 k[HU];
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const uint64_t i = i0 + gs * u;
      k[u] = ((const uint4*)key)[i < n4 ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      if (i0 + gs * u >= n4) break;
      count(k[u].x);
      count(k[u].y);
      count(k[u].z);
      count(k[u].w);
    }
  }
  for (uint64_t i = (uint64_t)n4 * 4 + g0; i < n; i += gs) count(key[i]);
  __syncthreads();
  for (uint32_t i = tid; i < npass * 256; i += 256) {
    const uint32_t c = h[0][i] + h[1][i] + h[2][i] + h[3][i];
    if (c) atomicAdd(&hist[i], c);
  }
}

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t tid, uint32_t* s_wsum) {
  uint32_t wt;
  uint32_t x = wave_excl_scan(v, tid & 63, &wt);
  __syncthreads();
  if ((tid & 63) == 0) s_wsum[tid >> 6] = wt;
  __syncthreads();
#pragma unroll
  for (uint32_t w = 0; w < SORT_THREADS / 64; ++w)
    if (w < (tid >> 6)) x += s_wsum[w];
  return x;
}

__global__ __launch_bounds__(SORT_THREADS) void k_sort_pass(const uint32_t* __restrict__ kin,
                                                           const uint64_t* __restrict__ vin,
                                                           uint32_t* __restrict__ kout, uint64_t* __restrict__ vout,
                                                           uint32_t n, uint32_t shift,
                                                           const uint32_t* __restrict__ hist, uint32_t* status,
                                                           uint32_t* ticket, MatchStats* stats) {
  __shared__ uint32_t s_key[SORT_TILE];
  __shared__ uint64_t s_val[SORT_TILE];
  __shared__ uint32_t s_cnt[SORT_THREADS / 64][256];   // per-wave digit counts, then each wave's offset
  __shared__ uint32_t s_start[256];                    // the digit's first slot in the sorted tile
  __shared__ uint32_t s_base[256];                     // the digit's first output position of this tile
  __shared__ uint32_t s_wsum[SORT_THREADS / 64];
  __shared__ uint32_t s_tile;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#if EGM_SORT_TICKET
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
#else
  if (tid == 0) s_tile = blockIdx.x;
#endif
  for (uint32_t i = tid; i < (SORT_THREADS / 64) * 256; i += SORT_THREADS) (&s_cnt[0][0])[i] = 0;
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t base = (uint64_t)tile * SORT_TILE;
  // rows of 64 pairs, wave-striped: pair (wave, i, lane) is input pair base + (wave * ITEMS + i) * 64 + lane
  const uint64_t wbase = base + (uint64_t)wv * 64 * SORT_ITEMS + lane;
  uint32_t k[SORT_ITEMS], r[SORT_ITEMS];
  uint64_t v[SORT_ITEMS];
#pragma unroll
  for (int i = 0; i < SORT_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * 64;
    const bool ok = idx < n;
    k[i] = ok ? kin[idx] : 0u;
    v[i] = ok ? vin[idx] : 0ull;
  }
  // stable ranks: row by row, a row's lanes of one digit found with 8 ballots
#pragma unroll
  for (int i = 0; i < SORT_ITEMS; ++i) {
    const bool ok = wbase + (uint64_t)i * 64 < n;
    const uint32_t d = (k[i] >> shift) & 0xFFu;
    uint64_t m = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t below = mbcnt(m);
    const uint32_t c = s_cnt[wv][d];
    r[i] = c + below;
    if (ok && below == 0) s_cnt[wv][d] = c + popc(m);   // the row's lowest lane of the digit adds its count
  }
  __syncthreads();
  const uint32_t d = tid;   // one digit per thread from here
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < SORT_THREADS / 64; ++w) {
    const uint32_t c = s_cnt[w][d];
    s_cnt[w][d] = tot;
    tot += c;
  }
  uint32_t* my = status + (uint64_t)tile * 256 + d;
  uint32_t excl = 0;
  if (tile == 0) {
    excl = block_excl_scan256(hist[d], tid, s_wsum);   // the digit's first position in the whole output
  } else {
    __hip_atomic_store(my, SORT_AGG | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // windowed look-back: SORT_LB predecessors' words in flight at once, summed
    // nearest first up to the first inclusive prefix (tile 0 always publishes
    // one); a word not yet published ends the window and is polled again
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    for (;;) {
      uint32_t x[SORT_LB];
#pragma unroll
      for (int q = 0; q < SORT_LB; ++q) {
        const int64_t jj = j - q;
        x[q] = __hip_atomic_load(status + (uint64_t)(jj > 0 ? jj : 0) * 256 + d, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
      uint32_t used = 0;
      bool stop = false, done = false;
#pragma unroll
      for (int q = 0; q < SORT_LB; ++q) {
        const uint32_t f = x[q] & ~SORT_CNT;
        if (stop || f == 0) {
          stop = true;
          continue;
        }
        excl += x[q] & SORT_CNT;
        ++used;
        if (f == SORT_PFX) done = stop = true;
      }
      if (done) break;
      j -= used;
      if (!used && ++spins > SORT_SPIN_LIMIT) {   // a bug, reported (rows not assembled), never a hang
        atomicOr(&stats->guard, GUARD_LOOP);
        break;
      }
    }
  }
  __hip_atomic_store(my, SORT_PFX | ((excl + tot) & SORT_CNT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t start = block_excl_scan256(tot, tid, s_wsum);
  s_start[d] = start;
  s_base[d] = excl;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < SORT_ITEMS; ++i) {
    if (wbase + (uint64_t)i * 64 >= n) continue;
    const uint32_t dg = (k[i] >> shift) & 0xFFu;
    const uint32_t p = s_start[dg] + s_cnt[wv][dg] + r[i];
    s_key[p] = k[i];
    s_val[p] = v[i];
  }
  __syncthreads();
  const uint32_t nt = (uint32_t)min<uint64_t>(SORT_TILE, n - base);
  for (uint32_t j = tid; j < nt; j += SORT_THREADS) {
    const uint32_t kk = s_key[j];
    const uint32_t dg = (kk >> shift) & 0xFFu;
#if defined(EGM_SORT_AB) && EGM_SORT_AB == 2   // measurement only: every tile's output contiguous (not a sort)
    const uint64_t dst = base + j + (dg & 0u);
#else
    const uint64_t dst = (uint64_t)s_base[dg] + (j - s_start[dg]);
#endif
#if defined(EGM_SORT_AB) && EGM_SORT_AB == 1   // measurement only: no output stores
    if (kk == 0x7FFFFFF1u && s_val[j] == 0x7FFFFFF1ull) vout[0] = dst;
#else
    if (kout) kout[dst] = kk;
    vout[dst] = s_val[j];
#endif
  }
}

// Sort (skey, sval) by the key's kbits high bits into w.order (records only).
static hipError_t walk_sort(const MatchWork& w, uint32_t n, uint32_t kbits, hipStream_t s) {
  const uint32_t begin = 32 - kbits, npass = sort_passes(kbits), tiles = sort_tiles(n);
  uint8_t* tmp = (uint8_t*)w.sort_tmp;
  uint32_t* tickets = (uint32_t*)tmp;
  uint32_t* hist = tickets + SORT_MAX_PASSES;
  uint64_t* vtmp = (uint64_t*)(tmp + SORT_HEAD);
  uint32_t* status = (uint32_t*)(tmp + SORT_HEAD + sort_vals_bytes(n));
  hipError_t e = hipMemsetAsync(tmp, 0, (SORT_MAX_PASSES + SORT_MAX_PASSES * 256) * 4, s);
  if (e != hipSuccess) return e;
  const uint64_t status_words = (uint64_t)npass * tiles * 256;
  const uint32_t hb = (uint32_t)std::min<uint64_t>(SORT_HIST_BLOCKS, std::max<uint64_t>(1, ((uint64_t)n / 4 + 255) / 256));
  hipLaunchKernelGGL(k_sort_hist, dim3(hb), dim3(256), 0, s, w.skey, n, begin, npass, hist, status, status_words);
  for (uint32_t p = 0; p < npass; ++p) {
    const bool last = p + 1 == npass;
    const uint32_t* kin = (p & 1) ? w.skey_out : w.skey;
    uint32_t* kout = last ? nullptr : ((p & 1) ? w.skey : w.skey_out);
    const uint64_t* vin = (p == 0 || !(p & 1)) ? w.sval : vtmp;
    uint64_t* vout = last ? w.order : ((p & 1) ? w.sval : vtmp);
    hipLaunchKernelGGL(k_sort_pass, dim3(tiles), dim3(SORT_THREADS), 0, s, kin, vin, kout, vout, n, begin + 8 * p,
                       hist + 256 * p, status + (uint64_t)p * tiles * 256, tickets + p, w.stats);
  }
  return hipGetLastError();
}

// Test hook (egm_debug_walk_sort): the walk sort alone over caller-given pairs.
// keys/vals are overwritten (scratch); tmp holds walk_sort_temp_bytes.
hipError_t launch_walk_sort(uint32_t* keys, uint32_t* keys_tmp, uint64_t* vals, uint64_t* out, void* tmp,
                            MatchStats* stats, uint32_t n, uint32_t kbits, hipStream_t s) {
  if (!n || !kbits || kbits > 32) return hipErrorInvalidValue;
  MatchWork w{};
  w.skey = keys;
  w.skey_out = keys_tmp;
  w.sval = vals;
  w.order = out;
  w.sort_tmp = tmp;
  w.stats = stats;
  return walk_sort(w, n, kbits, s);
}

constexpr uint32_t SORT_MIN_TOPICS = 16384;   // below this the sort's fixed cost outweighs the locality

hipError_t launch_match(const DevTable& tab, const uint8_t* blob, const uint32_t* off, uint32_t n,
                        int mode, const MatchWork& w_in, const MatchOut& out, hipStream_t s,
                        hipEvent_t* ev_walk, bool* walk_sorted) {
  if (walk_sorted) *walk_sorted = false;
  hipError_t e = hipMemsetAsync(w_in.stats, 0, sizeof(MatchStats), s);
  if (e != hipSuccess) return e;
  if (n == 0) {
    return hipMemsetAsync(out.row_ptr, 0, sizeof(uint64_t), s);
  }
  MatchWork w = w_in;
  w.walk_rows = out.topic != nullptr;
  w.ct = walk_chunk_topics(n);
  const uint32_t kbits = min(walk_key_bits(w.key_shape), 32u);
  // (fixed-stride word offsets t * FIX_WORDS stay 32-bit below 2^29 topics)
  const bool sorted = kbits && w.order && n >= SORT_MIN_TOPICS && n < (1u << 29) && !(w.debug & DEBUG_INPUT_ORDER);
  size_t tb = 0;
  if (sorted) {
    tb = walk_sort_temp_bytes(n, w.key_shape);
    if (tb > w.sort_tmp_bytes) return hipErrorInvalidValue;   // a host sizing bug: never sort into too little scratch
  }
  WalkOrderOut wo{};
  if (sorted) wo = WalkOrderOut{w.skey, w.sval, w.wfix, w.key_shape, nullptr};
  wo.n_live = w.n_live;
  hipLaunchKernelGGL(k_tokenise, dim3((n + TOK_BLOCK - 1) / TOK_BLOCK), dim3(TOK_BLOCK), 0, s, tab, blob,
                     off, n, w.wid, w.lv, w.tfl, wo);
  trace(s, "k_tokenise");
  if (sorted) {
    e = walk_sort(w, n, kbits, s);
    if (e != hipSuccess) return e;
    if (walk_sorted) *walk_sorted = true;
    trace(s, "walk order sort");
  } else {
    w.order = nullptr;
  }
  if (ev_walk) hipEventRecord(ev_walk[0], s);
  hipLaunchKernelGGL(k_walk<false>, dim3(walk_grid_blocks(n)), dim3(64), 0, s, tab, off, n, mode, w);
  trace(s, "k_walk");
  // the chunks of more than DEEP_MIN levels (their count is on the device: a
  // small grid that exits at once when there are none)
  hipLaunchKernelGGL(k_walk<true>, dim3(deep_grid_blocks(n)), dim3(64), 0, s, tab, off, n, mode, w);
  if (ev_walk) hipEventRecord(ev_walk[1], s);
  trace(s, "k_walk<deep>");
  hipLaunchKernelGGL(k_heavy, dim3(w.heavy_waves), dim3(64), 0, s, tab, off, n, mode, w);
  trace(s, "k_heavy");
  scan_counts(w.cnt, n, w.tile_sums, out.row_ptr, s);
  trace(s, "scan");
  // shorter window ranges per wave keep more copies in flight; small batches
  // get a small grid (the piece count is only known on the device)
  const uint32_t cblocks =
      (uint32_t)std::min<uint64_t>(EGM_COMPACT_BLOCKS, std::max<uint64_t>(256, ((uint64_t)n + 63) / 64));
#ifndef EGM_REC_ROWS
#define EGM_REC_ROWS 1   // 1: k_rec_burst; 0: k_rec_rows (A/B)
#endif
  const uint32_t rblocks = (uint32_t)std::min<uint64_t>(
      65536, std::max<uint64_t>(1, (((uint64_t)n + w.ct - 1) / w.ct + REC_WAVES - 1) / REC_WAVES));
#if EGM_REC_ROWS
  hipLaunchKernelGGL(k_rec_burst, dim3(rblocks), dim3(64 * REC_WAVES), 0, s, w.rec, w.rec_cap, w.chunks, w.dir,
                     w.order, n, out.row_ptr, out.topic, out.ids, out.ids_cap, w.stats, w.ct);
#else   // A/B: one record at a time, the next in flight
  hipLaunchKernelGGL(k_rec_rows, dim3(rblocks), dim3(64 * REC_WAVES), 0, s, w.rec, w.rec_cap, w.chunks, w.dir,
                     w.order, n, out.row_ptr, out.topic, out.ids, out.ids_cap, w.stats, w.ct);
#endif
  trace(s, "k_rec_rows");
  hipLaunchKernelGGL(k_compact, dim3(cblocks), dim3(64 * COMPACT_WAVES), 0, s, w.pieces, w.ids_tmp, n, out.row_ptr,
                     out.ids, out.ids_cap, w.pieces_cap, w.stats);
  return hipGetLastError();
}

// --------------------------------------------------------------- fan-out ----
// emqx_broker:dispatch/2 (emqx_broker.erl:283-308): every subscriber of every
// matched filter, the {shard, Topic, I} bags flattened into the same list
// (:297-308, emqx_broker_helper.erl:82-86), shared groups as (filter, group)
// entries (emqx_broker.erl:246-247).  Flattened over match entries: count ->
// scan -> fill.  The fill is wave-cooperative: a wave takes a window of 64
// match entries, whose deliveries are contiguous in the output (the scan), and
// its lanes write them in order — coalesced stores, and a 2 000-subscriber
// filter is spread over 64 lanes instead of looping in one.
// One aligned 16-B record per filter (k_sub_pairs, at egm_subs_build):
//   y = subscriber count (24 bits, saturated) << 8 | row start bits 32-39
//   z, w = its first two subscriber ids (when it has them)
//   x = row start bits 0-31, or — a row of at most 3 — its third subscriber
// A matched id costs the count pass one line request, and — round 4 — the
// fill reads no subscriber row at all for a filter of up to three
// subscribers (C4: 92 % of filters; the record travels to the fill as the
// entry's 16-B dsrc): the fill's random row reads were a 64-B line per
// entry for ~14 B of subscribers.
#ifndef EGM_FAN_DS0
#define EGM_FAN_DS0 0   // 1: the count pass copies each entry's record to ds0 for the fill (A/B); 0: the fill re-reads it
#endif
constexpr uint32_t FAN_CNT_BITS = 24;
constexpr uint32_t FAN_CNT_SAT = (1u << FAN_CNT_BITS) - 1;   // saturated: the fill reads the exact count from row[]
constexpr uint32_t FAN_INLINE_ALL = 3;   // a row this short is carried whole in its record
__device__ __forceinline__ uint64_t rec_start(uint4 r) { return (uint64_t)r.x | ((uint64_t)(r.y & 0xFFu) << 32); }
__device__ __forceinline__ uint32_t rec_count(uint4 r) { return r.y >> 8; }

__global__ __launch_bounds__(256) void k_sub_pairs(const uint64_t* __restrict__ row, const uint32_t* __restrict__ subs,
                                                   uint32_t n_slots, uint4* __restrict__ rp) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  if (f < n_slots) {
    const uint64_t r0 = row[f], r1 = row[f + 1], c = r1 - r0;
    const uint32_t cs = (uint32_t)min(c, (uint64_t)FAN_CNT_SAT);
    const uint32_t x = c <= FAN_INLINE_ALL ? (c > 2 ? subs[r0 + 2] : 0u) : (uint32_t)r0;
    rp[f] = make_uint4(x, ((uint32_t)(r0 >> 32) & 0xFFu) | (cs << 8), c > 0 ? subs[r0] : 0u, c > 1 ? subs[r0 + 1] : 0u);
  }
}

// Round 4: the count kernel copies each match entry's
// filter record (above) to ds0 and writes one subscriber total per window
// of 64 entries; the window totals are scanned (nids/64 of them), and the
// fill derives each entry's delivery offset with a wave scan inside its
// window.  Round 3 wrote a count AND a start per entry and scanned all nids
// counts into u64 offsets before the fill read them back (~8.8 GB of
// intermediate traffic at C4, ~4.3 ms of scans).
__global__ __launch_bounds__(256) void k_fan_count(const uint32_t* __restrict__ mids, uint64_t nids,
                                                   SubTable st, uint32_t* __restrict__ wsum,
                                                   uint4* __restrict__ ds0) {
  constexpr uint32_t U = 4;   // windows per wave in flight
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nwin = (nids + 63) / 64;
  const uint64_t wstride = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t w0 = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w0 < nwin; w0 += wstride * U) {
    uint32_t f[U];
    uint4 r[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) f[u] = mids[min((w0 + u * wstride) * 64 + lane, nids - 1)];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) r[u] = st.rp[f[u] < st.n_fid_slots ? f[u] : 0u];   // unconditional
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t w = w0 + u * wstride, i = w * 64 + lane;
      const bool ok = i < nids && f[u] < st.n_fid_slots;
      const uint32_t cs = ok ? rec_count(r[u]) : 0u;
      const uint32_t c = cs == FAN_CNT_SAT ? (uint32_t)min(st.row[f[u] + 1] - st.row[f[u]], (uint64_t)0xFFFFFFFFu) : cs;
#if EGM_FAN_DS0
      if (i < nids) ds0[i] = ok ? r[u] : make_uint4(0, 0, 0, 0);
#endif
      uint32_t sum = c;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
      if (lane == 0 && w < nwin) wsum[w] = sum;
    }
  }
}

// The same count in walk order (round 4): a wave takes 64
// consecutive topics of the batch's walk order — topics that share their
// first levels, so their rows repeat the same matched filters — lays their
// rows out as one run (wave scan, owner found by a 6-step LDS search as in
// k_compact_fix) and reads each entry's subscriber record: the repeats are L2
// hits instead of random misses over the 1.6 GB record table.  Entries are
// written where they are (ds0 in input order); each window's total is
// accumulated with one atomic per run of lanes in the same window (a
// segmented wave sum), wsum zeroed beforehand.
constexpr int FAN_ORD_WAVES = 4;
__global__ __launch_bounds__(64 * FAN_ORD_WAVES) void k_fan_count_ord(const uint64_t* __restrict__ order, uint32_t n,
                                                                      const uint64_t* __restrict__ mrow,
                                                                      const uint32_t* __restrict__ mids, uint64_t nids,
                                                                      SubTable st, uint32_t* __restrict__ wsum,
                                                                      uint4* __restrict__ ds0) {
  constexpr uint32_t U = 4;   // entries per lane in flight
  __shared__ uint32_t s_ex[FAN_ORD_WAVES][64];
  __shared__ uint64_t s_r0[FAN_ORD_WAVES][64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t ngroups = (n + 63) / 64;
  for (uint32_t g = blockIdx.x * FAN_ORD_WAVES + wave; g < ngroups; g += gridDim.x * FAN_ORD_WAVES) {
    const uint32_t p = g * 64 + lane;
    uint64_t r0 = 0;
    uint32_t c = 0;
    if (p < n) {
      const uint32_t t = (uint32_t)order[p];
      if (t < n) {
        r0 = mrow[t];
        const uint64_t r1 = mrow[t + 1];
        c = (r1 > r0 && r1 <= nids) ? (uint32_t)(r1 - r0) : 0u;
      }
    }
    uint32_t tot;
    const uint32_t ex = wave_excl_scan(c, lane, &tot);
    s_ex[wave][lane] = ex;
    s_r0[wave][lane] = r0;
    wave_sync();
    for (uint32_t q0 = 0; q0 < tot; q0 += 64 * U) {
      uint64_t idx[U];
      uint32_t f[U];
      uint4 r[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t q = min(q0 + 64 * u + lane, tot - 1);
        uint32_t k = 0;
#pragma unroll
        for (uint32_t b = 32; b; b >>= 1)
          if (s_ex[wave][k + b] <= q) k += b;
        idx[u] = s_r0[wave][k] + (q - s_ex[wave][k]);
        f[u] = mids[idx[u]];
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) r[u] = st.rp[f[u] < st.n_fid_slots ? f[u] : 0u];   // unconditional
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const bool act = q0 + 64 * u + lane < tot;
        const bool ok = act && f[u] < st.n_fid_slots;
        const uint32_t cs = ok ? rec_count(r[u]) : 0u;
        const uint32_t cu =
            cs == FAN_CNT_SAT ? (uint32_t)min(st.row[f[u] + 1] - st.row[f[u]], (uint64_t)0xFFFFFFFFu) : cs;
        if (act) ds0[idx[u]] = ok ? r[u] : make_uint4(0, 0, 0, 0);
        // segmented sum over runs of lanes in one window (lanes of one row are consecutive entries)
        const uint32_t win = act ? (uint32_t)(idx[u] >> 6) : 0xFFFFFFFFu;
        const uint32_t prev = __shfl_up(win, 1, 64);
        const bool head = lane == 0 || prev != win;
        const uint64_t heads = __ballot(head);
        uint32_t incl = cu;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(incl, d, 64);
          if (lane >= (uint32_t)d) incl += y;
        }
        const uint32_t start = 63u - (uint32_t)__builtin_clzll(heads & (~0ull >> (63 - lane)));   // this run's first lane
        const uint32_t before = __shfl(incl, (int)(start ? start - 1 : 0), 64);
        const bool last = lane == 63 || ((heads >> (lane + 1)) & 1ull);
        const uint32_t run = incl - (start ? before : 0u);
        if (last && win != 0xFFFFFFFFu && run) atomicAdd(&wsum[win], run);
      }
    }
    wave_sync();
  }
}

hipError_t launch_sub_pairs(const uint64_t* row, const uint32_t* subs, uint32_t n_slots, uint4* rp, hipStream_t s) {
  if (n_slots) hipLaunchKernelGGL(k_sub_pairs, dim3((n_slots + 255) / 256), dim3(256), 0, s, row, subs, n_slots, rp);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_fan_rows(const uint64_t* __restrict__ mrow, uint32_t n,
                                                  const uint64_t* __restrict__ dpos, uint64_t* __restrict__ drow) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t <= n; t += gridDim.x * blockDim.x)
    drow[t] = dpos[mrow[t]];
}

constexpr int FAN_WAVES = 4;
constexpr uint32_t FAN_BIG = 128;   // entries with this many subscribers are copied by the whole wave

struct FanLds {   // one wave's window of 64 entries
  uint32_t pre[64], off[64], fid[64], cnt[64], in0[64], in1[64], in2[64];
  uint64_t src[64];
};

// The deliveries of one window of 64 match entries, whose deliveries are
// contiguous from `base`: small rows lane per delivery (the owning entry found
// by a 6-step LDS search; a row's first subscribers come with its record v,
// the rest from the subscriber table), big rows streamed by the whole wave.
// Only deliveries below `cap` are written.
__device__ __forceinline__ void fan_window(FanLds& L, const SubTable& st, uint32_t lane, uint32_t f, uint4 v,
                                           uint32_t c, uint32_t off, uint64_t base, uint32_t* __restrict__ dfid,
                                           uint32_t* __restrict__ dsub, uint64_t cap) {
  const bool big = c >= FAN_BIG;
  uint32_t tot_s;
  const uint32_t pre_s = wave_excl_scan(big ? 0u : c, lane, &tot_s);   // small entries, packed
  L.pre[lane] = pre_s;
  L.off[lane] = off;
  L.fid[lane] = f;
  L.cnt[lane] = c;
  L.src[lane] = rec_start(v);   // (meaningful only past FAN_INLINE_ALL subscribers)
  L.in0[lane] = v.z;
  L.in1[lane] = v.w;
  L.in2[lane] = v.x;
  wave_sync();
  for (uint32_t q = lane; q < tot_s; q += 64) {
    // the last k with pre[k] <= q (an entry with no small deliveries shares its
    // successor's pre, so the last one found has deliveries)
    uint32_t k = 0;
#pragma unroll
    for (uint32_t b = 32; b; b >>= 1)
      if (L.pre[k + b] <= q) k += b;
    const uint32_t o = q - L.pre[k];
    const uint64_t d = base + L.off[k] + o;
    if (d >= cap) continue;
    if (dfid) dfid[d] = L.fid[k];   // null: the compact form (the entry offsets give the filter)
    const uint32_t inl = L.cnt[k] <= FAN_INLINE_ALL ? FAN_INLINE_ALL : 2u;   // subscribers in the record
    uint32_t sub;
    if (o >= inl) sub = st.subs[L.src[k] + o];   // only these lanes read the table
    else sub = o == 0 ? L.in0[k] : (o == 1 ? L.in1[k] : L.in2[k]);
    dsub[d] = sub;
  }
  // big entries (C4: 2 000-subscriber filters): the wave streams the row, 4 per lane in flight
  for (uint64_t mb = __ballot(big); mb; mb &= mb - 1) {
    const uint32_t k = (uint32_t)__builtin_ctzll(mb);
    const uint32_t cnt = L.cnt[k], fk = L.fid[k];
    const uint64_t src = L.src[k], dst = base + L.off[k];
    for (uint32_t j0 = lane; j0 < cnt; j0 += 256) {
      uint32_t vv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) vv[r] = st.subs[src + min(j0 + 64u * r, cnt - 1)];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (j0 + 64u * r < cnt && dst + j0 + 64u * r < cap) {
          if (dfid) dfid[dst + j0 + 64u * r] = fk;
          dsub[dst + j0 + 64u * r] = vv[r];
        }
    }
  }
  wave_sync();
}

// The subscriber count of a matched entry from its record.
__device__ __forceinline__ uint32_t fan_count_of(const SubTable& st, uint32_t f, uint4 v) {
  const uint32_t c = rec_count(v);
  return c == FAN_CNT_SAT ? (uint32_t)min(st.row[f + 1] - st.row[f], (uint64_t)0xFFFFFFFFu) : c;   // rare: 2^24+
}

// One wave per window of 64 match entries; the entry offsets (dpos, the
// compact form's output and the rows' source) come from the window's scanned
// total plus a wave scan of the entries' counts.  The fill reads each entry's
// subscriber record again (mostly an L2 hit: the count pass just read it) —
// round 4 had the count copy it to a 16-B-per-entry buffer (EGM_FAN_DS0=1,
// A/B: C4 fan-out 14.17 vs 13.18 ms on one box, r5i).  A single-pass form
// (count, decoupled look-back scan, fill; tiles of 8 windows per ticket)
// measured 13.9 ms, 98 ms with one ticket per window: the ticket atomic, one
// address hit by every wave, serialises (r5h/r5i).  An
// overflowed batch (total > cap) still gets its offsets, so the caller learns
// the size.
__global__ __launch_bounds__(64 * FAN_WAVES) void k_fan_fill(const uint32_t* __restrict__ mids, uint64_t nids,
                                                             SubTable st, const uint64_t* __restrict__ wbase,
                                                             const uint4* __restrict__ ds0,
                                                             uint64_t* __restrict__ dpos,
                                                             uint32_t* __restrict__ dfid, uint32_t* __restrict__ dsub,
                                                             uint64_t cap, unsigned int* overflow) {
  const uint64_t nwin = (nids + 63) / 64;
  const bool ovf = wbase[nwin] > cap;
  if (ovf && blockIdx.x == 0 && threadIdx.x == 0) *overflow = 1u;
  __shared__ FanLds S[FAN_WAVES];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint64_t w = (uint64_t)blockIdx.x * FAN_WAVES + wave; w < nwin; w += (uint64_t)gridDim.x * FAN_WAVES) {
    const uint64_t w0 = w * 64, i = w0 + lane, ic = min(i, nids - 1);
    const uint64_t base = wbase[w];
    const uint32_t f = mids[ic];
#if EGM_FAN_DS0
    const uint4 v = ds0[ic];
#else
    const uint4 rv = st.rp[f < st.n_fid_slots ? f : 0u];   // unconditional
    const uint4 v = f < st.n_fid_slots ? rv : make_uint4(0, 0, 0, 0);
#endif
    const uint32_t c = i < nids ? fan_count_of(st, f, v) : 0u;
    uint32_t tot;
    const uint32_t off = wave_excl_scan(c, lane, &tot);
    if (i < nids) dpos[i] = base + off;
    if (i == nids - 1) dpos[nids] = base + off + c;
    if (ovf) continue;
    fan_window(S[wave], st, lane, f, v, c, off, base, dfid, dsub, cap);
  }
}

// EGM_FAN_ORDER=walk: the count in the match's walk order when it is known
// (A/B: no faster at C4, 5.79 vs 5.77 ms — a chunk's topics share few matched
// filters there; profiles/r4_c4_fan_order_ab.jsonl).  Read at each launch.
static bool fan_count_walk_order() {
  const char* e = getenv("EGM_FAN_ORDER");
  return e && strcmp(e, "walk") == 0;
}

// whether launch_fanout reads the 16-B-per-entry record copies (ds0)
bool fan_uses_ds0(bool walk_order_known) { return (walk_order_known && fan_count_walk_order()) || EGM_FAN_DS0; }

hipError_t launch_fanout(const SubTable& st, const uint64_t* mrow, const uint32_t* mids, uint32_t n,
                         uint64_t nids, uint64_t* drow, uint32_t* dfid, uint32_t* dsub, uint64_t cap,
                         uint32_t* wsum, uint4* ds0, uint64_t* dpos, uint64_t* wbase, uint64_t* tile_sums,
                         unsigned int* overflow, hipStream_t s, hipEvent_t* ev, const uint64_t* walk_order) {
  hipError_t e = hipMemsetAsync(overflow, 0, 4, s);
  if (e != hipSuccess) return e;
  if (ev) hipEventRecord(ev[0], s);
  const uint64_t nwin = (nids + 63) / 64;
  const bool ord = nids && walk_order && fan_count_walk_order();
  if (nids == 0) {
    if ((e = hipMemsetAsync(dpos, 0, 8, s)) != hipSuccess) return e;
  } else {
    if (ord) {
      if ((e = hipMemsetAsync(wsum, 0, (nwin + 1) * 4, s)) != hipSuccess) return e;
      const uint32_t g = std::min<uint32_t>((n + 64 * FAN_ORD_WAVES - 1) / (64 * FAN_ORD_WAVES), 16384);
      hipLaunchKernelGGL(k_fan_count_ord, dim3(g), dim3(64 * FAN_ORD_WAVES), 0, s, walk_order, n, mrow, mids, nids,
                         st, wsum, ds0);
    } else {
      const uint32_t g = (uint32_t)std::min<uint64_t>((nwin + 3) / 4 + 1, 8192);
      hipLaunchKernelGGL(k_fan_count, dim3(g), dim3(256), 0, s, mids, nids, st, wsum, ds0);
    }
    scan_counts(wsum, (uint32_t)nwin, tile_sums, wbase, s);   // window totals -> window bases, wbase[nwin] = all
    const uint32_t gf = (uint32_t)std::min<uint64_t>((nwin + FAN_WAVES - 1) / FAN_WAVES, 16384);
    hipLaunchKernelGGL(k_fan_fill, dim3(gf), dim3(64 * FAN_WAVES), 0, s, mids, nids, st, wbase, ds0, dpos, dfid, dsub,
                       cap, overflow);
  }
  hipLaunchKernelGGL(k_fan_rows, dim3(std::min<uint32_t>(n / 256 + 1, 8192)), dim3(256), 0, s, mrow, n, dpos, drow);
  if (ev) hipEventRecord(ev[1], s);
  return hipGetLastError();
}

// ----------------------------------------------------------- shard merge ----
// Filter-sharded layout: rank 0 holds every shard's CSR for the
// same topic batch as counts cnt[g][t] plus the shard's ids back to back.
// The match set over F is the disjoint union over the shards, so the merged
// row of topic t is shard 0's ids, then shard 1's, ... — no dedup.
// k_merge_sum: tot[t] = sum_g cnt[g][t] (scanned into the output row_ptr).
__global__ __launch_bounds__(256) void k_merge_sum(const uint32_t* __restrict__ cnt, uint32_t G, uint32_t n,
                                                   uint32_t* __restrict__ tot) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    uint32_t s = 0;
    for (uint32_t g = 0; g < G; ++g) s += cnt[(uint64_t)g * n + t];
    tot[t] = s;
  }
}

// One wave per window of 64 topics; for each shard the window's source ids
// are one contiguous run [srow[g][t0], srow[g][t0 + 64]), laid out by a wave
// scan and copied lane per id (coalesced reads; writes contiguous per topic).
constexpr int MERGE_WAVES = 4;
constexpr int MERGE_IPL = 4;
__global__ __launch_bounds__(64 * MERGE_WAVES) void k_merge_fill(const uint32_t* __restrict__ cnt,
                                                                 const uint64_t* __restrict__ srow,
                                                                 ShardIds src, uint32_t G,
                                                                 uint32_t n, const uint64_t* __restrict__ row,
                                                                 uint32_t* __restrict__ out, uint64_t cap) {
  if (row[n] > cap) return;   // the caller's buffer is too small: write nothing
  __shared__ uint32_t s_scan[MERGE_WAVES][64];
  __shared__ uint64_t s_dst[MERGE_WAVES][64];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t nwin = (n + 63) / 64;
  for (uint32_t w = blockIdx.x * MERGE_WAVES + wave; w < nwin; w += gridDim.x * MERGE_WAVES) {
    const uint32_t t = w * 64 + lane;
    const bool on = t < n;
    uint64_t dst = on ? row[t] : 0;   // advances past each shard's ids of topic t
    for (uint32_t g = 0; g < G; ++g) {
      const uint32_t c = on ? cnt[(uint64_t)g * n + t] : 0u;
      const uint64_t base = srow[(uint64_t)g * (n + 1) + w * 64];   // the window's first source id
      uint32_t tot;
      const uint32_t ex = wave_excl_scan(c, lane, &tot);
      s_scan[wave][lane] = ex;
      s_dst[wave][lane] = dst;
      dst += c;
      wave_sync();
      const uint32_t* ids = src.ids[g] + base;
      for (uint32_t q0 = lane; q0 < tot; q0 += 64 * MERGE_IPL) {
        uint32_t v[MERGE_IPL];
        uint64_t d[MERGE_IPL];
#pragma unroll
        for (int r = 0; r < MERGE_IPL; ++r) {
          const uint32_t q = min(q0 + 64u * r, tot - 1);
          uint32_t k = 0;
#pragma unroll
          for (uint32_t step = 32; step >= 1; step >>= 1)
            if (s_scan[wave][k + step] <= q) k += step;
          d[r] = s_dst[wave][k] + (q - s_scan[wave][k]);
          v[r] = ids[q];
        }
#pragma unroll
        for (int r = 0; r < MERGE_IPL; ++r)
          if (q0 + 64u * r < tot) out[d[r]] = v[r];
      }
      wave_sync();
    }
  }
}

hipError_t launch_shard_merge(const uint32_t* cnt, uint32_t G, uint32_t n, const ShardIds& src, uint64_t* srow,
                              uint64_t* tile_sums, uint32_t* tot, uint64_t* row, uint32_t* out, uint64_t cap,
                              hipStream_t s) {
  const uint32_t g1 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192));
  for (uint32_t g = 0; g < G; ++g) scan_counts(cnt + (uint64_t)g * n, n, tile_sums, srow + (uint64_t)g * (n + 1), s);
  hipLaunchKernelGGL(k_merge_sum, dim3(g1), dim3(256), 0, s, cnt, G, n, tot);
  scan_counts(tot, n, tile_sums, row, s);
  if (n) {
    const uint32_t gf = (uint32_t)std::min<uint64_t>((n + 64 * MERGE_WAVES - 1) / (64 * MERGE_WAVES), 16384);
    hipLaunchKernelGGL(k_merge_fill, dim3(gf), dim3(64 * MERGE_WAVES), 0, s, cnt, srow, src, G, n, row, out, cap);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------- copy out ----
// The host-visible path (egm_match_submit / egm_match_wait, VERDICT r3 item
// 4): a batch's CSR is written straight into the slot's pinned host buffer by
// a kernel on the copy stream, sized on the device (row_ptr[n] ids) — so the
// copy starts the moment the match ends, beside the next batch's match, and
// the host never issues a D2H after waiting for the count.  16-B units with
// nontemporal stores (write-combined PCIe writes), element tails separately.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
#ifndef EGM_COPY_OUT_BLOCKS
#define EGM_COPY_OUT_BLOCKS 64   // host path at C2: 64 -> 159M topics/s, 256 -> 141M, 1024 -> 140M (profiles/r4_host_ab.jsonl)
#endif

__device__ __forceinline__ void seg_copy16(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t bytes,
                                           uint32_t elem, uint64_t gtid, uint64_t gsize) {
  const uint64_t units = bytes / 16;
  for (uint64_t i = gtid; i < units; i += gsize) {
    const uint4 v = ((const uint4*)src)[i];
    const u32x4_t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (u32x4_t*)dst + i);
  }
  for (uint64_t b = units * 16 + gtid * elem; b < bytes; b += gsize * elem) {   // the tail, element by element
    if (elem == 8) *(uint64_t*)(dst + b) = *(const uint64_t*)(src + b);
    else if (elem == 4) *(uint32_t*)(dst + b) = *(const uint32_t*)(src + b);
    else dst[b] = src[b];
  }
}

__global__ __launch_bounds__(256) void k_copy_out(const uint64_t* __restrict__ row, uint32_t n,
                                                  const uint32_t* __restrict__ ids, uint64_t ids_cap,
                                                  const uint8_t* __restrict__ flags, uint8_t* __restrict__ h_row,
                                                  uint8_t* __restrict__ h_ids, uint8_t* __restrict__ h_fl,
                                                  const MatchStats* __restrict__ st, MatchStats* __restrict__ h_st) {
  const uint64_t gtid = (uint64_t)blockIdx.x * 256 + threadIdx.x, gsize = (uint64_t)gridDim.x * 256;
  const uint64_t nid = min(row[n], ids_cap);   // an overflowed batch is rerun: its copy is discarded
  seg_copy16((const uint8_t*)ids, h_ids, nid * 4, 4, gtid, gsize);
  seg_copy16((const uint8_t*)row, h_row, ((uint64_t)n + 1) * 8, 8, gtid, gsize);
  seg_copy16(flags, h_fl, n, 1, gtid, gsize);
  if (st && gtid < sizeof(MatchStats) / 4) ((uint32_t*)h_st)[gtid] = ((const uint32_t*)st)[gtid];
}

hipError_t launch_copy_out(const uint64_t* row, uint32_t n, const uint32_t* ids, uint64_t ids_cap,
                           const uint8_t* flags, uint8_t* h_row, uint8_t* h_ids, uint8_t* h_fl, hipStream_t s,
                           const MatchStats* st, MatchStats* h_st) {
  // one 256-thread block per CU is enough for the PCIe link (tools/d2hbench: 54 GB/s at 256 blocks) and
  // leaves the CUs' other wave slots to the next batch's match on the other stream (1 024 blocks held
  // them all for the copy's ~4 ms: r4a/r4b host_e2e 146 M topics/s)
  hipLaunchKernelGGL(k_copy_out, dim3(EGM_COPY_OUT_BLOCKS), dim3(256), 0, s, row, n, ids, ids_cap, flags, h_row, h_ids,
                     h_fl, st, h_st);
  return hipGetLastError();
}

// ------------------------------------------------------- prefix partition --
// Route a rank's topic batch to the ranks owning its prefix (SURVEY §8e,
// "partition by root word"; egm_common.h prefix_vpart): each topic goes to
// rank vpart_rank[prefix_vpart(topic)], into that rank's slot of the send
// buffer (PrefixSlots, egm_kernels.h).  One thread per topic finds its key
// (the bytes before the second '/') and its slot position: a block first
// counts its topics per destination with LDS atomics on a packed
// {topics << 40 | bytes} counter, then takes one global range per destination
// (G atomics per block instead of one per topic: 10M per-topic atomics on 8
// counters would serialise), so a topic's index and byte offset in its slot
// come from one counter and stay in step.  k_prefix_copy then moves the
// bytes, a quarter-wave per topic; k_prefix_finish writes the headers.
//
// Capacity: a topic is placed iff pos < cap_topics and bpos + len <= cap_bytes.
// pos and bpos come from one packed counter, so they grow together and the
// placed topics of a slot are exactly its positions [0, placed): the header's
// count, bytes and offsets describe them (and only them) even when the slot
// overflowed.  `placed` is the max over placed topics of the packed
// {pos + 1, bpos + len}, one LDS atomicMax per topic and one global per block
// and destination.
constexpr uint32_t PREFIX_MAX_RANKS = 16;
constexpr uint32_t PFX_BYTES_BITS = 34;   // packed counter: topics << 34 | bytes (a batch < 2^30 topics, < 2^32 B)
constexpr unsigned long long PFX_BYTES_MASK = (1ull << PFX_BYTES_BITS) - 1;

__global__ __launch_bounds__(256) void k_prefix_route(const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off,
                                                      uint32_t n, const uint8_t* __restrict__ vpart_rank,
                                                      uint32_t n_vparts, PrefixSlots ps, uint8_t* __restrict__ send,
                                                      unsigned long long* __restrict__ ctr, uint64_t* __restrict__ dst) {
  __shared__ unsigned long long lctr[PREFIX_MAX_RANKS], lbase[PREFIX_MAX_RANKS], lacc[PREFIX_MAX_RANKS];
  const uint32_t tid = threadIdx.x, G = ps.n_ranks;
  if (tid < G) {
    lctr[tid] = 0;
    lacc[tid] = 0;
  }
  __syncthreads();
  const uint32_t t = blockIdx.x * 256 + tid;
  uint32_t r = 0, len = 0;
  unsigned long long loc = 0;
  if (t < n) {
    const uint32_t a = off[t];
    len = off[t + 1] - a;
    r = vpart_rank[prefix_vpart(blob + a, len, n_vparts)];
    loc = atomicAdd(&lctr[r], (1ull << PFX_BYTES_BITS) | len);
  }
  __syncthreads();
  if (tid < G) lbase[tid] = lctr[tid] ? atomicAdd(&ctr[tid], lctr[tid]) : 0ull;
  __syncthreads();
  if (t < n) {
    const unsigned long long pos = (lbase[r] >> PFX_BYTES_BITS) + (loc >> PFX_BYTES_BITS);
    const unsigned long long bpos = (lbase[r] & PFX_BYTES_MASK) + (loc & PFX_BYTES_MASK);
    const bool ok = pos < ps.cap_topics && bpos + len <= ps.cap_bytes;
    dst[t] = ok ? ((uint64_t)r | (bpos << 8)) : ~0ull;   // ~0: not placed (the header says overflow)
    if (ok) {
      uint8_t* slot = send + (uint64_t)r * ps.slot_bytes();
      ((uint32_t*)(slot + 16))[pos] = t;
      ((uint32_t*)(slot + ps.off_offsets()))[pos] = (uint32_t)bpos;
      atomicMax(&lacc[r], ((pos + 1) << PFX_BYTES_BITS) | (bpos + len));
    }
  }
  __syncthreads();
  if (tid < G && lacc[tid]) atomicMax(&ctr[PREFIX_MAX_RANKS + tid], lacc[tid]);
}

// A quarter-wave (16 lanes) per topic copies its bytes into its slot.
__global__ __launch_bounds__(256) void k_prefix_copy(const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off,
                                                     uint32_t n, PrefixSlots ps, uint8_t* __restrict__ send,
                                                     const uint64_t* __restrict__ dst) {
  const uint32_t q = threadIdx.x >> 4, l16 = threadIdx.x & 15;
  for (uint64_t t = (uint64_t)blockIdx.x * 16 + q; t < n; t += (uint64_t)gridDim.x * 16) {
    const uint64_t d = dst[t];
    if (d == ~0ull) continue;
    const uint32_t a = off[t], len = off[t + 1] - a;
    uint8_t* out = send + (uint64_t)(d & 0xFF) * ps.slot_bytes() + ps.off_bytes() + (d >> 8);
    for (uint32_t i = l16; i < len; i += 16) out[i] = blob[a + i];
  }
}

// Headers, and the offsets past each slot's placed topics (= its placed
// bytes: empty padding topics, skipped by egm_match_device_counted through
// the count).  ctr[r] = every topic routed to r; ctr[PREFIX_MAX_RANKS + r] =
// the placed prefix.
__global__ __launch_bounds__(256) void k_prefix_finish(PrefixSlots ps, uint8_t* __restrict__ send,
                                                       const unsigned long long* __restrict__ ctr) {
  const uint32_t r = blockIdx.y;
  uint8_t* slot = send + (uint64_t)r * ps.slot_bytes();
  const uint64_t routed = ctr[r] >> PFX_BYTES_BITS, acc = ctr[PREFIX_MAX_RANKS + r];
  const uint32_t cnt = (uint32_t)(acc >> PFX_BYTES_BITS);
  const uint32_t bytes = (uint32_t)(acc & PFX_BYTES_MASK);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t* h = (uint32_t*)slot;
    h[0] = cnt;
    h[1] = bytes;
    h[2] = routed > cnt ? 1u : 0u;
    h[3] = 0;
  }
  uint32_t* po = (uint32_t*)(slot + ps.off_offsets());
  for (uint64_t k = cnt + (uint64_t)blockIdx.x * 256 + threadIdx.x; k <= ps.cap_topics; k += (uint64_t)gridDim.x * 256)
    po[k] = bytes;
}

hipError_t launch_prefix_route(const uint8_t* blob, const uint32_t* off, uint32_t n, const uint8_t* vpart_rank,
                               uint32_t n_vparts, const PrefixSlots& ps, uint8_t* send, unsigned long long* ctr,
                               uint64_t* dst, hipStream_t s) {
  if (ps.n_ranks == 0 || ps.n_ranks > PREFIX_MAX_RANKS || n_vparts == 0) return hipErrorInvalidValue;
  if (n >= PFX_TOPICS_MAX || ps.cap_topics >= PFX_TOPICS_MAX || ps.cap_bytes >= (1ull << 32)) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(ctr, 0, sizeof(unsigned long long) * 2 * PREFIX_MAX_RANKS, s);
  if (e != hipSuccess) return e;
  if (n) {
    hipLaunchKernelGGL(k_prefix_route, dim3((n + 255) / 256), dim3(256), 0, s, blob, off, n, vpart_rank, n_vparts, ps,
                       send, ctr, dst);
    const uint32_t gc = (uint32_t)std::min<uint64_t>((n + 15) / 16, 65536);
    hipLaunchKernelGGL(k_prefix_copy, dim3(gc), dim3(256), 0, s, blob, off, n, ps, send, dst);
  }
  const uint32_t gx = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(((uint64_t)ps.cap_topics + 256) / 256, 1024));
  hipLaunchKernelGGL(k_prefix_finish, dim3(gx, ps.n_ranks), dim3(256), 0, s, ps, send, ctr);
  return hipGetLastError();
}

// -------------------------------------------------------------- table patch --
// Incremental epoch commit: the records a batch of route
// adds/deletes changed (emqx_router.erl:114-125,164-170 -> emqx_trie:insert/
// delete, emqx_trie.erl:82-96) are packed on the host as {index, record} and
// scattered into the device copy of the previous image.  One lane per
// 16-byte piece of a record: a 32-B slot is two neighbouring lanes, so the
// stores of a wave cover whole 64-B lines where the indices are adjacent.
template <int Q>   // 16-byte quads per record
__global__ __launch_bounds__(256) void k_patch(uint4* __restrict__ dst, const uint32_t* __restrict__ idx,
                                               const uint4* __restrict__ src, uint64_t n) {
  const uint64_t total = n * Q;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = i / Q, q = i % Q;
    dst[(uint64_t)idx[r] * Q + q] = src[i];
  }
}

__global__ __launch_bounds__(256) void k_patch_u32(uint32_t* __restrict__ dst, const uint32_t* __restrict__ idx,
                                                   const uint32_t* __restrict__ src, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[idx[i]] = src[i];
}

hipError_t launch_patch(void* dst, uint32_t rec_bytes, const uint32_t* idx, const void* src, uint64_t n,
                        hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t lanes = rec_bytes == 4 ? n : n * (rec_bytes / 16);
  const uint32_t g = (uint32_t)std::min<uint64_t>((lanes + 255) / 256, 4096);
  switch (rec_bytes) {
    case 4:
      hipLaunchKernelGGL(k_patch_u32, dim3(g), dim3(256), 0, s, (uint32_t*)dst, idx, (const uint32_t*)src, n);
      break;
    case 16:
      hipLaunchKernelGGL(k_patch<1>, dim3(g), dim3(256), 0, s, (uint4*)dst, idx, (const uint4*)src, n);
      break;
    case 32:
      hipLaunchKernelGGL(k_patch<2>, dim3(g), dim3(256), 0, s, (uint4*)dst, idx, (const uint4*)src, n);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ------------------------------------------------- retained reverse match ----
// emqx_retainer_mnesia:match_messages/1 (apps/emqx_retainer/src/
// emqx_retainer_mnesia.erl:200-204, 215-228): one subscription filter against
// every stored retained topic.  The store is a word trie of the topics whose
// topics are ranked in depth-first order, so the topics under a node are the
// contiguous rank range [lo, hi) — a trailing '#' (the improper tail '_' of
// condition/1) emits that range whole, '+' (the match-spec '_') fans out to
// every child.  Filters advance level-synchronously over a (filter, node)
// frontier: count -> scan -> fill per level, balanced by output position.
__device__ __forceinline__ uint32_t rs_edge(const RetainView& v, uint32_t node, uint32_t w) {
  uint32_t b = edge_bucket(node, w, v.edge_mask);
  for (;;) {
    const uint4* sl = v.edges + (size_t)b * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 e = sl[k];
      if (e.x == node && e.y == w) return e.z;
      if (e.x == NONE) return NONE;
    }
    b = (b + 1) & v.edge_mask;
  }
}

__device__ __forceinline__ bool rs_alive(uint64_t e, uint64_t now, bool ge) {
  return e == 0 || e > now || (ge && e == now);
}

// one emitted range per lane at most: wave-aggregated append
__device__ __forceinline__ void rs_emit(const RetainWork& w, bool on, uint32_t f, uint32_t lo, uint32_t hi) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t m = __ballot(on);
  if (!m) return;
  const uint32_t leader = __builtin_ctzll(m);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(w.n_ranges, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  if (!on) return;
  const uint32_t i = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
  if (i < w.range_cap) {
    w.rf[i] = f;
    w.rlo[i] = lo;
    w.rhi[i] = hi;
  }
}

__global__ __launch_bounds__(256) void k_rs_alive(const uint64_t* __restrict__ expiry, uint32_t m, uint64_t now,
                                                  uint32_t* __restrict__ alive) {
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < m; r += gridDim.x * blockDim.x)
    alive[r] = rs_alive(expiry[r], now, false) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_rs_init(uint32_t n, uint32_t* __restrict__ pf, uint32_t* __restrict__ pn) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    pf[i] = i;
    pn[i] = 0;   // the root: no words consumed
  }
}

// one (filter, node) pair per lane at word index `level`
__global__ __launch_bounds__(256) void k_rs_step(RetainView v, RetainWork w, uint32_t level, uint32_t np,
                                                 const uint32_t* __restrict__ pf, const uint32_t* __restrict__ pn) {
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t n_iter = (np + stride - 1) / stride;   // uniform trip count: rs_emit ballots the whole wave
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t p = it * stride + blockIdx.x * blockDim.x + threadIdx.x;
    bool emit = false;
    uint32_t f = 0, lo = 0, hi = 0;
    if (p < np) {
      f = pf[p];
      const uint32_t node = pn[p];
      const uint32_t L = w.lv[f];
      const uint4 rec = v.nodes[node];   // {first_child, n_children | RN_TERM, lo, hi}
      uint32_t c = 0, aux = 0;
      if (level == L) {                  // every word consumed: the topic at this node
        const bool ge = w.ge_plain && !(w.tfl[f] & TF_WILDCARD);
        if ((rec.y & RN_TERM) && rs_alive(v.expiry[rec.z], w.now, ge)) {
          emit = true;
          lo = rec.z;
          hi = (rec.z + 1) | RS_SINGLE;
        }
      } else {
        const uint32_t wd = w.wid[w.off[f] + f + level];
        if (wd == WID_HASH) {            // '#' : only as the last word (condition/1, :217-219)
          if (level + 1 == L && rec.w > rec.z) {
            emit = true;
            lo = rec.z;
            hi = rec.w;
          }
        } else if (wd == WID_PLUS) {     // '_' : every child
          c = rec.y & ~RN_TERM;
          aux = rec.x;
        } else if (wd < WID_MAX && (rec.y & ~RN_TERM)) {
          const uint32_t ch = rs_edge(v, node, wd);
          if (ch != NONE) {
            c = 1;
            aux = ch;
          }
        }
      }
      w.pc[p] = c;
      w.paux[p] = aux;
    }
    rs_emit(w, emit, f, lo, hi);
  }
}

// next frontier, one lane per output pair: its source pair by binary search
__global__ __launch_bounds__(256) void k_rs_fill(RetainWork w, uint32_t np, uint64_t nnext,
                                                 const uint32_t* __restrict__ pf, uint32_t* __restrict__ pf2,
                                                 uint32_t* __restrict__ pn2) {
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nnext;
       q += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t lo = 0, hi = np;            // largest src with poff[src] <= q
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (w.poff[mid] <= q) lo = mid;
      else hi = mid;
    }
    pf2[q] = pf[lo];
    pn2[q] = w.paux[lo] + (uint32_t)(q - w.poff[lo]);
  }
}

// per range: its alive count and its offset inside the filter's row.  A
// filter's ranges are mostly adjacent in the list (frontiers stay ordered by
// filter), so lanes holding the same filter are summed with a segmented wave
// scan and reserve their space with ONE atomic per segment — a '+'-heavy
// filter emits thousands of ranges, which as per-range atomics on one counter
// serialised the whole kernel.
__global__ __launch_bounds__(256) void k_rs_count(RetainWork w, uint32_t nr) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t n_iter = (nr + stride - 1) / stride;   // uniform: the wave works together
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t r = it * stride + blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = r < nr;
    uint32_t f = NONE, c = 0;
    if (on) {
      const uint32_t hi = w.rhi[r], lo = w.rlo[r];
      f = w.rf[r];
      c = (hi & RS_SINGLE) ? 1u : (uint32_t)(w.apre[hi] - w.apre[lo]);
    }
    const uint32_t fprev = __shfl_up(f, 1, 64);
    const uint64_t heads = __ballot(lane == 0 || f != fprev);
    const uint32_t seg0 = 63 - __builtin_clzll(heads & ((2ull << lane) - 1));   // my segment's head
    uint32_t x = c;   // segmented inclusive scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= seg0 + (uint32_t)d) x += y;
    }
    const uint64_t later = heads & ~((2ull << lane) - 1);
    const uint32_t tail = later ? (uint32_t)__builtin_ctzll(later) - 1 : 63u;
    uint32_t base = 0;
    if (lane == tail && on && x) base = atomicAdd(&w.fcnt[f], x);
    base = __shfl(base, tail, 64);
    if (on) w.roff[r] = base + x - c;
  }
}

// one wave per range: its alive ranks -> message ids in the filter's row
__global__ __launch_bounds__(256) void k_rs_expand(RetainView v, RetainWork w, uint32_t nr,
                                                   const uint64_t* __restrict__ row, uint32_t* __restrict__ ids) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < nr; r += nw) {
    const uint32_t hr = w.rhi[r], lo = w.rlo[r];
    uint32_t* out = ids + row[w.rf[r]] + w.roff[r];
    if (hr & RS_SINGLE) {
      if (lane == 0) out[0] = v.msg[lo];
      continue;
    }
    const uint64_t a0 = w.apre[lo];
    const uint32_t cnt = (uint32_t)(w.apre[hr] - a0);
    if (cnt == hr - lo) {                // nothing expired in the range: ranks in order
      for (uint32_t k = lane; k < cnt; k += 64) out[k] = v.msg[lo + k];
      continue;
    }
    for (uint32_t k = lane; k < cnt; k += 64) {   // k-th alive rank: apre[rank + 1] > a0 + k
      uint32_t a = lo, b = hr - 1;
      while (a < b) {
        const uint32_t mid = (a + b) >> 1;
        if (w.apre[mid + 1] > a0 + k) b = mid;
        else a = mid + 1;
      }
      out[k] = v.msg[a];
    }
  }
}

hipError_t launch_tokenise(const DevTable& tab, const uint8_t* blob, const uint32_t* off, uint32_t n, uint32_t* wid,
                           uint32_t* lv, uint8_t* tfl, hipStream_t s) {
  const WalkOrderOut none{};
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_tokenise, dim3((n + TOK_BLOCK - 1) / TOK_BLOCK), dim3(TOK_BLOCK), 0, s, tab, blob, off, n,
                     wid, lv, tfl, none);
  return hipGetLastError();
}

static uint32_t grid_for(uint64_t n, uint32_t cap = 8192) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, cap));
}

hipError_t launch_rs_alive(const RetainView& v, const RetainWork& w, hipStream_t s) {
  if (v.n_topics) {
    hipLaunchKernelGGL(k_rs_alive, dim3(grid_for(v.n_topics)), dim3(256), 0, s, v.expiry, v.n_topics, w.now, w.alive);
  }
  scan_counts(w.alive, v.n_topics, w.tiles, w.apre, s);
  return hipGetLastError();
}

hipError_t launch_rs_init(uint32_t n, uint32_t* pf, uint32_t* pn, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_rs_init, dim3(grid_for(n)), dim3(256), 0, s, n, pf, pn);
  return hipGetLastError();
}

hipError_t launch_rs_level(const RetainView& v, const RetainWork& w, uint32_t level, uint32_t np,
                           const uint32_t* pf, const uint32_t* pn, hipStream_t s) {
  hipLaunchKernelGGL(k_rs_step, dim3(grid_for(np)), dim3(256), 0, s, v, w, level, np, pf, pn);
  scan_counts(w.pc, np, w.tiles, w.poff, s);
  return hipGetLastError();
}

hipError_t launch_rs_fill(const RetainWork& w, uint32_t np, uint64_t nnext, const uint32_t* pf, uint32_t* pf2,
                          uint32_t* pn2, hipStream_t s) {
  if (nnext) hipLaunchKernelGGL(k_rs_fill, dim3(grid_for(nnext)), dim3(256), 0, s, w, np, nnext, pf, pf2, pn2);
  return hipGetLastError();
}

hipError_t launch_rs_rows(const RetainWork& w, uint32_t nr, uint32_t n, uint64_t* row, hipStream_t s) {
  hipError_t e = hipMemsetAsync(w.fcnt, 0, ((size_t)n + 1) * 4, s);
  if (e != hipSuccess) return e;
  if (nr) hipLaunchKernelGGL(k_rs_count, dim3(grid_for(nr)), dim3(256), 0, s, w, nr);
  scan_counts(w.fcnt, n, w.tiles, row, s);
  return hipGetLastError();
}

hipError_t launch_rs_expand(const RetainView& v, const RetainWork& w, uint32_t nr, const uint64_t* row,
                            uint32_t* ids, hipStream_t s) {
  if (nr)
    hipLaunchKernelGGL(k_rs_expand, dim3(std::min<uint32_t>((nr + 3) / 4, 16384)), dim3(256), 0, s, v, w, nr, row,
                       ids);
  return hipGetLastError();
}

}  // namespace egm
