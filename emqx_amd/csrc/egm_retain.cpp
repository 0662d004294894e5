// egm_retain.cpp — retained-message store and its reverse match on the GPU
// (C-ABI in include/emqx_gpu_match.h, egm_rstore_*).
//
// Mirrors apps/emqx_retainer/src/emqx_retainer_mnesia.erl:
//   store_retained/2 :73-101  -> egm_rstore_put     (a topic keeps one record)
//   delete_message/2 :114-129 -> egm_rstore_delete  (plain topic; a wildcard
//                                delete is match + delete, see retainer.py)
//   clean/1          :148-150 -> egm_rstore_clean
//   match_messages/1 :200-204 -> egm_rstore_match   (condition/1 :215-220,
//                                make_match_spec/1 :222-228)
//   read_messages/1  :187-198 -> egm_rstore_match, EGM_RMODE_DISPATCH
//
// Device image (egm_kernels.h RetainView): the topics' word trie, nodes
// numbered breadth-first (children contiguous), topics ranked depth-first so
// the topics under a node are one rank range; a (node, word) -> child hash
// table; the dictionary in the layout k_tokenise reads; rank -> message id and
// expiry.  The image is rebuilt from the host records at each commit.
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/emqx_gpu_match.h"
#include "egm_alloc.h"
#include "egm_kernels.h"

using namespace egm;

namespace {

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() { release(); }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    size_t b = std::max<size_t>(bytes, 256);
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

template <class T>
hipError_t put_vec(Buf& b, const std::vector<T>& v) {
  hipError_t e = b.ensure(v.size() * sizeof(T) + 16);
  if (e == hipSuccess && !v.empty()) e = hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return e;
}

struct Rec {
  uint32_t msg;
  uint64_t expiry;
};

// The host image (built at commit).
struct Image {
  std::vector<uint4> nodes;           // RetainView::nodes
  std::vector<uint4> edges;           // 16 B slots, 4 per bucket
  uint32_t edge_mask = 0;
  std::vector<DictSlot> dict;
  std::vector<uint8_t> dict_blob;
  std::vector<uint64_t> dict_off;
  std::vector<uint32_t> msg;
  std::vector<uint64_t> expiry;
};

bool split_words(const std::string& t, std::vector<std::pair<uint32_t, uint32_t>>* out) {
  out->clear();
  uint32_t ws = 0;
  for (uint32_t i = 0; i <= t.size(); ++i) {
    if (i < t.size() && t[i] != '/') continue;
    out->push_back({ws, i - ws});
    ws = i + 1;
  }
  return true;
}

void build_image(const std::unordered_map<std::string, Rec>& recs, Image* im) {
  // dictionary: every distinct topic word, in the k_tokenise probe layout
  std::unordered_map<std::string, uint32_t> wmap;
  std::vector<const std::string*> topics;
  topics.reserve(recs.size());
  for (const auto& kv : recs) topics.push_back(&kv.first);
  std::vector<uint64_t> woff(1, 0);   // per topic: first word in flat
  std::vector<uint32_t> flat;
  std::vector<std::pair<uint32_t, uint32_t>> ws;
  im->dict_blob.clear();
  im->dict_off.assign(1, 0);
  for (const std::string* t : topics) {
    split_words(*t, &ws);
    for (auto [s, l] : ws) {
      std::string w = t->substr(s, l);
      auto it = wmap.find(w);
      uint32_t id;
      if (it == wmap.end()) {
        id = (uint32_t)wmap.size();
        wmap.emplace(w, id);
        im->dict_blob.insert(im->dict_blob.end(), w.begin(), w.end());
        im->dict_off.push_back(im->dict_blob.size());
      } else {
        id = it->second;
      }
      flat.push_back(id);
    }
    woff.push_back(flat.size());
  }
  size_t dcap = 64;
  while (dcap < wmap.size() * 2) dcap <<= 1;
  im->dict.assign(dcap, DictSlot{0, NONE, 0, {0}});
  for (uint32_t w = 0; w + 1 < im->dict_off.size(); ++w) {
    const uint8_t* p = im->dict_blob.data() + im->dict_off[w];
    const uint32_t len = (uint32_t)(im->dict_off[w + 1] - im->dict_off[w]);
    const uint64_t h = word_hash(p, len);
    uint32_t i = (uint32_t)(h & (dcap - 1));
    while (im->dict[i].wid != NONE) i = (i + 1) & (uint32_t)(dcap - 1);
    DictSlot s{h, w, len, {0}};
    memcpy(s.inl, p, len < 16 ? len : 16);
    im->dict[i] = s;
  }

  // depth-first ranks: topics sorted by their word-id sequences (a prefix
  // sorts before its extensions)
  const uint32_t M = (uint32_t)topics.size();
  std::vector<uint32_t> order(M);
  std::iota(order.begin(), order.end(), 0u);
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return std::lexicographical_compare(flat.begin() + woff[a], flat.begin() + woff[a + 1], flat.begin() + woff[b],
                                        flat.begin() + woff[b + 1]);
  });
  // trie in depth-first order: node = (parent, word, lo, hi, term)
  struct DNode {
    uint32_t parent, word, lo, hi;
    bool term;
  };
  std::vector<DNode> dn;
  dn.push_back({NONE, NONE, 0, M, false});   // root: no word consumed
  std::vector<uint32_t> path(1, 0);            // path[d] = node after d words
  im->msg.resize(M);
  im->expiry.resize(M);
  for (uint32_t r = 0; r < M; ++r) {
    const uint32_t t = order[r];
    const uint64_t a = woff[t], b = woff[t + 1];
    const uint32_t D = (uint32_t)(b - a);
    // common prefix with the current path
    uint32_t c = 0;
    while (c + 1 < path.size() && c < D && dn[path[c + 1]].word == flat[a + c]) ++c;
    for (size_t d = path.size() - 1; d > c; --d) dn[path[d]].hi = r;   // close the rest
    path.resize(c + 1);
    for (uint32_t d = c; d < D; ++d) {
      dn.push_back({path[d], flat[a + d], r, M, false});
      path.push_back((uint32_t)dn.size() - 1);
    }
    dn[path[D]].term = true;   // D >= 1: words/1 of any topic has >= 1 word
    const Rec& rec = recs.at(*topics[t]);
    im->msg[r] = rec.msg;
    im->expiry[r] = rec.expiry;
  }
  // breadth-first numbering: the children of a node are contiguous
  const uint32_t N = (uint32_t)dn.size();
  std::vector<uint32_t> kstart(N + 1, 0), kids;
  for (uint32_t i = 1; i < N; ++i) ++kstart[dn[i].parent + 1];
  for (uint32_t i = 0; i < N; ++i) kstart[i + 1] += kstart[i];
  kids.resize(kstart[N]);
  {
    std::vector<uint32_t> pos(kstart.begin(), kstart.end() - 1);
    for (uint32_t i = 1; i < N; ++i) kids[pos[dn[i].parent]++] = i;   // depth-first = word order
  }
  std::vector<uint32_t> bfs;
  bfs.reserve(N);
  std::vector<uint32_t> nid(N, NONE);
  bfs.push_back(0);
  nid[0] = 0;
  for (size_t q = 0; q < bfs.size(); ++q)
    for (uint32_t k = kstart[bfs[q]]; k < kstart[bfs[q] + 1]; ++k) {
      nid[kids[k]] = (uint32_t)bfs.size();
      bfs.push_back(kids[k]);
    }
  im->nodes.assign(N, uint4{0, 0, 0, 0});
  for (uint32_t o = 0; o < N; ++o) {
    const uint32_t i = nid[o];
    const uint32_t nk = kstart[o + 1] - kstart[o];
    const uint32_t first = nk ? nid[kids[kstart[o]]] : 0u;
    im->nodes[i] = uint4{first, nk | (dn[o].term ? RN_TERM : 0u), dn[o].lo, dn[o].hi};
  }
  // (node, word) -> child, 25-50 % slot load
  size_t nb = 16;
  while (nb * 4 < (size_t)(N - 1) * 2) nb <<= 1;
  im->edges.assign(nb * 4, uint4{NONE, 0, 0, 0});
  im->edge_mask = (uint32_t)(nb - 1);
  for (uint32_t o = 1; o < N; ++o) {
    const uint32_t par = nid[dn[o].parent], w = dn[o].word;
    uint32_t bkt = edge_bucket(par, w, im->edge_mask);
    for (;;) {
      uint4* sl = &im->edges[(size_t)bkt * 4];
      int k = 0;
      while (k < 4 && sl[k].x != NONE) ++k;
      if (k < 4) {
        sl[k] = uint4{par, w, nid[o], 0};
        break;
      }
      bkt = (bkt + 1) & im->edge_mask;
    }
  }
}

}  // namespace

struct egm_rstore {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::unordered_map<std::string, Rec> recs;
  bool dirty = true;
  std::string err;
  // committed image
  Buf nodes, edges, dict, dict_blob, dict_off, msg, expiry;
  RetainView view{};
  DevTable dtab{};
  uint64_t n_nodes = 0;
  // per-batch workspace
  Buf in_blob, in_off, wid, lv, tfl, pf[2], pn[2], pc, paux, poff, tiles, rf, rlo, rhi, nr, alive, apre, fcnt, roff,
      row, ids;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip_fail(hipError_t e, const char* where) {
    err = std::string(where) + ": " + hipGetErrorString(e);
    return EGM_E_DEVICE;
  }
};

static int rs_commit_locked(egm_rstore* r) {
  if (!r->dirty) return EGM_OK;
  Image im;
  build_image(r->recs, &im);
  hipError_t e;
  hipStreamSynchronize(r->stream);
  if ((e = put_vec(r->nodes, im.nodes)) || (e = put_vec(r->edges, im.edges)) || (e = put_vec(r->dict, im.dict)) ||
      (e = put_vec(r->dict_blob, im.dict_blob)) || (e = put_vec(r->dict_off, im.dict_off)) ||
      (e = put_vec(r->msg, im.msg)) || (e = put_vec(r->expiry, im.expiry)))
    return r->hip_fail(e, "retained image upload");
  r->view.nodes = r->nodes.as<uint4>();
  r->view.edges = r->edges.as<uint4>();
  r->view.edge_mask = im.edge_mask;
  r->view.msg = r->msg.as<uint32_t>();
  r->view.expiry = r->expiry.as<uint64_t>();
  r->view.n_topics = (uint32_t)im.msg.size();
  r->dtab = DevTable{};
  r->dtab.dict = r->dict.as<DictSlot>();
  r->dtab.dict_mask = (uint32_t)(im.dict.size() - 1);
  r->dtab.dict_blob = r->dict_blob.as<uint8_t>();
  r->dtab.dict_off = r->dict_off.as<uint64_t>();
  r->n_nodes = im.nodes.size();
  r->dirty = false;
  return EGM_OK;
}

static bool has_wildcard_word(const uint8_t* p, uint32_t len) {
  uint32_t ws = 0;
  for (uint32_t i = 0; i <= len; ++i) {
    if (i < len && p[i] != '/') continue;
    if (i - ws == 1 && (p[ws] == '+' || p[ws] == '#')) return true;
    ws = i + 1;
  }
  return false;
}

extern "C" {

int egm_rstore_open(int device, egm_rstore** out) {
  if (!out) return EGM_E_INVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return EGM_E_DEVICE;
  egm_rstore* r = new (std::nothrow) egm_rstore();
  if (!r) return EGM_E_NOMEM;
  r->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
    delete r;
    return EGM_E_DEVICE;
  }
  if (rs_commit_locked(r) != EGM_OK) {
    hipStreamDestroy(r->stream);
    delete r;
    return EGM_E_DEVICE;
  }
  *out = r;
  return EGM_OK;
}

void egm_rstore_close(egm_rstore* r) {
  if (!r) return;
  hipSetDevice(r->device);
  hipStreamSynchronize(r->stream);
  hipStreamDestroy(r->stream);
  delete r;
}

const char* egm_rstore_last_error(egm_rstore* r) { return r ? r->err.c_str() : "null store"; }

int egm_rstore_put(egm_rstore* r, const uint8_t* topic, uint32_t len, uint32_t msg_id, uint64_t expiry_ms) {
  if (!r || (!topic && len)) return EGM_E_INVAL;
  if (has_wildcard_word(topic, len)) return EGM_E_INVAL;   // publish topics carry no wildcard
  std::lock_guard<std::mutex> g(r->mu);
  r->recs[std::string((const char*)topic, len)] = Rec{msg_id, expiry_ms};
  r->dirty = true;
  return EGM_OK;
}

int egm_rstore_delete(egm_rstore* r, const uint8_t* topic, uint32_t len) {
  if (!r || (!topic && len)) return EGM_E_INVAL;
  std::lock_guard<std::mutex> g(r->mu);
  r->dirty |= r->recs.erase(std::string((const char*)topic, len)) > 0;
  return EGM_OK;
}

int egm_rstore_clean(egm_rstore* r) {
  if (!r) return EGM_E_INVAL;
  std::lock_guard<std::mutex> g(r->mu);
  r->recs.clear();
  r->dirty = true;
  return EGM_OK;
}

int egm_rstore_size(egm_rstore* r, uint64_t* n) {
  if (!r || !n) return EGM_E_INVAL;
  std::lock_guard<std::mutex> g(r->mu);
  *n = r->recs.size();
  return EGM_OK;
}

int egm_rstore_commit(egm_rstore* r) {
  if (!r) return EGM_E_INVAL;
  std::lock_guard<std::mutex> g(r->mu);
  if (hipSetDevice(r->device) != hipSuccess) return EGM_E_DEVICE;
  return rs_commit_locked(r);
}

int egm_rstore_match(egm_rstore* r, const uint8_t* blob, const uint32_t* off, uint32_t n, uint64_t now_ms, int mode,
                     egm_result** out) {
  if (!r || !out || (mode != EGM_RMODE_MATCH && mode != EGM_RMODE_DISPATCH)) return EGM_E_INVAL;
  if (n && !off) return EGM_E_INVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return EGM_E_INVAL;
  if (n && !blob && off[n] > off[0]) return EGM_E_INVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> g(r->mu);
  if (hipSetDevice(r->device) != hipSuccess) return EGM_E_DEVICE;
  int rc = rs_commit_locked(r);   // queries see every put/delete made before them
  if (rc) return rc;
  hipStream_t s = r->stream;
  hipError_t e;
  const uint32_t base0 = n ? off[0] : 0;
  const uint64_t bytes = n ? (uint64_t)off[n] - base0 : 0;
  std::vector<uint32_t> loff(n + 1);
  for (uint32_t i = 0; i <= n; ++i) loff[i] = n ? off[i] - base0 : 0;
  const uint32_t M = r->view.n_topics;
  const size_t nn = (size_t)n + 1;
  if ((e = r->in_blob.ensure(bytes + 16)) || (e = r->in_off.ensure(nn * 4)) ||
      (e = r->wid.ensure((bytes + nn) * 4)) || (e = r->lv.ensure(nn * 4)) || (e = r->tfl.ensure(nn)) ||
      (e = r->alive.ensure(((size_t)M + 1) * 4)) || (e = r->apre.ensure(((size_t)M + 2) * 8)) ||
      (e = r->fcnt.ensure(nn * 4)) || (e = r->row.ensure(nn * 8)) || (e = r->nr.ensure(16)))
    return r->hip_fail(e, "retained workspace");
  if (bytes && (e = hipMemcpyAsync(r->in_blob.p, blob + base0, bytes, hipMemcpyHostToDevice, s)))
    return r->hip_fail(e, "H2D filters");
  if ((e = hipMemcpyAsync(r->in_off.p, loff.data(), nn * 4, hipMemcpyHostToDevice, s)))
    return r->hip_fail(e, "H2D offsets");

  RetainWork w{};
  w.off = r->in_off.as<uint32_t>();
  w.wid = r->wid.as<uint32_t>();
  w.lv = r->lv.as<uint32_t>();
  w.tfl = r->tfl.as<uint8_t>();
  w.alive = r->alive.as<uint32_t>();
  w.apre = r->apre.as<uint64_t>();
  w.fcnt = r->fcnt.as<uint32_t>();
  w.n_ranges = r->nr.as<uint32_t>();
  w.now = now_ms;
  w.ge_plain = mode == EGM_RMODE_DISPATCH;
  auto tiles_for = [&](uint64_t m) { return (scan_tiles((uint32_t)std::min<uint64_t>(m, 0xFFFFFFFFull)) + 2) * 8; };
  size_t tiles_need = std::max(tiles_for(M), tiles_for(n));
  if ((e = r->tiles.ensure(tiles_need))) return r->hip_fail(e, "tiles");
  w.tiles = r->tiles.as<uint64_t>();

  if ((e = launch_tokenise(r->dtab, r->in_blob.as<uint8_t>(), w.off, n, r->wid.as<uint32_t>(), r->lv.as<uint32_t>(),
                           r->tfl.as<uint8_t>(), s)) ||
      (e = launch_rs_alive(r->view, w, s)))
    return r->hip_fail(e, "tokenise/alive");

  // frontier walk, level by level; ranges may overflow -> rerun with room
  uint64_t range_cap = std::max<uint64_t>(4 * (uint64_t)n + 1024, r->rf.cap / 4);
  uint32_t n_ranges = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (range_cap > 0xFFFFFFF0ull) return r->fail(EGM_E_NOMEM, "too many result ranges in one batch");
    if ((e = r->rf.ensure(range_cap * 4)) || (e = r->rlo.ensure(range_cap * 4)) || (e = r->rhi.ensure(range_cap * 4)) ||
        (e = r->roff.ensure(range_cap * 4)))
      return r->hip_fail(e, "ranges");
    w.rf = r->rf.as<uint32_t>();
    w.rlo = r->rlo.as<uint32_t>();
    w.rhi = r->rhi.as<uint32_t>();
    w.roff = r->roff.as<uint32_t>();
    w.range_cap = (uint32_t)range_cap;
    if ((e = hipMemsetAsync(w.n_ranges, 0, 4, s))) return r->hip_fail(e, "memset");
    uint64_t np = n;
    int cur = 0;
    if ((e = r->pf[0].ensure(nn * 4)) || (e = r->pn[0].ensure(nn * 4))) return r->hip_fail(e, "frontier");
    if ((e = launch_rs_init(n, r->pf[0].as<uint32_t>(), r->pn[0].as<uint32_t>(), s)))
      return r->hip_fail(e, "init");
    for (uint32_t level = 0; np; ++level) {
      if (np > 0xFFFFFFF0ull) return r->fail(EGM_E_NOMEM, "frontier too large (split the batch)");
      if ((e = r->pc.ensure((np + 1) * 4)) || (e = r->paux.ensure((np + 1) * 4)) ||
          (e = r->poff.ensure((np + 2) * 8)) || (e = r->tiles.ensure(std::max(tiles_need, tiles_for(np)))))
        return r->hip_fail(e, "level workspace");
      w.pc = r->pc.as<uint32_t>();
      w.paux = r->paux.as<uint32_t>();
      w.poff = r->poff.as<uint64_t>();
      w.tiles = r->tiles.as<uint64_t>();
      if ((e = launch_rs_level(r->view, w, level, (uint32_t)np, r->pf[cur].as<uint32_t>(), r->pn[cur].as<uint32_t>(),
                               s)))
        return r->hip_fail(e, "level");
      uint64_t nnext = 0;
      if ((e = hipMemcpyAsync(&nnext, w.poff + np, 8, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
        return r->hip_fail(e, "level readback");
      if (nnext) {
        if ((e = r->pf[cur ^ 1].ensure(nnext * 4 + 16)) || (e = r->pn[cur ^ 1].ensure(nnext * 4 + 16)))
          return r->hip_fail(e, "frontier");
        if ((e = launch_rs_fill(w, (uint32_t)np, nnext, r->pf[cur].as<uint32_t>(), r->pf[cur ^ 1].as<uint32_t>(),
                                r->pn[cur ^ 1].as<uint32_t>(), s)))
          return r->hip_fail(e, "fill");
        // the next level may grow (reallocate) the buffers this fill reads
        if ((e = hipStreamSynchronize(s))) return r->hip_fail(e, "fill sync");
      }
      cur ^= 1;
      np = nnext;
    }
    if ((e = hipMemcpyAsync(&n_ranges, w.n_ranges, 4, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
      return r->hip_fail(e, "ranges readback");
    if (n_ranges <= range_cap) break;
    range_cap = (uint64_t)n_ranges + n_ranges / 4 + 1024;
    if (attempt == 1) return r->fail(EGM_E_NOMEM, "ranges capacity");
  }
  uint64_t* d_row = r->row.as<uint64_t>();
  if ((e = launch_rs_rows(w, n_ranges, n, d_row, s))) return r->hip_fail(e, "rows");
  uint64_t total = 0;
  if ((e = hipMemcpyAsync(&total, d_row + n, 8, hipMemcpyDeviceToHost, s)) || (e = hipStreamSynchronize(s)))
    return r->hip_fail(e, "rows readback");
  if ((e = r->ids.ensure(total * 4 + 16))) return r->hip_fail(e, "ids");
  if ((e = launch_rs_expand(r->view, w, n_ranges, d_row, r->ids.as<uint32_t>(), s))) return r->hip_fail(e, "expand");

  size_t sz = sizeof(egm_result);
  const size_t o_counts = sz;
  sz += ((uint64_t)n * 4 + 7) & ~7ull;
  const size_t o_row = sz;
  sz += nn * 8;
  const size_t o_ids = sz;
  sz += (total * 4 + 7) & ~7ull;
  const size_t o_flags = sz;
  sz += n + 8;
  uint8_t* mem = (uint8_t*)result_alloc(sz);
  if (!mem) return r->fail(EGM_E_NOMEM, "result");
  egm_result* res = (egm_result*)mem;
  memset(res, 0, sizeof(*res));
  res->n_topics = n;
  res->n_ids = total;
  res->counts = (uint32_t*)(mem + o_counts);
  res->row_ptr = (uint64_t*)(mem + o_row);
  res->ids = (uint32_t*)(mem + o_ids);
  res->flags = (uint8_t*)(mem + o_flags);
  if ((e = hipMemcpyAsync(res->row_ptr, d_row, nn * 8, hipMemcpyDeviceToHost, s)) ||
      (total && (e = hipMemcpyAsync(res->ids, r->ids.p, total * 4, hipMemcpyDeviceToHost, s))) ||
      (n && (e = hipMemcpyAsync(res->flags, r->tfl.p, n, hipMemcpyDeviceToHost, s))) ||
      (e = hipStreamSynchronize(s))) {
    result_discard(mem);
    return r->hip_fail(e, "D2H result");
  }
  for (uint32_t i = 0; i < n; ++i) res->counts[i] = (uint32_t)(res->row_ptr[i + 1] - res->row_ptr[i]);
  res->visited = n_ranges;
  *out = res;
  return EGM_OK;
}

}  // extern "C"
