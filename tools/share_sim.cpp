// Offline analysis of the C2 walk (not product code): how many random reads
// the NFA walk issues per topic, which of them a smarter layout could avoid,
// and how many a prefix-sharing walk over a sorted batch would still issue.
// g++ -O3 -std=c++17 -I emqx_amd/csrc tools/share_sim.cpp emqx_amd/csrc/egm_table.cpp emqx_amd/csrc/egm_synth.cpp -o /tmp/share_sim
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <numeric>
#include <vector>
#include "egm_table.h"
using namespace egm;
extern "C" {
typedef struct egs_strings { uint8_t* blob; uint64_t bytes; uint32_t* off; uint32_t n; } egs_strings;
int egs_filters(uint64_t, uint32_t, int, int, double, double, double, double, double, uint32_t, egs_strings*);
int egs_topics(uint64_t, const egs_strings*, uint32_t, int, int, double, double, double, double, uint32_t, egs_strings*);
}
static const EdgeSlot* probe(const HostTable& T, uint32_t node, uint32_t w, uint32_t* bucket) {
  uint32_t b = edge_bucket(node, w, T.edge_mask());
  *bucket = b;
  for (;;) {
    for (int k = 0; k < EDGE_BUCKET; ++k) {
      const EdgeSlot& s = T.edges[(size_t)b * EDGE_BUCKET + k];
      if (s.parent == node && s.wid == w) return &s;
      if (s.parent == NONE) return nullptr;
    }
    b = (b + 1) & T.edge_mask();
  }
}
int main(int argc, char** argv) {
  uint32_t nf = argc > 1 ? atoi(argv[1]) : 10000000, nt = argc > 2 ? atoi(argv[2]) : 2000000;
  uint64_t seed = 0xE3C00000ull + 2;
  egs_strings F, Tp;
  egs_filters(seed, nf, 4, 8, 1.0, 0.15, 0.5, 0.05, 1.1, 100000, &F);
  egs_topics(seed, &F, nt, 4, 8, 0.5, 0.01, 0.05, 1.1, 100000, &Tp);
  HostTable T;
  for (uint32_t i = 0; i < F.n; ++i) { uint32_t o; T.insert(F.blob + F.off[i], F.off[i + 1] - F.off[i], i, &o); }
  T.relayout();
  fprintf(stderr, "table: %zu nodes, %zu buckets\n", T.nodes.size(), T.edges.size() / 4);
  // literal-child signature per node: bit (mix64(wid) % SB) of every literal child word
  const int SB = argc > 3 ? atoi(argv[3]) : 28;
  std::vector<uint32_t> sig(T.nodes.size(), 0);
  for (const EdgeSlot& e : T.edges)
    if (e.parent != NONE && e.parent != TOMB) sig[e.parent] |= 1u << (mix64(e.wid) % SB);
  // tokenise
  std::vector<uint32_t> woff(nt + 1), wids;
  std::vector<uint8_t> dollar(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    woff[t] = wids.size();
    const uint8_t* p = Tp.blob + Tp.off[t];
    uint32_t len = Tp.off[t + 1] - Tp.off[t], s = 0;
    dollar[t] = len && p[0] == '$';
    for (uint32_t i = 0; i <= len; ++i)
      if (i == len || p[i] == '/') { wids.push_back(T.dict_find(p + s, i - s)); s = i + 1; }
  }
  woff[nt] = wids.size();
  // sorted order by word-id sequence
  std::vector<uint32_t> ord(nt);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
    return std::lexicographical_compare(wids.begin() + woff[a], wids.begin() + woff[a + 1], wids.begin() + woff[b],
                                        wids.begin() + woff[b + 1]);
  });
  auto lcp = [&](uint32_t a, uint32_t b) {
    uint32_t da = woff[a + 1] - woff[a], db = woff[b + 1] - woff[b], k = 0;
    while (k < da && k < db && wids[woff[a] + k] == wids[woff[b] + k]) ++k;
    return k;
  };
  struct St { uint32_t node, level, fl, plus, wc, via_plus; };
  uint64_t lit_sig = 0, plus_b = 0;
  uint64_t lit = 0, litok = 0, plus = 0, plus_leaf = 0, plus_noexp = 0, popped = 0, emits = 0;
  const int NG = 4;
  const uint32_t groups[NG] = {1, 64, 1024, 0xFFFFFFFFu};
  uint64_t sh_reads[NG] = {0};
  std::vector<St> stk;
  for (uint32_t i = 0; i < nt; ++i) {
    const uint32_t t = ord[i];
    const uint32_t D = woff[t + 1] - woff[t];
    const uint32_t* w = &wids[woff[t]];
    bool wild = false;
    for (uint32_t l = 0; l < D; ++l) wild |= (w[l] == WID_PLUS || w[l] == WID_HASH);
    if (wild) continue;
    uint32_t lc[NG];
    for (int g = 0; g < NG; ++g) lc[g] = (i % groups[g] == 0 || i == 0) ? 0 : lcp(ord[i - 1], t);
    const NodeRec& r = T.nodes[0];
    stk.clear();
    uint32_t fl = r.flags & (F_LIT | (dollar[t] ? 0 : F_PLUS));
    if (fl) stk.push_back({0, 0, fl, r.plus_child, 0, 0});
    while (!stk.empty()) {
      St s = stk.back(); stk.pop_back(); ++popped;
      const uint32_t nl = s.level + 1; const bool leaf = nl == D;
      if ((s.fl & F_PLUS) && s.via_plus) ++plus_b;
      if ((s.fl & F_LIT) && w[s.level] < WID_MAX && (sig[s.node] >> (mix64(w[s.level]) % SB) & 1)) ++lit_sig;
      if ((s.fl & F_LIT) && w[s.level] < WID_MAX) {
        ++lit;
        for (int g = 0; g < NG; ++g) sh_reads[g] += lc[g] >= s.level + 1 ? 0 : 1;
        uint32_t b; const EdgeSlot* e = probe(T, s.node, w[s.level], &b);
        if (e) {
          ++litok;
          emits += (e->child_flags & F_HASH) ? 1 : 0;
          if (!leaf && (e->child_flags & (F_LIT | F_PLUS))) stk.push_back({e->child, nl, e->child_flags, e->child_plus, s.wc, 0});
          else if (leaf) emits += (e->child_flags & F_TERM) ? 1 : 0;
        }
      }
      if (s.fl & F_PLUS) {
        ++plus;
        for (int g = 0; g < NG; ++g) sh_reads[g] += lc[g] >= s.level ? 0 : 1;
        const NodeRec& c = T.nodes[s.plus];
        if (leaf) ++plus_leaf;
        else if (!(c.flags & (F_LIT | F_PLUS))) ++plus_noexp;
        if (!leaf && (c.flags & (F_LIT | F_PLUS))) stk.push_back({s.plus, nl, c.flags, c.plus_child, 1, 1});
      }
    }
  }
  printf("topics %u: popped %.2f/t, lit probes %.2f/t (found %.2f), plus reads %.2f/t (leaf %.2f, no-expand %.2f)\n",
         nt, popped / (double)nt, lit / (double)nt, litok / (double)nt, plus / (double)nt, plus_leaf / (double)nt,
         plus_noexp / (double)nt);
  printf("signature %d bits: lit probes %.2f/t; plus reads if '+' records ride with their parent: %.2f/t\n", SB,
         lit_sig / (double)nt, plus_b / (double)nt);
  for (int g = 0; g < NG; ++g)
    printf("prefix-shared reads, sorted groups of %u: %.2f/t (%.1f%% of %.2f)\n", groups[g], sh_reads[g] / (double)nt,
           100.0 * sh_reads[g] / (lit + plus), (lit + plus) / (double)nt);
  return 0;
}
