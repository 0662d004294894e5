// egm_synth.cpp — deterministic synthetic filter / topic / subscriber sets for
// the benchmark configs of BASELINE.json (distributions: SURVEY.md §8d).
//
// The reference has no such generator; its only harness renders two fixed
// patterns (apps/emqx/src/emqx_broker_bench.erl:25-34,169-184).  This is test
// and benchmark infrastructure, not part of the drop-in boundary.
//
// Words: level-l vocabulary "w{l}_{k}", k ~ Zipf(s) over V_l = min(16*8^l, vmax);
// a fraction of words is '' (empty level).  RNG: xoshiro256** seeded through
// splitmix64 (SURVEY names PCG64; any fixed PRNG is equivalent for these
// distributions — the seed convention 0xE3C00000 + config index is kept).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_set>
#include <vector>

namespace {

struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (int i = 0; i < 4; ++i) {
      seed += 0x9e3779b97f4a7c15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  int range(int lo, int hi) { return lo + (int)below((uint32_t)(hi - lo + 1)); }
};

struct Vocab {
  std::vector<std::vector<double>> cdf;  // per level
  double s;
  uint32_t vmax;
  Vocab(double s_, uint32_t vmax_) : s(s_), vmax(vmax_) {}
  const std::vector<double>& level(int l) {
    while ((int)cdf.size() <= l) {
      int L = (int)cdf.size();
      double v = 16.0 * std::pow(8.0, L);
      uint32_t V = (uint32_t)std::min<double>(v, (double)vmax);
      std::vector<double> c(V);
      double acc = 0;
      for (uint32_t k = 0; k < V; ++k) {
        acc += 1.0 / std::pow((double)(k + 1), s);
        c[k] = acc;
      }
      for (auto& x : c) x /= acc;
      cdf.push_back(std::move(c));
    }
    return cdf[l];
  }
  uint32_t sample(Rng& r, int l) {
    const auto& c = level(l);
    double u = r.uni();
    return (uint32_t)(std::lower_bound(c.begin(), c.end(), u) - c.begin());
  }
};

// "w{l}_{k}" (formatted by hand: snprintf dominated generation time)
void put_uint(std::string& out, uint32_t v) {
  char buf[12];
  int i = 12;
  do {
    buf[--i] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  out.append(buf + i, 12 - i);
}

void put_word(std::string& out, int l, uint32_t k) {
  out += 'w';
  put_uint(out, (uint32_t)l);
  out += '_';
  put_uint(out, k);
}

struct Strings {
  std::string blob;
  std::vector<uint32_t> off{0};
  void push(const std::string& s) {
    blob += s;
    off.push_back((uint32_t)blob.size());
  }
};

}  // namespace

extern "C" {

typedef struct egs_strings {
  uint8_t* blob;
  uint64_t bytes;
  uint32_t* off;  // [n+1]
  uint32_t n;
} egs_strings;

static int export_strings(Strings& s, egs_strings* out) {
  out->n = (uint32_t)(s.off.size() - 1);
  out->bytes = s.blob.size();
  out->blob = (uint8_t*)malloc(out->bytes + 16);
  out->off = (uint32_t*)malloc(s.off.size() * 4);
  if (!out->blob || !out->off) return -2;
  memcpy(out->blob, s.blob.data(), out->bytes);
  memcpy(out->off, s.off.data(), s.off.size() * 4);
  return 0;
}

void egs_free(egs_strings* s) {
  if (!s) return;
  free(s->blob);
  free(s->off);
  s->blob = nullptr;
  s->off = nullptr;
}

// One candidate filter (the distribution of egs_filters).
static void gen_filter(Rng& r, Vocab& voc, std::string& f, int dmin, int dmax, double wc_frac, double p_plus,
                       double p_hash, double p_empty) {
  f.clear();
  int d = r.range(dmin, dmax);
  bool wild = r.uni() < wc_frac, any = false;
  for (int l = 0; l < d; ++l) {
    if (l) f += '/';
    if (wild && l == d - 1 && (r.uni() < p_hash || !any)) {
      f += '#';
      any = true;
    } else if (wild && r.uni() < p_plus) {
      f += '+';
      any = true;
    } else if (r.uni() < p_empty) {
      // '' level
    } else {
      put_word(f, l, voc.sample(r, l));
    }
  }
}

static unsigned synth_threads() {
  const char* e = getenv("EGM_BUILD_THREADS");
  if (e && *e) return (unsigned)std::max(1, atoi(e));
  unsigned n = std::max(1u, std::thread::hardware_concurrency());
  if (FILE* fp = fopen("/sys/fs/cgroup/cpu.max", "r")) {   // the cgroup CPU quota
    char q[64] = {0};
    unsigned long long period = 0;
    if (fscanf(fp, "%63s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period)
      n = std::min<unsigned>(n, (unsigned)std::max<unsigned long long>(1, (strtoull(q, nullptr, 10) + period - 1) / period));
    fclose(fp);
  }
  return std::min(n, 64u);
}

// Large sets (n > PAR_MIN): candidates in blocks of PAR_BLOCK, block k from
// its own stream (seed, k), generated in parallel; duplicates dropped in
// candidate order (first occurrence kept) by hash partitions in parallel;
// rounds of blocks until n filters are unique.  Deterministic for any thread
// count.  Smaller sets keep the single-stream generator (the C0-C3 sets of
// earlier rounds are unchanged).
constexpr uint32_t PAR_MIN = 16u << 20;
constexpr uint32_t PAR_BLOCK = 1u << 20;

static int egs_filters_par(uint64_t seed, uint32_t n, int dmin, int dmax, double wc_frac, double p_plus,
                           double p_hash, double p_empty, double zipf_s, uint32_t vmax, egs_strings* out) {
  const unsigned T = synth_threads();
  struct Block {
    std::string blob;
    std::vector<uint32_t> off{0};
    std::vector<uint64_t> h;
    std::vector<uint8_t> keep;
  };
  std::vector<Block> blocks;
  std::vector<std::unordered_set<std::string_view>> part(T);
  uint64_t have = 0;
  uint32_t next_block = 0;
  while (have < n) {
    if ((uint64_t)next_block * PAR_BLOCK > (uint64_t)n * 50) return -1;   // the sequential bound on attempts
    const uint32_t want = (uint32_t)std::max<uint64_t>(1, ((n - have) * 103 / 100 + PAR_BLOCK - 1) / PAR_BLOCK);
    const size_t b0 = blocks.size();
    blocks.resize(b0 + want);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        Vocab voc(zipf_s, vmax);
        std::string f;
        for (size_t k = b0 + t; k < blocks.size(); k += T) {
          Block& B = blocks[k];
          Rng r(seed ^ (0x9E3779B97F4A7C15ull * (next_block + (k - b0) + 1)));
          B.blob.reserve((size_t)PAR_BLOCK * (dmax * 6 + 4));
          B.off.reserve(PAR_BLOCK + 1);
          B.h.resize(PAR_BLOCK);
          for (uint32_t i = 0; i < PAR_BLOCK; ++i) {
            gen_filter(r, voc, f, dmin, dmax, wc_frac, p_plus, p_hash, p_empty);
            B.blob += f;
            B.off.push_back((uint32_t)B.blob.size());
            B.h[i] = std::hash<std::string_view>()(std::string_view(f));
          }
          B.keep.assign(PAR_BLOCK, 0);
        }
      });
    for (auto& x : th) x.join();
    th.clear();
    // dedup: partition t owns the hashes = t mod T, walks the candidates in order
    for (unsigned t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (size_t k = b0; k < blocks.size(); ++k) {
          Block& B = blocks[k];
          for (uint32_t i = 0; i < PAR_BLOCK; ++i) {
            if (B.h[i] % T != t) continue;
            std::string_view v(B.blob.data() + B.off[i], B.off[i + 1] - B.off[i]);
            if (part[t].insert(v).second) B.keep[i] = 1;
          }
        }
      });
    for (auto& x : th) x.join();
    for (size_t k = b0; k < blocks.size(); ++k) {
      for (uint32_t i = 0; i < PAR_BLOCK; ++i) have += blocks[k].keep[i];
      std::vector<uint64_t>().swap(blocks[k].h);
    }
    next_block += want;
  }
  // the first n unique candidates, in candidate order
  Strings res;
  uint64_t total = 0, taken = 0;
  for (auto& B : blocks)
    for (uint32_t i = 0; i < PAR_BLOCK && taken < n; ++i)
      if (B.keep[i]) {
        total += B.off[i + 1] - B.off[i];
        ++taken;
      }
  if (total > 0xFFFFFFF0ull) return -1;   // offsets are u32 (the C-ABI's egm_table_build)
  std::vector<std::unordered_set<std::string_view>>().swap(part);
  res.blob.reserve(total);
  res.off.reserve((size_t)n + 1);
  taken = 0;
  for (auto& B : blocks) {
    for (uint32_t i = 0; i < PAR_BLOCK && taken < n; ++i)
      if (B.keep[i]) {
        res.blob.append(B.blob.data() + B.off[i], B.off[i + 1] - B.off[i]);
        res.off.push_back((uint32_t)res.blob.size());
        ++taken;
      }
    std::string().swap(B.blob);
  }
  return export_strings(res, out);
}

// n unique filters.  A "wildcard" filter (fraction wc_frac) has each level '+'
// with p_plus and its last level '#' with p_hash, forced to carry at least one
// wildcard; the rest are all-literal.  p_empty: a literal level is ''.
int egs_filters(uint64_t seed, uint32_t n, int dmin, int dmax, double wc_frac, double p_plus, double p_hash,
                double p_empty, double zipf_s, uint32_t vmax, egs_strings* out) {
  if (!out || dmin < 1 || dmax < dmin) return -1;
  if (n > PAR_MIN) return egs_filters_par(seed, n, dmin, dmax, wc_frac, p_plus, p_hash, p_empty, zipf_s, vmax, out);
  Rng r(seed);
  Vocab voc(zipf_s, vmax);
  Strings res;
  res.blob.reserve((size_t)n * (dmax * 6 + 4));
  res.off.reserve((size_t)n + 1);
  std::unordered_set<std::string_view> seen;
  seen.reserve((size_t)n * 2);
  std::vector<std::string> pending;  // keep storage stable: views point into `store`
  std::string f;
  uint64_t attempts = 0;
  std::vector<std::string> store;
  store.reserve(n);
  while (store.size() < n && attempts < (uint64_t)n * 50) {
    ++attempts;
    gen_filter(r, voc, f, dmin, dmax, wc_frac, p_plus, p_hash, p_empty);
    store.push_back(f);
    if (!seen.insert(std::string_view(store.back())).second) {
      store.pop_back();
      continue;
    }
  }
  // string_views in `seen` may dangle after reallocation; we reserved n so no realloc
  uint64_t total = 0;
  for (const auto& s : store) total += s.size();
  if (total > 0xFFFFFFF0ull) return -1;   // offsets are u32 (the C-ABI's egm_table_build)
  for (const auto& s : store) res.push(s);
  return export_strings(res, out);
}

// n topics: fraction p_from_filter instantiated from a random filter ('+' ->
// a vocabulary word of that level, '#' -> 0..3 words), the rest independent;
// a fraction p_sys starts with "$SYS".
int egs_topics(uint64_t seed, const egs_strings* filters, uint32_t n, int dmin, int dmax, double p_from_filter,
               double p_sys, double p_empty, double zipf_s, uint32_t vmax, egs_strings* out) {
  if (!out || dmin < 1 || dmax < dmin) return -1;
  Rng r(seed ^ 0x70b1c5ull);
  Vocab voc(zipf_s, vmax);
  Strings res;
  res.blob.reserve((size_t)n * (dmax * 7 + 4));
  res.off.reserve((size_t)n + 1);
  std::string t;
  const uint32_t nf = filters ? filters->n : 0;
  for (uint32_t i = 0; i < n; ++i) {
    t.clear();
    int level = 0;
    auto lit = [&](int l) {
      if (r.uni() < p_empty) return;
      put_word(t, l, voc.sample(r, l));
    };
    if (nf && r.uni() < p_from_filter) {
      uint32_t k = r.below(nf);
      const char* p = (const char*)filters->blob + filters->off[k];
      uint32_t len = filters->off[k + 1] - filters->off[k];
      uint32_t ws = 0;
      for (uint32_t j = 0; j <= len; ++j) {
        if (j < len && p[j] != '/') continue;
        uint32_t wl = j - ws;
        if (wl == 1 && p[ws] == '+') {
          if (level) t += '/';
          lit(level++);
        } else if (wl == 1 && p[ws] == '#') {
          int extra = (int)r.below(4);
          for (int e = 0; e < extra; ++e) {
            if (level) t += '/';
            lit(level++);
          }
        } else {
          if (level) t += '/';
          t.append(p + ws, wl);
          ++level;
        }
        ws = j + 1;
      }
      if (level == 0) lit(level++);  // "#" with 0 extra words -> one word
    } else {
      int d = r.range(dmin, dmax);
      for (int l = 0; l < d; ++l) {
        if (l) t += '/';
        lit(l);
      }
    }
    if (r.uni() < p_sys) {  // replace the first word by $SYS
      size_t sl = t.find('/');
      t = std::string("$SYS") + (sl == std::string::npos ? std::string() : t.substr(sl));
    }
    res.push(t);
  }
  return export_strings(res, out);
}

// Subscriber table for the fan-out configs: per filter 1 + Poisson(lambda)
// local subscribers, a fraction p_big of filters with n_big subscribers, a
// fraction p_share of filters subscribed through $share groups instead
// (group ids g0..g{groups-1}, 2..16 members; one (filter, group) entry).
// Output CSR row[n+1] (u64) and ids (u32; group ids carry bit 31).
int egs_subscribers(uint64_t seed, uint32_t n, double lambda, double p_big, uint32_t n_big, double p_share,
                    uint32_t groups, uint64_t** row_out, uint32_t** ids_out, uint64_t* total_out) {
  Rng r(seed ^ 0x5b5b5bull);
  std::vector<uint64_t> row(n + 1, 0);
  std::vector<uint32_t> ids;
  ids.reserve((size_t)n * 2 + 16);
  const double L = std::exp(-lambda);
  uint32_t next_sub = 0;
  for (uint32_t f = 0; f < n; ++f) {
    if (r.uni() < p_share) {
      uint32_t g = r.below(groups ? groups : 1);
      ids.push_back(0x80000000u | g);
      // a second group on the same filter with small probability
      if (r.uni() < 0.1) {
        uint32_t g2 = r.below(groups ? groups : 1);
        if (g2 != g) ids.push_back(0x80000000u | g2);
      }
    } else {
      uint32_t k;
      if (r.uni() < p_big) {
        k = n_big;
      } else {  // 1 + Poisson(lambda) (Knuth)
        uint32_t x = 0;
        double p = r.uni();
        while (p > L) {
          ++x;
          p *= r.uni();
        }
        k = 1 + x;
      }
      for (uint32_t j = 0; j < k; ++j) ids.push_back((next_sub++) & 0x7FFFFFFFu);
    }
    row[f + 1] = ids.size();
  }
  *row_out = (uint64_t*)malloc(row.size() * 8);
  *ids_out = (uint32_t*)malloc(ids.size() * 4 + 4);
  if (!*row_out || !*ids_out) return -2;
  memcpy(*row_out, row.data(), row.size() * 8);
  memcpy(*ids_out, ids.data(), ids.size() * 4);
  *total_out = ids.size();
  return 0;
}

// The strings idx[0..m) of a set, in that order (shard tables, samples).
int egs_subset(const egs_strings* in, const uint32_t* idx, uint32_t m, egs_strings* out) {
  if (!in || !out || (m && !idx)) return -1;
  uint64_t total = 0;
  for (uint32_t k = 0; k < m; ++k) {
    if (idx[k] >= in->n) return -1;
    total += in->off[idx[k] + 1] - in->off[idx[k]];
  }
  if (total > 0xFFFFFFF0ull) return -1;
  out->n = m;
  out->bytes = total;
  out->blob = (uint8_t*)malloc(total + 16);
  out->off = (uint32_t*)malloc(((size_t)m + 1) * 4);
  if (!out->blob || !out->off) return -2;
  uint64_t o = 0;
  out->off[0] = 0;
  for (uint32_t k = 0; k < m; ++k) {
    const uint32_t a = in->off[idx[k]], len = in->off[idx[k] + 1] - a;
    memcpy(out->blob + o, in->blob + a, len);
    o += len;
    out->off[k + 1] = (uint32_t)o;
  }
  return 0;
}

void egs_free_ptr(void* p) { free(p); }

}  // extern "C"
