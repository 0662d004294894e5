"""One-off source edit: always stage topic words in LDS (sub-chunks for deep
chunks) so that the walk's finish() issues no global loads."""
p = '/root/repo/emqx_amd/csrc/egm_kernels.hip'
s = open(p).read()
a = s.index('    // ---- topic info; words staged as [topic][level] with a chunk-wide stride ----')
b = s.index('// Admit new topics while the stack is short')
new = '''    // ---- topic info (lane j: topic t0 + j) ----
    uint32_t dmax = 0;
    {
      uint32_t D = 0, f = 0;
      if (lane < nt) {
        D = w.lv[t0 + lane];
        f = w.tfl[t0 + lane];
      }
      dmax = D;
      L.tinfo[lane] = D | (f << 24);
      L.cnt[lane] = 0;
      L.fcnt[lane] = 0;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) dmax = max(dmax, (uint32_t)__shfl_xor(dmax, d, 64));
    // Words are always staged in LDS as [topic][level] (finish() must not
    // load from global memory, see issue()): a chunk of deep topics is walked
    // as sub-chunks of S topics with S * dmax <= WALK_WORDS.  Topics deeper
    // than WALK_WORDS levels go to the heavy kernel.
    uint32_t S = WALK_CHUNK;
    while (S > 1 && S * dmax > (uint32_t)WALK_WORDS) S >>= 1;
    uint32_t sp = 0, nstage = 0;
    bool ovf = (w.debug & DEBUG_FORCE_HEAVY) != 0 || dmax > (uint32_t)WALK_WORDS;
    wave_sync();
    for (uint32_t sub = 0; sub < nt && !ovf; sub += S) {
    const uint32_t end = min(sub + S, nt);
    if (lane < end - sub) {
      const uint32_t j = sub + lane, D = L.tinfo[j] & 0xFFFFFFu;
      const uint32_t* src = w.wid + off[t0 + j] + t0 + j;
      uint32_t* dst = L.words + lane * dmax;
      L.tbase[j] = lane * dmax;
      uint32_t i = 0;
      for (; i + 4 <= D; i += 4) {
        uint32_t a0 = src[i], a1 = src[i + 1], a2 = src[i + 2], a3 = src[i + 3];
        dst[i] = a0;
        dst[i + 1] = a1;
        dst[i + 2] = a2;
        dst[i + 3] = a3;
      }
      for (; i < D; ++i) dst[i] = src[i];
    }
    wave_sync();
    uint32_t next = sub;

'''
s = s[:a] + new + s[b:]


def rep(old, new_):
    global s
    assert old in s, old[:80]
    s = s.replace(old, new_)


rep('''    if (sp < 64u && next < nt) {                                                                       \\
      const uint32_t k = min(64u - sp, nt - next);                                                     \\''',
    '''    if (sp < 64u && next < end) {                                                                      \\
      const uint32_t k = min(64u - sp, end - next);                                                    \\''')
rep('''      if (ovf || (!tb && sp == 0 && next >= nt)) break;''',
    '''      if (ovf || (!tb && sp == 0 && next >= end)) break;''')
rep('''      if (ovf || (!ta && sp == 0 && next >= nt)) break;
    }''', '''      if (ovf || (!ta && sp == 0 && next >= end)) break;
    }
    }  // sub-chunks''')
rep('''__device__ __forceinline__ uint32_t word_at(const WaveLds& L, const MatchWork& w, bool staged, uint32_t tt,
                                            uint32_t level) {
  if (staged) return L.words[min(L.tbase[tt] + level, (uint32_t)WALK_WORDS - 1)];
  return w.wid[L.tbase[tt] + level];
}''', '''__device__ __forceinline__ uint32_t word_at(const WaveLds& L, uint32_t tt, uint32_t level) {
  return L.words[min(L.tbase[tt] + level, (uint32_t)WALK_WORDS - 1)];
}''')
rep('__device__ __forceinline__ void issue(const DevTable& tab, const WaveLds& L, bool staged, uint32_t ws, Pend& p) {',
    '__device__ __forceinline__ void issue(const DevTable& tab, const WaveLds& L, Pend& p) {')
rep('''  // LDS reads overlapping the global ones: the topic's info and, when the
  // words are staged, the next level's word (clamped; used only if level+1 < D)
  const uint32_t tt = (meta >> MT_SHIFT) & 0x7Fu, level = meta & LEVEL_MAX;
  p.ti = L.tinfo[tt];
  p.nw = L.words[min(tt * ws + level + 1, (uint32_t)WALK_WORDS - 1)];
  (void)staged;''', '''  // LDS reads overlapping the global ones: the topic's info and the next
  // level's word (clamped; used only if level + 1 < D)
  const uint32_t tt = (meta >> MT_SHIFT) & 0x7Fu, level = meta & LEVEL_MAX;
  p.ti = L.tinfo[tt];
  p.nw = word_at(L, tt, level + 1);''')
rep('''__device__ __forceinline__ void finish(const DevTable& tab, int mode, const WaveLds& L, const MatchWork& w,
                                       bool staged, Pend& p, Out& o) {''',
    '''__device__ __forceinline__ void finish(const DevTable& tab, int mode, Pend& p, Out& o) {''')
rep('''  uint32_t nw = p.nw;
  if (!staged) nw = leaf ? WID_NONE : w.wid[L.tbase[tt] + nl];
''', '''  const uint32_t nw = p.nw;
''')
rep('''__device__ bool exact_walk(const DevTable& tab, const WaveLds& L, const MatchWork& w, bool staged, uint32_t j,
                           uint32_t D, uint32_t* fid) {''',
    '''__device__ bool exact_walk(const DevTable& tab, const WaveLds& L, uint32_t j, uint32_t D, uint32_t* fid) {''')
rep('''    const uint32_t wd = word_at(L, w, staged, j, l);''', '''    const uint32_t wd = word_at(L, j, l);''')
rep('''em = exact_walk(tab, L, w, staged, j, D, &fid);''', '''em = exact_walk(tab, L, j, D, &fid);''')
rep('''const uint32_t w0 = word_at(L, w, staged, j, 0);''', '''const uint32_t w0 = word_at(L, j, 0);''')
rep('''      issue(tab, L, staged, ws, P);''', '''      issue(tab, L, P);''')
rep('''      finish(tab, mode, L, w, staged, P, o);''', '''      finish(tab, mode, P, o);''')
rep('''static_assert(WALK_CHUNK <= 128, "t field is 7 bits");''',
    '''static_assert(WALK_CHUNK == 64, "one topic per lane in the chunk prologue");''')
open(p, 'w').write(s)
print("ok")
