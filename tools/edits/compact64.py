"""One-off source edit: k_compact back to 64-piece windows (the 256-piece
window measured no faster), keeping the contiguous window ranges."""
p = '/root/repo/emqx_amd/csrc/egm_kernels.hip'
s = open(p).read()
a = s.index('constexpr int COMPACT_WAVES = 4;')
b = s.index('// ------------------------------------------------------------- launchers ----')
new = '''constexpr int COMPACT_WAVES = 4;
__global__ __launch_bounds__(64 * COMPACT_WAVES) void k_compact(const uint4* __restrict__ pieces,
                                                                const uint8_t* __restrict__ tfl,
                                                                const uint32_t* __restrict__ ids_tmp, uint32_t n,
                                                                const uint64_t* __restrict__ row_ptr,
                                                                uint32_t* __restrict__ ids, uint64_t ids_cap,
                                                                uint64_t pieces_cap, MatchStats* stats) {
  __shared__ uint32_t s_scan[COMPACT_WAVES][64];
  __shared__ uint32_t s_src[COMPACT_WAVES][64];
  __shared__ uint64_t s_dst[COMPACT_WAVES][64];
  const uint64_t total = row_ptr[n];
  if (blockIdx.x == 0 && threadIdx.x == 0) stats->total_ids = total;
  if (stats->overflow) return;
  if (total > ids_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&stats->overflow, 2u);
    return;
  }
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t np = min((uint64_t)stats->pieces, pieces_cap);
  const bool any_heavy = stats->n_deferred != 0;   // else no light piece can be stale
  // a contiguous range of windows per wave (not a grid stride): the flushes
  // of one chunk sit next to each other in pieces[], so one wave completes
  // the cache lines of a chunk's rows
  const uint64_t nwin = (np + 63) / 64, nw = (uint64_t)gridDim.x * COMPACT_WAVES;
  const uint64_t per = (nwin + nw - 1) / nw, me = (uint64_t)blockIdx.x * COMPACT_WAVES + wave;
  const uint64_t wend = min(nwin, (me + 1) * per) * 64;
  for (uint64_t w0 = me * per * 64; w0 < wend; w0 += 64) {
    const uint64_t i = w0 + lane;
    const uint4 pc = pieces[min(i, np - 1)];   // unconditional (a load under a branch is waited for at once)
    uint32_t c = i < np ? (pc.y & ~HEAVY_PIECE) : 0u;
    const uint64_t rp = row_ptr[c ? pc.x : 0u];
    if (any_heavy && c && (tfl[pc.x] & TF_HEAVY) && !(pc.y & HEAVY_PIECE)) c = 0;
    uint32_t tot;
    const uint32_t ex = wave_excl_scan(c, lane, &tot);
    s_scan[wave][lane] = ex;
    s_src[wave][lane] = pc.z;
    s_dst[wave][lane] = rp + pc.w;
    wave_sync();
    // four ids per lane per round: their searches, loads and stores overlap
    for (uint32_t q0 = lane; q0 < tot; q0 += 256) {
      uint32_t v[4];
      uint64_t d[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t q = min(q0 + 64u * r, tot - 1);
        uint32_t k = 0;
#pragma unroll
        for (uint32_t step = 32; step >= 1; step >>= 1)
          if (s_scan[wave][k + step] <= q) k += step;
        const uint32_t o = q - s_scan[wave][k];
        d[r] = s_dst[wave][k] + o;
        v[r] = ids_tmp[s_src[wave][k] + o];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (q0 + 64u * r < tot) ids[d[r]] = v[r];
    }
    wave_sync();
  }
}

'''
s = s[:a] + new + s[b:]
open(p, 'w').write(s)
print("ok")
