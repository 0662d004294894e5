// What bounds k_walk?  A synthetic wave loop with the
// walk's memory mix, dependent rounds and a tunable amount of VALU between
// them, at a tunable number of waves per CU:
//   * per round every lane reads one 64-B "bucket" line (four 16-B loads) and
//     one 16-B "record" — 4 lanes share each line, so a wave requests 32
//     distinct lines per round (the walk: ~35 per iteration, §4.1.2);
//   * 35 % of the lines come from a 2 MB hot set (L2 hits), 65 % are random
//     lines of a 2.8 GB table (misses), the walk's hit ratio;
//   * the next round's addresses depend on this round's data (a walk pops
//     the children its reads produced);
//   * NV VALU instructions (inline asm, exact count) run between the rounds;
//   * LDS is allocated to set waves per CU (10 KB = the walk's 16 per CU).
// Reports rounds/s, L2 requests/s and misses/s per configuration; the walk at
// C2 makes 7.32M iterations with ~314 VALU each and 326M misses in ~10.1 ms.
// Build: hipcc --offload-arch=gfx950 -O3 tools/walkmix.hip -o tools/walkmix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t fmix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

template <int NV>
__device__ __forceinline__ void valu(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
#pragma unroll
  for (int i = 0; i < NV / 4; ++i) {
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b) : "v"(c));
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(d));
    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(a));
  }
}

template <int NV, int LDS_BYTES, int SHARE = 4, bool STORES = false>
__global__ __launch_bounds__(64) void k_mix(const uint4* __restrict__ t, uint32_t nlines, uint32_t hot_lines, int rounds,
                                            uint32_t* out) {
  __shared__ uint32_t pad[LDS_BYTES / 4];
  const uint32_t lane = threadIdx.x;
  uint32_t x = fmix(blockIdx.x * 64u + lane + 1u);
  uint32_t a = x, b = x ^ 1u, c = x ^ 2u, d = x ^ 3u;
  pad[lane] = x;
  for (int r = 0; r < rounds; ++r) {
    // SHARE lanes share a bucket line and a record line: 2 x 64 / SHARE distinct lines per wave
    const uint32_t kb = fmix(__shfl(x, (int)(lane & ~(uint32_t)(SHARE - 1)), 64) + (uint32_t)r * 0x9E3779B9u);
    const uint32_t kr = fmix(kb ^ 0x5bd1e995u);
    const uint32_t lb = (kb & 1023u) < 358u ? (kb >> 10) % hot_lines : kb % nlines;
    const uint32_t lr = (kr & 1023u) < 358u ? (kr >> 10) % hot_lines : kr % nlines;
    const uint4* pb = t + (uint64_t)lb * 4;
    const uint4 v0 = pb[0], v1 = pb[1], v2 = pb[2], v3 = pb[3];
    const uint4 w = t[(uint64_t)lr * 4 + (lane & 3u)];
    x ^= v0.x ^ v1.y ^ v2.z ^ v3.w ^ w.x;
    a += x;
    valu<NV>(a, b, c, d);
    x += (a ^ b ^ c ^ d) & 1u;
    if (STORES && (lane & 7u) == 0) {   // ~8 line writes per round (the walk's flush stores: 8.6 per iteration)
      uint32_t* o = out + 64 + ((uint64_t)fmix(x + lane) % (nlines / 16 - 8)) * 16;
      o[0] = x;
    }
  }
  if (x == 0x12345678u) out[0] = x + pad[(lane + 1) & 63];
}

template <int NV, int LDS_BYTES, int SHARE = 4, bool STORES = false>
static void run(const uint4* t, uint32_t nlines, uint32_t hot_lines, int wpc, uint32_t* out) {
  const int blocks = 256 * wpc, rounds = 1500;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_mix<NV, LDS_BYTES, SHARE, STORES>), dim3(blocks), dim3(64), 0, 0, t, nlines, hot_lines, 50, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_mix<NV, LDS_BYTES, SHARE, STORES>), dim3(blocks), dim3(64), 0, 0, t, nlines, hot_lines, rounds,
                     out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double wr = (double)blocks * rounds;   // wave-rounds
  const double req = wr * 2.0 * 64 / SHARE, miss = req * 0.65;
  printf("{\"lines_per_round\": %d, \"stores\": %d, \"valu_per_round\": %d, \"lds_bytes_per_wave\": %d, "
         "\"waves_per_cu_target\": %d, \"ms\": %.3f, "
         "\"M_rounds_per_s\": %.1f, \"G_lines_per_s\": %.2f, \"G_misses_per_s\": %.2f, \"ms_for_7.32M_rounds\": %.2f}\n",
         2 * 64 / SHARE, (int)STORES, NV, LDS_BYTES, wpc, ms, wr / ms / 1e3, req / ms / 1e6, miss / ms / 1e6,
         7.32e6 / (wr / ms));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <int LDS_BYTES>
static void sweep(const uint4* t, uint32_t nlines, uint32_t hot, int wpc, uint32_t* out) {
  run<0, LDS_BYTES>(t, nlines, hot, wpc, out);
  run<100, LDS_BYTES>(t, nlines, hot, wpc, out);
  run<200, LDS_BYTES>(t, nlines, hot, wpc, out);
  run<300, LDS_BYTES>(t, nlines, hot, wpc, out);
  run<450, LDS_BYTES>(t, nlines, hot, wpc, out);
  run<600, LDS_BYTES>(t, nlines, hot, wpc, out);
}

int main(int argc, char**) {
  const uint64_t big = 2800ull << 20;
  uint4* t = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&t, big) != hipSuccess || hipMalloc(&out, (big / 16) + 4096) != hipSuccess) return 1;
  hipMemset(t, 1, big);
  hipDeviceSynchronize();
  const uint32_t nlines = (uint32_t)(big / 64), hot = (2u << 20) / 64;
  if (argc > 1) {   // round 4, second probe: the walk's measured 68 L2 requests per iteration
    // (498M per launch / 7.32M iterations) instead of the 32 distinct lines of the emulation,
    // and its flush stores, at the walk's 16 waves per CU
    run<0, 10240, 2>(t, nlines, hot, 16, out);
    run<300, 10240, 2>(t, nlines, hot, 16, out);
    run<0, 10240, 2, true>(t, nlines, hot, 16, out);
    run<300, 10240, 2, true>(t, nlines, hot, 16, out);
    run<300, 10240, 4, true>(t, nlines, hot, 16, out);
    run<600, 10240, 2, true>(t, nlines, hot, 16, out);
    hipDeviceSynchronize();
    return 0;
  }
  sweep<20480>(t, nlines, hot, 8, out);    // 8 waves per CU
  sweep<13312>(t, nlines, hot, 12, out);   // 12
  sweep<10240>(t, nlines, hot, 16, out);   // 16: the walk
  sweep<8192>(t, nlines, hot, 20, out);    // 20
  sweep<6144>(t, nlines, hot, 24, out);    // 24
  sweep<4096>(t, nlines, hot, 32, out);    // 32
  hipDeviceSynchronize();
  return 0;
}
