// HBM granule of random reads on MI355X: does reading
// one 64-B half of a random 128-B line cost the memory system a 64-B or a
// 128-B fetch?  Each lane reads W16 x 16 B at the start of a random slot of
// S16 x 16 B in a 2.8 GB table (HBM, 11x the Infinity Cache), K independent
// reads in flight per lane.  Run it under `rocprofv3 --pmc FETCH_SIZE` and
// divide each kernel's FETCH_SIZE by its reads (printed below): the slot
// shapes compared are
//   W16=4 S16=4   64 B of a random 64-B line (the walk's bucket half today)
//   W16=4 S16=8   the first 64 B of a random 128-B line
//   W16=8 S16=8   a whole random 128-B line
//   W16=2 S16=8   32 B (one edge slot) of a random 128-B line
//   W16=1 S16=8   16 B of a random 128-B line
// Build: hipcc --offload-arch=gfx950 -O3 tools/granule.hip -o tools/granule
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

template <int K, int W16, int S16, int G = 1, bool STRIDED = false>
__global__ __launch_bounds__(64) void k_granule(const uint4* __restrict__ t, uint64_t nslots, int iters,
                                                uint32_t* out) {
  // G lanes read the same slot (G = 64: the whole wave one line per read):
  // G lanes in a row, or (STRIDED) lanes 64/G apart
  const uint64_t gid = blockIdx.x * 64ull + (STRIDED ? threadIdx.x % (64 / G) : threadIdx.x / G);
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    uint4 v[K][W16];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t s = mix(gid * 1315423911ull + (uint64_t)i * K + k) % nslots;
#pragma unroll
      for (int w = 0; w < W16; ++w) v[k][w] = t[s * S16 + w];
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int w = 0; w < W16; ++w) acc ^= v[k][w].x ^ v[k][w].y ^ v[k][w].z ^ v[k][w].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int K, int W16, int S16, int G = 1, bool STRIDED = false>
static void run(const uint4* t, uint64_t bytes, int blocks, int iters, uint32_t* out) {
  const uint64_t nslots = bytes / (16 * S16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_granule<K, W16, S16, G, STRIDED>), dim3(blocks), dim3(64), 0, 0, t, nslots, 1, out);   // warm
  hipEventRecord(a);
  hipLaunchKernelGGL((k_granule<K, W16, S16, G, STRIDED>), dim3(blocks), dim3(64), 0, 0, t, nslots, iters, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double reads = (double)blocks * 64 * iters * K;
  const double warm_reads = (double)blocks * 64 * 1 * K;
  printf("{\"kernel\": \"k_granule<%d, %d, %d, %d, %d>\", \"read_bytes\": %d, \"slot_bytes\": %d, \"K\": %d, "
         "\"lanes_per_line\": %d, \"strided\": %d, \"reads_timed\": %.0f, \"reads_per_dispatch\": [%.0f, %.0f], \"ms\": %.3f, "
         "\"G_reads_per_s\": %.2f, \"GB_per_s_read\": %.1f}\n",
         K, W16, S16, G, (int)STRIDED, 16 * W16, 16 * S16, K, G, (int)STRIDED, reads, warm_reads, reads, ms, reads / ms / 1e6,
         reads * 16 * W16 / ms / 1e6);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const uint64_t big = 2800ull << 20;
  uint4* t = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&t, big) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  hipMemset(t, 1, big);
  hipDeviceSynchronize();
  const int blocks = 16384, iters = 16;
  run<4, 4, 4>(t, big, blocks, iters, out);
  run<4, 4, 8>(t, big, blocks, iters, out);
  run<4, 8, 8>(t, big, blocks, iters, out);
  run<4, 2, 8>(t, big, blocks, iters, out);
  run<4, 1, 8>(t, big, blocks, iters, out);
  run<1, 4, 4>(t, big, blocks, iters, out);
  run<1, 4, 8>(t, big, blocks, iters, out);
  run<1, 8, 8>(t, big, blocks, iters, out);
  run<1, 2, 8>(t, big, blocks, iters, out);
  // lanes sharing a line inside one load instruction: does the CU merge them
  // into one request (count TCC_REQ per read under rocprofv3 --pmc)?
  run<4, 4, 4, 4>(t, big, blocks, iters, out);
  run<4, 4, 4, 16>(t, big, blocks, iters, out);
  run<4, 4, 4, 64>(t, big, blocks, iters, out);
  run<4, 1, 4, 64>(t, big, blocks, iters, out);
  // the same sharing with the sharing lanes spread over the wave (a walk's
  // duplicates are not in adjacent lanes)
  run<4, 4, 4, 4, true>(t, big, blocks, iters, out);
  run<4, 4, 4, 16, true>(t, big, blocks, iters, out);
  run<4, 1, 4, 4, true>(t, big, blocks, iters, out);
  hipDeviceSynchronize();
  return 0;
}
