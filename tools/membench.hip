// Random-read ceiling of the MI355X memory system for the walk's access
// shape: each lane reads WIDTH bytes at a random, WIDTH-aligned offset of a
// table of TABLE bytes, K independent reads in flight per lane.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}

template <int K, int W16>
__global__ __launch_bounds__(64) void k_rand(const uint4* __restrict__ t, uint64_t nslots, int iters, uint32_t* out, int group) {
  const uint64_t gid = (blockIdx.x * 64ull + threadIdx.x) / group;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    uint4 v[K][W16];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t s = mix(gid * 1315423911ull + (uint64_t)i * K + k) % nslots;
#pragma unroll
      for (int w = 0; w < W16; ++w) v[k][w] = t[s * W16 + w];
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int w = 0; w < W16; ++w) acc ^= v[k][w].x ^ v[k][w].y ^ v[k][w].z ^ v[k][w].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int K, int W16>
void run(const uint4* t, uint64_t bytes, int blocks, int iters, uint32_t* out, int group = 1) {
  const uint64_t nslots = bytes / (16 * W16);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  k_rand<K, W16><<<blocks, 64>>>(t, nslots, 2, out, group);
  hipEventRecord(a);
  k_rand<K, W16><<<blocks, 64>>>(t, nslots, iters, out, group);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double reqs = (double)blocks * 64 * iters * K;
  printf("group %2d table %6.0f MB width %3d B K=%d blocks %6d: %7.2f G reads/s  %7.1f GB/s (%.2f ms)\n", group, bytes / 1e6, 16 * W16,
         K, blocks, reqs / ms / 1e6, reqs * 16 * W16 / ms / 1e6, ms);
  (void)0;
}

int main() {
  const uint64_t big = 2800ull << 20;
  uint4* t; uint32_t* out;
  if (hipMalloc(&t, big) != hipSuccess) return 1;
  hipMalloc(&out, 4);
  hipMemset(t, 1, big);
  for (uint64_t bytes : {(uint64_t)2 << 20, (uint64_t)16 << 20, (uint64_t)64 << 20, big}) {
    for (int g : {1, 4, 16, 64}) {
      run<4, 4>(t, bytes, 16384, 16, out, g);
      run<4, 2>(t, bytes, 16384, 16, out, g);
    }
  }
  return 0;
}
