// Cost of a device radix sort of (u32 key, u32 topic) pairs at batch sizes
// (the question: can a locality sort of the batch pay for itself in k_walk?).
//   hipcc --offload-arch=gfx950 -O3 tools/sortbench.hip -o tools/sortbench && tools/sortbench
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <random>

int main() {
  const int n = 10000000;
  std::vector<uint32_t> hk(n), hv(n);
  std::mt19937 rng(1);
  for (int i = 0; i < n; ++i) {
    hk[i] = rng();
    hv[i] = i;
  }
  uint32_t *k0, *k1, *v0, *v1;
  hipMalloc(&k0, n * 4);
  hipMalloc(&k1, n * 4);
  hipMalloc(&v0, n * 4);
  hipMalloc(&v1, n * 4);
  hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice);
  for (int bits : {16, 24, 32}) {
    size_t tmp = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k0, k1, v0, v1, n, 0, bits);
    void* t = nullptr;
    hipMalloc(&t, tmp);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipcub::DeviceRadixSort::SortPairs(t, tmp, k0, k1, v0, v1, n, 0, bits);
    hipEventRecord(a);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipcub::DeviceRadixSort::SortPairs(t, tmp, k0, k1, v0, v1, n, 0, bits);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"n\": %d, \"key_bits\": %d, \"ms\": %.4f, \"temp_bytes\": %zu}\n", n, bits, ms / reps, tmp);
    hipFree(t);
  }
  return 0;
}
