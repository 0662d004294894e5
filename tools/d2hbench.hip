// Device -> pinned host copy rates on MI355X for the host-visible path's
// result (212 MB per 1M-topic batch moved at 31 GB/s).
// Compares, for 200 MB: one hipMemcpyAsync; the same split over 2 / 4
// streams; a kernel storing 16 B per lane straight into the pinned buffer
// (zero-copy); and the H2D direction of the inbound blob (40 MB).
// Build: hipcc --offload-arch=gfx950 -O3 tools/d2hbench.hip -o tools/d2hbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_store_host(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = src[i];
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (u32x4*)(dst + i));
  }
}

__global__ __launch_bounds__(256) void k_load_host(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

static double time_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  const size_t bytes = 200ull << 20, in_bytes = 40ull << 20;
  void *d = nullptr, *h = nullptr, *hin = nullptr, *din = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&hin, in_bytes, hipHostMallocDefault));
  CK(hipMalloc(&din, in_bytes));
  CK(hipMemset(d, 7, bytes));
  hipStream_t s[4];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    for (int ns : {1, 2, 4}) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s[0]));
      for (int k = 1; k < ns; ++k) CK(hipStreamWaitEvent(s[k], e0, 0));
      const size_t per = bytes / ns;
      for (int k = 0; k < ns; ++k)
        CK(hipMemcpyAsync((char*)h + k * per, (char*)d + k * per, per, hipMemcpyDeviceToHost, s[k]));
      for (int k = 1; k < ns; ++k) {
        hipEvent_t ek;
        CK(hipEventCreateWithFlags(&ek, hipEventDisableTiming));
        CK(hipEventRecord(ek, s[k]));
        CK(hipStreamWaitEvent(s[0], ek, 0));
        CK(hipEventDestroy(ek));
      }
      CK(hipEventRecord(e1, s[0]));
      CK(hipEventSynchronize(e1));
      const double ms = time_ms(e0, e1);
      printf("{\"what\": \"memcpy_d2h\", \"streams\": %d, \"MB\": %zu, \"ms\": %.3f, \"GB_per_s\": %.1f}\n", ns,
             bytes >> 20, ms, bytes / ms / 1e6);
    }
    for (int blocks : {256, 1024, 4096}) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s[0]));
      hipLaunchKernelGGL(k_store_host, dim3(blocks), dim3(256), 0, s[0], (const uint4*)d, (uint4*)h, bytes / 16);
      CK(hipEventRecord(e1, s[0]));
      CK(hipEventSynchronize(e1));
      const double ms = time_ms(e0, e1);
      printf("{\"what\": \"kernel_store_to_pinned\", \"blocks\": %d, \"MB\": %zu, \"ms\": %.3f, \"GB_per_s\": %.1f}\n",
             blocks, bytes >> 20, ms, bytes / ms / 1e6);
    }
    for (int ns : {1, 2}) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s[0]));
      for (int k = 1; k < ns; ++k) CK(hipStreamWaitEvent(s[k], e0, 0));
      const size_t per = in_bytes / ns;
      for (int k = 0; k < ns; ++k)
        CK(hipMemcpyAsync((char*)din + k * per, (char*)hin + k * per, per, hipMemcpyHostToDevice, s[k]));
      for (int k = 1; k < ns; ++k) {
        hipEvent_t ek;
        CK(hipEventCreateWithFlags(&ek, hipEventDisableTiming));
        CK(hipEventRecord(ek, s[k]));
        CK(hipStreamWaitEvent(s[0], ek, 0));
        CK(hipEventDestroy(ek));
      }
      CK(hipEventRecord(e1, s[0]));
      CK(hipEventSynchronize(e1));
      const double ms = time_ms(e0, e1);
      printf("{\"what\": \"memcpy_h2d\", \"streams\": %d, \"MB\": %zu, \"ms\": %.3f, \"GB_per_s\": %.1f}\n", ns,
             in_bytes >> 20, ms, in_bytes / ms / 1e6);
    }
    {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s[0]));
      hipLaunchKernelGGL(k_load_host, dim3(1024), dim3(256), 0, s[0], (const uint4*)hin, (uint4*)din, in_bytes / 16);
      CK(hipEventRecord(e1, s[0]));
      CK(hipEventSynchronize(e1));
      const double ms = time_ms(e0, e1);
      printf("{\"what\": \"kernel_load_from_pinned\", \"blocks\": 1024, \"MB\": %zu, \"ms\": %.3f, \"GB_per_s\": %.1f}\n",
             in_bytes >> 20, ms, in_bytes / ms / 1e6);
    }
    // both directions at once: the pipeline's batch k D2H beside batch k+1 H2D
    {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s[0]));
      CK(hipStreamWaitEvent(s[1], e0, 0));
      CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s[0]));
      CK(hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, s[1]));
      hipEvent_t ek;
      CK(hipEventCreateWithFlags(&ek, hipEventDisableTiming));
      CK(hipEventRecord(ek, s[1]));
      CK(hipStreamWaitEvent(s[0], ek, 0));
      CK(hipEventRecord(e1, s[0]));
      CK(hipEventSynchronize(e1));
      CK(hipEventDestroy(ek));
      const double ms = time_ms(e0, e1);
      printf("{\"what\": \"d2h_and_h2d_together\", \"MB\": %zu, \"ms\": %.3f}\n", (bytes + in_bytes) >> 20, ms);
    }
  }
  return 0;
}
