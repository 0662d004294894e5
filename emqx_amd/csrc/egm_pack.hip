// egm_pack.hip — pack a pipeline batch's CSR for the PCIe link (egm_pack.h).
// A streaming kernel: a thread takes a group of four ids (one 16-B load) and
// writes them as 12 bytes (three 4-B stores), so consecutive lanes write
// consecutive bytes; the row starts are narrowed beside it.  ~0.2 GB moved per
// 1M-topic C2 batch: well under the copy it saves.
#include <hip/hip_runtime.h>

#include "egm_pack.h"

namespace egm {

__global__ __launch_bounds__(256) void k_pack_result(const uint64_t* __restrict__ row, uint32_t n,
                                                     const uint32_t* __restrict__ ids, uint64_t ids_cap,
                                                     uint32_t* __restrict__ row32, uint8_t* __restrict__ pk) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = tid; i <= n; i += stride) row32[i] = (uint32_t)row[i];
  const uint64_t total = row[n] < ids_cap ? row[n] : ids_cap;
  const uint64_t groups = (total + 3) / 4;
  uint32_t* out = (uint32_t*)pk;
  for (uint64_t g = tid; g < groups; g += stride) {
    const uint4 v = *(const uint4*)(ids + 4 * g);
    out[3 * g] = (v.x & 0xFFFFFFu) | (v.y << 24);
    out[3 * g + 1] = ((v.y >> 8) & 0xFFFFu) | (v.z << 16);
    out[3 * g + 2] = ((v.z >> 16) & 0xFFu) | (v.w << 8);
  }
}

hipError_t launch_pack_result(const uint64_t* row, uint32_t n, const uint32_t* ids, uint64_t ids_cap,
                              uint32_t* row32, uint8_t* pk, hipStream_t s) {
  hipLaunchKernelGGL(k_pack_result, dim3(1024), dim3(256), 0, s, row, n, ids, ids_cap, row32, pk);
  return hipGetLastError();
}

}  // namespace egm
