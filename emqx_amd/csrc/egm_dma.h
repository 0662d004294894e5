// Device -> host copies on the SDMA engines through the HSA runtime (round 4,
// host pipeline).  hipMemcpyAsync D2H into pinned memory runs as a blit
// KERNEL on this image (`__amd_rocclr_copyBuffer` in the trace), and CU
// stores to host memory stall the next batch's memory-bound kernels
// (k_tokenise 0.1 -> 0.75-1.9 ms beside them, profiles/r4_host_trace_*.json);
// the DMA engines move the result without a CU.
#pragma once
#include <stddef.h>

namespace egm {

struct DmaPart {
  void* dst;        // pinned host memory (hipHostMalloc)
  const void* src;  // device memory (hipMalloc)
  size_t bytes;
};

struct Dma;
// The HSA agents of HIP device `device` and of the host; null when the HSA
// runtime or an agent is not found (the caller then copies with HIP).
Dma* dma_open(int device);
void dma_close(Dma* d);
// Copy the parts (in flight together) and wait for all of them; false on a
// copy error.  Only one thread may use a Dma at a time.
bool dma_copy_d2h(Dma* d, const DmaPart* parts, int nparts);

}  // namespace egm
