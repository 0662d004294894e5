// SDMA device -> host copies (egm_dma.h).
#include "egm_dma.h"

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>

namespace egm {

constexpr int DMA_MAX_PARTS = 8;
struct Dma {
  hsa_agent_t gpu{}, cpu{};
  hsa_signal_t sig[DMA_MAX_PARTS]{};   // one per copy, each 1 -> 0 (a profiler's copy tracer expects that)
  int nsig = 0;
};

namespace {
struct Find {
  uint32_t bdf = 0, domain = 0;
  bool have_gpu = false, have_cpu = false;
  hsa_agent_t gpu{}, cpu{};
};

hsa_status_t visit(hsa_agent_t a, void* p) {
  Find& f = *(Find*)p;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !f.have_cpu) {
    f.cpu = a;
    f.have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !f.have_gpu) {
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    if (bdf == f.bdf && dom == f.domain) {
      f.gpu = a;
      f.have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}
}  // namespace

Dma* dma_open(int device) {
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, device) != hipSuccess) return nullptr;
  if (hsa_init() != HSA_STATUS_SUCCESS) return nullptr;   // reference-counted: HIP has initialised it
  Find f;
  f.bdf = ((uint32_t)pr.pciBusID << 8) | ((uint32_t)pr.pciDeviceID << 3);   // function 0
  f.domain = (uint32_t)pr.pciDomainID;
  hsa_iterate_agents(visit, &f);
  Dma* d = nullptr;
  if (f.have_gpu && f.have_cpu) {
    d = new Dma();
    d->gpu = f.gpu;
    d->cpu = f.cpu;
    for (; d->nsig < DMA_MAX_PARTS; ++d->nsig)
      if (hsa_signal_create(0, 0, nullptr, &d->sig[d->nsig]) != HSA_STATUS_SUCCESS) break;
    if (d->nsig < DMA_MAX_PARTS) {
      for (int i = 0; i < d->nsig; ++i) hsa_signal_destroy(d->sig[i]);
      delete d;
      d = nullptr;
    }
  }
  if (!d) hsa_shut_down();
  return d;
}

void dma_close(Dma* d) {
  if (!d) return;
  for (int i = 0; i < d->nsig; ++i) hsa_signal_destroy(d->sig[i]);
  delete d;
  hsa_shut_down();
}

bool dma_copy_d2h(Dma* d, const DmaPart* parts, int nparts) {
  if (nparts > DMA_MAX_PARTS) return false;
  int k = 0;
  bool ok = true;
  for (int i = 0; i < nparts && ok; ++i) {
    if (!parts[i].bytes) continue;
    hsa_signal_store_screlease(d->sig[k], 1);
    if (hsa_amd_memory_async_copy(parts[i].dst, d->cpu, parts[i].src, d->gpu, parts[i].bytes, 0, nullptr, d->sig[k]) !=
        HSA_STATUS_SUCCESS) {
      ok = false;
      break;
    }
    ++k;
  }
  for (int j = 0; j < k; ++j)   // every issued copy is waited for, even after a failed issue
    ok &= hsa_signal_wait_scacquire(d->sig[j], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                    HSA_WAIT_STATE_BLOCKED) == 0;
  return ok;
}

}  // namespace egm
