// egm_alloc.h — memory behind the results the C-ABI hands out.  Every result
// (egm_result, egm_delivery) is preceded by a header saying how to release it,
// so egm_result_free() works for all of them: plain host allocations, and
// pipeline results that live in a context's pinned staging (egm_match_wait).
#pragma once
#include <stdint.h>
#include <stdlib.h>

namespace egm {

struct ResultHdr {          // 32 B: keeps the result that follows 16-B aligned
  uint64_t magic;
  void* owner;              // pipeline results: the context
  uint64_t slot;            // pipeline results: the staging slot
  uint64_t pad;
};
constexpr uint64_t RES_MALLOC = 0x6567726573756c74ull;   // "egresult"
constexpr uint64_t RES_PIPE = 0x6567706970656c6eull;     // "egpipeln"

inline void* result_alloc(size_t sz) {
  ResultHdr* h = (ResultHdr*)malloc(sizeof(ResultHdr) + sz);
  if (!h) return nullptr;
  h->magic = RES_MALLOC;
  h->owner = nullptr;
  h->slot = 0;
  return h + 1;
}

inline void result_discard(void* p) {
  if (p) free((ResultHdr*)p - 1);
}

}  // namespace egm
