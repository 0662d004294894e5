// egm_pack.h — the packed host result of a pipeline batch (round 6,
// VERDICT r5 item 7): the host path is bound by the PCIe link, so a batch
// whose filter ids all fit 24 bits crosses it as u32 row starts and 3-byte
// ids (egm_result.id_bytes == 3, include/emqx_gpu_match.h) — 3 bytes per id
// and 4 per row start instead of 4 and 8.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace egm {

// row[n + 1] (u64) -> row32[n + 1]; ids[0, row[n]) -> pk (3 bytes each,
// little-endian).  The id count is read on the device; ids beyond ids_cap are
// never read (an overflowed batch is rerun by the caller before it is packed).
// ids must be readable up to 4 entries past the last one (the kernel reads whole
// groups of four) and pk writable up to 12 bytes past 3 * count.
hipError_t launch_pack_result(const uint64_t* row, uint32_t n, const uint32_t* ids, uint64_t ids_cap,
                              uint32_t* row32, uint8_t* pk, hipStream_t s);

}  // namespace egm
