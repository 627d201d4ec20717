// crc32c_host.h -- the shim's own host CRC-32C for the synchronous scalar call
// surface (crc_func crc32c, crc32c.h:15-16).  Single calls from storage.c are
// latency-bound (one 4 KiB item ~0.5 us on a core) and stay on the host; batched
// callers use the GPU entry points in crc32c_batch.h.
//
//   crc32c_host_sw : slice-by-8 tables (same results as crc32c_sw, crc32c.c:366-424)
//   crc32c_host_hw : the CRC32C instruction (SSE4.2 crc32 / ARMv8 crc32cx), three independent streams merged
//                    with zeros operators (same results as crc32c_hw, crc32c.c:161-246)
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace mcrc {

void host_tables_init();  // idempotent, thread-safe
uint32_t crc32c_host_sw(uint32_t crc, const void *buf, size_t len);
uint32_t crc32c_host_hw(uint32_t crc, const void *buf, size_t len);
// crc32c_sw_big (crc32c.c:467-498) as the reference computes it on this host
uint32_t crc32c_host_sw_big(uint32_t crc, const void *buf, size_t len);
bool host_has_hw_crc();  // SSE4.2 (x86-64) or the ARMv8 CRC extension (arm64)
// crc32c(crc, A || B) from crc32c(crc, A), crc32c(0, B) and |B|.
uint32_t crc32c_host_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

}  // namespace mcrc
