/* crc32c.h -- drop-in replacement for memcached's crc32c.h.
 *
 * Same call surface as the reference header (/root/reference/crc32c.h:15-21):
 *
 *   crc_func crc32c;          a DATA symbol holding a function pointer; callers
 *                             invoke it directly as crc32c(crc, buf, len)
 *                             (storage.c:165,169,172,567; proxy_internal.c:28;
 *                             testapp.c:861,867,873).
 *   void crc32c_init(void);   must run before the first call (storage.c:1601,
 *                             testapp.c:2344); replaces crc32c.c:266-275.
 *   uint32_t crc32c_sw(...);  table-driven variant kept for tests
 *                             (crc32c.c:507-513).
 *
 * Semantics are the reference's: standard reflected CRC-32C (Castagnoli,
 * polynomial 0x82f63b78), ~crc on entry and exit, chaining
 * crc32c(crc32c(0, A), B) == crc32c(0, A || B), len == 0 returns crc.  The
 * scalar symbol stays on the host: one call checksums one buffer synchronously
 * (a 4 KiB item costs ~0.3 us on a core, far below a GPU round trip).  Batched
 * callers use crc32c_batch.h, which runs the gfx950 kernels.
 */
#ifndef CRC32C_H
#define CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint32_t (*crc_func)(uint32_t crc, const void *buf, size_t len);
extern crc_func crc32c;

void crc32c_init(void);

uint32_t crc32c_sw(uint32_t crc, void const *buf, size_t len);

/* Non-static in the reference (crc32c.c:52-53); exported for completeness.
 * crc32c_sw_big is the big-endian slice-by-8 (crc32c.c:467-498) evaluated
 * with this host's native loads, exactly as the reference's own symbol: the
 * CRC-32C on a big-endian host, the reference's same non-CRC function on a
 * little-endian one (crc32c_sw picks crc32c_sw_little there). */
uint32_t crc32c_sw_little(uint32_t crc, void const *buf, size_t len);
uint32_t crc32c_sw_big(uint32_t crc, void const *buf, size_t len);

#ifdef __cplusplus
}
#endif

#endif /* CRC32C_H */
