/* crc32c_oracle.c -- CPU restatement of the reference CRC-32C path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in memcached_amd/ links, loads or calls
 * this file.  It is the checker for tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Parity is pinned (tests/test_oracle.py) by the
 * reference's own known-answer tests (testapp.c:853-879) and by golden vectors
 * that tests/golden/make_golden.py generates from the reference crc32c.c
 * compiled under oracle/_ref/ (oracle/Makefile).
 *
 * Follows /root/reference:
 *   crc32c.c:50        reflected polynomial 0x82f63b78
 *   crc32c.c:366-389   byte table and its k-zero-byte extensions
 *   crc32c.c:393-424   slice-by-8 little-endian loop, ~crc in and out
 *   crc32c.c:58-137    GF(2) zeros operators (matrix square / times)
 *   storage.c:567      spill CRC over item + STORE_OFFSET (32) .. ntotal
 *   storage.c:160-178  read-back verify: crc stored in item->exptime (byte 28)
 *   storage.c:950-960  packed-page walk: stop at nkey == 0, advance ITEM_ntotal
 *   memcached.h:613-636, :149-152  item header layout and ITEM_ntotal
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_POLY 0x82f63b78u

static uint32_t tab[8][256];
static int tab_ready;

static void oracle_tables(void) {
    if (tab_ready) return;
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY : c >> 1;
        tab[0][n] = c;
    }
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = tab[0][n];
        for (int k = 1; k < 8; k++) {
            c = tab[0][c & 0xffu] ^ (c >> 8);
            tab[k][n] = c;
        }
    }
    tab_ready = 1;
}

/* Bit-at-a-time definition: the slowest, most literal form. */
uint32_t oracle_crc32c_bitwise(uint32_t crc, const void *buf, size_t len) {
    const unsigned char *p = (const unsigned char *)buf;
    uint32_t r = ~crc;
    while (len--) {
        r ^= *p++;
        for (int k = 0; k < 8; k++) r = (r & 1u) ? (r >> 1) ^ ORACLE_POLY : r >> 1;
    }
    return ~r;
}

/* Slice-by-8 (crc32c.c:393-424 restated). */
uint32_t oracle_crc32c(uint32_t crc, const void *buf, size_t len) {
    const unsigned char *p = (const unsigned char *)buf;
    oracle_tables();
    uint32_t r = ~crc;
    while (len && ((uintptr_t)p & 7u)) {
        r = tab[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
        len--;
    }
    while (len >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        w ^= r;
        r = tab[7][w & 0xffu] ^ tab[6][(w >> 8) & 0xffu] ^ tab[5][(w >> 16) & 0xffu] ^
            tab[4][(w >> 24) & 0xffu] ^ tab[3][(w >> 32) & 0xffu] ^ tab[2][(w >> 40) & 0xffu] ^
            tab[1][(w >> 48) & 0xffu] ^ tab[0][w >> 56];
        p += 8;
        len -= 8;
    }
    while (len--) r = tab[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
    return ~r;
}

/* GF(2) 32x32 matrices by rows of images of basis vectors (crc32c.c:58-78). */
static uint32_t mat_times(const uint32_t *mat, uint32_t vec) {
    uint32_t sum = 0;
    for (int i = 0; vec; i++, vec >>= 1)
        if (vec & 1u) sum ^= mat[i];
    return sum;
}

static void mat_square(uint32_t *sq, const uint32_t *mat) {
    for (int i = 0; i < 32; i++) sq[i] = mat_times(mat, mat[i]);
}

/* Advance a CRC register over n zero bytes (crc32c.c:85-131 generalised to
 * any n by square-and-multiply). */
uint32_t oracle_shift_zeros(uint32_t reg, uint64_t n) {
    uint32_t op[32], tmp[32];
    /* one zero bit, then square three times: one zero byte */
    op[0] = ORACLE_POLY;
    for (int i = 1; i < 32; i++) op[i] = 1u << (i - 1);
    for (int s = 0; s < 3; s++) {
        mat_square(tmp, op);
        memcpy(op, tmp, sizeof op);
    }
    while (n) {
        if (n & 1u) reg = mat_times(op, reg);
        n >>= 1;
        if (n) {
            mat_square(tmp, op);
            memcpy(op, tmp, sizeof op);
        }
    }
    return reg;
}

/* crc32c(crc_a, A || B) from crc_a = crc32c(x, A), crc_b = crc32c(0, B). */
uint32_t oracle_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return oracle_shift_zeros(crc_a, len_b) ^ crc_b;
}

/* Batch over (offset, len, crc_in) descriptors into one buffer. */
void oracle_crc32c_batch(const unsigned char *base, const uint64_t *offsets, const uint64_t *lens,
                         const uint32_t *crc_in, uint32_t *out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = oracle_crc32c(crc_in ? crc_in[i] : 0u, base + offsets[i], (size_t)lens[i]);
}

/* memcached item geometry (memcached.h:613-636, :149-152). */
#define ORACLE_ITEM_HDR 48u   /* sizeof(item) on LP64 */
#define ORACLE_STORE_OFFSET 32u
#define ORACLE_EXPTIME_OFF 28u
#define ORACLE_NBYTES_OFF 32u
#define ORACLE_FLAGS_OFF 38u
#define ORACLE_NKEY_OFF 41u
#define ORACLE_ITEM_CAS 2u
#define ORACLE_ITEM_CFLAGS 256u

/* ITEM_ntotal with cfl = sizeof(client_flags_t): 4, or 8 in a build with
 * --enable-large-client-flags (memcached.h:96-100, configure.ac:139-140). */
uint32_t oracle_item_ntotal_cfl(const unsigned char *it, uint32_t cfl) {
    int32_t nbytes;
    uint16_t flags;
    memcpy(&nbytes, it + ORACLE_NBYTES_OFF, 4);
    memcpy(&flags, it + ORACLE_FLAGS_OFF, 2);
    uint32_t n = ORACLE_ITEM_HDR + it[ORACLE_NKEY_OFF] + 1u + (uint32_t)nbytes;
    if (flags & ORACLE_ITEM_CFLAGS) n += cfl;
    if (flags & ORACLE_ITEM_CAS) n += 8;
    return n;
}

uint32_t oracle_item_ntotal(const unsigned char *it) { return oracle_item_ntotal_cfl(it, 4); }

/* Spill CRC of one item image (storage.c:567). */
uint32_t oracle_item_crc_cfl(const unsigned char *it, uint32_t cfl) {
    return oracle_crc32c(0, it + ORACLE_STORE_OFFSET, oracle_item_ntotal_cfl(it, cfl) - ORACLE_STORE_OFFSET);
}

uint32_t oracle_item_crc(const unsigned char *it) { return oracle_item_crc_cfl(it, 4); }

/* Walk one packed span the way storage.c:950-960 does and verify every item's
 * stored CRC (storage.c:160-178).  Returns the number of items; ok[i] = 1 when
 * the CRC matches; offsets[i] receives each item's offset.  max_items bounds
 * the output arrays. */
uint64_t oracle_verify_span_cfl(const unsigned char *buf, uint64_t size, uint64_t *offsets,
                                uint8_t *ok, uint64_t max_items, uint32_t cfl) {
    uint64_t off = 0, n = 0;
    while (off + ORACLE_ITEM_HDR <= size && n < max_items) {
        const unsigned char *it = buf + off;
        if (it[ORACLE_NKEY_OFF] == 0) break;
        const uint32_t ntotal = oracle_item_ntotal_cfl(it, cfl);
        if (off + ntotal > size) break;
        uint32_t stored;
        memcpy(&stored, it + ORACLE_EXPTIME_OFF, 4);
        offsets[n] = off;
        ok[n] = stored == oracle_item_crc_cfl(it, cfl);
        n++;
        off += ntotal;
    }
    return n;
}

uint64_t oracle_verify_span(const unsigned char *buf, uint64_t size, uint64_t *offsets,
                            uint8_t *ok, uint64_t max_items) {
    return oracle_verify_span_cfl(buf, size, offsets, ok, max_items, 4);
}
