/* storage_sim.c -- memcached's extstore CRC flow driven through the drop-in
 * library from C, the way storage.c would call it after integration
 * (INTEGRATION.md sections 2-4).
 *
 *   write path  storage_write (storage.c:499-593): each item image is copied
 *               into a wbuf and its spill CRC crc32c(0, img + 32, ntotal - 32)
 *               is stored in exptime (storage.c:567).  Reference flow: one
 *               scalar crc32c() call per item (the drop-in function pointer).
 *               Batched flow: crc32c_stamp_items over the whole wbuf set.
 *   read path   _storage_get_item_cb (storage.c:159-178): an IO batch of
 *               read-back images (extstore.c:853-869) is checked in one
 *               crc32c_batch call instead of one crc32c() per callback.
 *   compaction  storage_compact_readback (storage.c:933-1072): the page is
 *               walked (nkey == 0 ends a wbuf) and verified in one call.
 *
 * Item images follow memcached.h:613-636 (48-byte header, exptime at 28,
 * nbytes at 32, it_flags at 38, nkey at 41, CAS after the header).
 *
 * Usage: storage_sim [--gpu].  Without --gpu only the scalar drop-in is
 * exercised, and the batch entry points must fail with CRC32C_ENODEV (the
 * library has no CPU fallback).  Exit status 0 = every check passed.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc32c.h"
#include "crc32c_batch.h"

#define WBUF (1u << 20)
#define NWBUF 6
#define ITEM_CAS 2u

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint64_t splitmix64(void) {
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* ITEM_ntotal (memcached.h:149-152) of the image at p */
static uint32_t ntotal_of(const uint8_t *p) {
    uint16_t flags;
    memcpy(&flags, p + 38, 2);
    return 48 + p[41] + 1 + rd32(p + 32) + ((flags & ITEM_CAS) ? 8 : 0);
}

/* one image: key "key%07d", value of vlen random bytes + "\r\n" */
static uint32_t make_item(uint8_t *dst, uint32_t id, uint32_t vlen) {
    char key[16];
    const int nkey = snprintf(key, sizeof key, "key%07u", id);
    const uint32_t nbytes = vlen + 2, ntotal = 48 + nkey + 1 + nbytes + 8;
    uint16_t refcount = 1, flags = ITEM_CAS;
    memset(dst, 0, 48);
    memcpy(dst + 32, &nbytes, 4);
    memcpy(dst + 36, &refcount, 2);
    memcpy(dst + 38, &flags, 2);
    dst[40] = 1;
    dst[41] = (uint8_t)nkey;
    const uint64_t cas = id + 1;
    memcpy(dst + 48, &cas, 8);
    memcpy(dst + 56, key, nkey + 1);
    uint8_t *v = dst + 56 + nkey + 1;
    for (uint32_t i = 0; i < vlen; i += 8) {
        const uint64_t r = splitmix64();
        memcpy(v + i, &r, vlen - i < 8 ? vlen - i : 8);
    }
    v[vlen] = '\r';
    v[vlen + 1] = '\n';
    return ntotal;
}

static int fails = 0;
#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);               \
            fprintf(stderr, "\n");                      \
            ++fails;                                    \
        }                                               \
    } while (0)

int main(int argc, char **argv) {
    const int gpu = argc > 1 && strcmp(argv[1], "--gpu") == 0;
    crc32c_init();
    CHECK(crc32c(0, "123456789", 9) == 0xe3069283u, "check value");

    /* ---- write path: pack images into wbufs (extstore.c:627-659) ---- */
    /* the batched wbufs are pinned (extstore.c:127-140 with crc32c_host_alloc):
     * the host path then DMAs them without a staging copy */
    uint8_t *ref = calloc(NWBUF, WBUF), *bat = gpu ? crc32c_host_alloc((size_t)NWBUF * WBUF) : NULL;
    if (!gpu) {
        CHECK(crc32c_host_alloc(4096) == NULL, "pinned allocation without a GPU must fail");
        bat = calloc(NWBUF, WBUF);
    }
    if (!ref || !bat) {
        fprintf(stderr, "allocation failed\n");
        return 2;
    }
    uint64_t *offs = malloc(sizeof(uint64_t) * NWBUF * WBUF / 64);
    uint64_t n = 0;
    for (uint32_t w = 0; w < NWBUF; ++w) {
        uint32_t used = 0;
        for (;;) {
            const uint32_t vlen = (uint32_t)(splitmix64() % 12000);
            if (used + 48 + 11 + vlen + 2 + 8 > WBUF) break;  /* next wbuf (tail stays zero) */
            const uint32_t nt = make_item(ref + (uint64_t)w * WBUF + used, (uint32_t)n, vlen);
            offs[n++] = (uint64_t)w * WBUF + used;
            used += nt;
        }
    }
    memcpy(bat, ref, (size_t)NWBUF * WBUF);
    for (uint64_t i = 0; i < n; ++i) {  /* reference: storage.c:567 per item */
        uint8_t *it = ref + offs[i];
        const uint32_t crc = crc32c(0, it + 32, ntotal_of(it) - 32);
        memcpy(it + 28, &crc, 4);
    }
    uint64_t nbad = 0;
    int rc = crc32c_stamp_items(bat, (uint64_t)NWBUF * WBUF, WBUF, offs, n, NULL, &nbad, 0, NULL);
    if (!gpu) {
        CHECK(rc == CRC32C_ENODEV, "stamp without a GPU must fail loudly, got %d", rc);
        printf("storage_sim: scalar drop-in ok, %llu items, batch entry points report %s\n",
               (unsigned long long)n, crc32c_strerror(rc));
        return fails ? 1 : 0;
    }
    CHECK(rc == CRC32C_OK && nbad == 0, "stamp rc %d nbad %llu", rc, (unsigned long long)nbad);
    CHECK(memcmp(ref, bat, (size_t)NWBUF * WBUF) == 0, "batched spill CRCs differ from per-item crc32c()");

    /* ---- compaction read-back: walk (storage.c:950-960) + verify ---- */
    uint64_t m = 0;
    for (uint32_t w = 0; w < NWBUF; ++w)
        for (uint64_t o = (uint64_t)w * WBUF; o + 48 <= (uint64_t)(w + 1) * WBUF && bat[o + 41] != 0;
             o += ntotal_of(bat + o))
            offs[m++] = o;
    CHECK(m == n, "walk found %llu items, wrote %llu", (unsigned long long)m, (unsigned long long)n);
    uint8_t *ok = malloc(n);
    rc = crc32c_verify_items(bat, (uint64_t)NWBUF * WBUF, WBUF, offs, n, ok, &nbad, 0, NULL);
    CHECK(rc == CRC32C_OK && nbad == 0, "verify rc %d nbad %llu", rc, (unsigned long long)nbad);

    /* ---- read path: one IO batch of 256 reads into a read arena ---- */
    const uint32_t nrd = 256;
    uint64_t *roff = malloc(sizeof(uint64_t) * nrd), *src = malloc(sizeof(uint64_t) * nrd);
    uint32_t *rlen = malloc(sizeof(uint32_t) * nrd), *rcrc = malloc(sizeof(uint32_t) * nrd);
    uint64_t arena_bytes = 0;
    for (uint32_t r = 0; r < nrd; ++r) {
        src[r] = offs[splitmix64() % n];
        roff[r] = arena_bytes;
        arena_bytes += (ntotal_of(bat + src[r]) + 7) & ~7u;  /* slab chunks are 8-B aligned */
    }
    uint8_t *arena = malloc(arena_bytes);
    for (uint32_t r = 0; r < nrd; ++r) memcpy(arena + roff[r], bat + src[r], ntotal_of(bat + src[r]));
    uint64_t *span_off = malloc(sizeof(uint64_t) * nrd);
    for (uint32_t r = 0; r < nrd; ++r) {
        span_off[r] = roff[r] + 32;
        rlen[r] = ntotal_of(arena + roff[r]) - 32;
    }
    arena[span_off[77] + rlen[77] / 2] ^= 0x20;  /* one torn read */
    crc32c_spans s = {arena, arena_bytes, span_off, 0, rlen, 0, NULL, rcrc, nrd};
    rc = crc32c_batch(&s, 0, NULL);
    CHECK(rc == CRC32C_OK, "read batch rc %d", rc);
    uint32_t badcrc = 0;
    for (uint32_t r = 0; r < nrd; ++r) {
        const uint8_t *it = arena + roff[r];
        const int bad = rcrc[r] != rd32(it + 28);
        badcrc += bad;  /* storage.c:176-178: miss + badcrc_from_extstore */
        CHECK(rcrc[r] == crc32c(0, it + 32, rlen[r]), "read %u: batch CRC differs from crc32c()", r);
        CHECK(bad == (r == 77), "read %u: bad=%d", r, bad);
    }
    printf("storage_sim: %llu items stamped and verified, %u reads, badcrc %u\n", (unsigned long long)n, nrd,
           badcrc);
    crc32c_host_free(bat);
    return fails ? 1 : 0;
}
