/* extstore_config1.c -- BASELINE configs[0]: "extstore on tmpfile, 10 k SET of
 * 4 KiB values forcing spill" (SURVEY.md section 8d, config 1), driven through
 * libmcrc32c.so the way storage.c and extstore.c drive crc32c.
 *
 *   SET       10 000 items, key "key%07u" (nkey 10), a 4096-byte value from
 *             splitmix64 (seed 1, 8 bytes per draw, little-endian) + "\r\n",
 *             CAS = id + 1, client flags 0: ITEM_ntotal = 4165
 *             (memcached.h:149-152, :613-636).
 *   spill     storage_write (storage.c:499-593): the image is copied into the
 *             current 4 MiB wbuf (extstore.c:627-659; an item never straddles
 *             a wbuf, the tail stays zero, extstore.c:567-568) and its CRC
 *             crc32c(0, img + 32, ntotal - 32) is stored in exptime
 *             (storage.c:567).  Full wbufs are written to the page file with
 *             pwrite (extstore.c:559-580, one 64 MiB page of 16 wbufs).
 *   read      extstore_read -> pread(ntotal) at the item's offset, then the
 *             read-back check of _storage_get_item_cb (storage.c:159-178):
 *             a mismatch is a miss plus badcrc_from_extstore.
 *
 * The CPU leg uses only the scalar drop-in (crc32c after crc32c_init), as
 * config 1 prescribes.  With --gpu the same flow also runs batched: the wbufs
 * are stamped by crc32c_stamp_items, the page read back from the file is
 * verified by crc32c_verify_items, and the 10 000 reads are checked in one
 * crc32c_batch; every batched CRC must equal the scalar one.
 *
 * Prints the counts and a digest (crc32c over the 10 000 CRCs, little-endian)
 * that tests/test_integration.py compares with the value the reference
 * crc32c.c gives on the same items (tests/golden/config1.json).
 *
 * Usage: extstore_config1 <dir> [--gpu]     (writes <dir>/extstore.page)
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "crc32c.h"
#include "crc32c_batch.h"

#define NITEMS 10000u
#define VLEN 4096u
#define WBUF (4u << 20)
#define PAGE (64u << 20)
#define ITEM_CAS 2u

static uint64_t rng_state = 1;  /* splitmix64, seed 1 */
static uint64_t splitmix64(void) {
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

/* ITEM_ntotal (memcached.h:149-152) of the image at p */
static uint32_t ntotal_of(const uint8_t *p) {
    uint16_t flags;
    memcpy(&flags, p + 38, 2);
    return 48 + p[41] + 1 + rd32(p + 32) + ((flags & ITEM_CAS) ? 8 : 0);
}

/* the item image as do_item_alloc + the SET leave it (exptime holds 0) */
static uint32_t make_item(uint8_t *dst, uint32_t id) {
    char key[16];
    const int nkey = snprintf(key, sizeof key, "key%07u", id);
    const uint32_t nbytes = VLEN + 2, ntotal = 48 + nkey + 1 + nbytes + 8;
    const uint16_t refcount = 1, flags = ITEM_CAS;
    memset(dst, 0, 48);
    memcpy(dst + 32, &nbytes, 4);
    memcpy(dst + 36, &refcount, 2);
    memcpy(dst + 38, &flags, 2);
    dst[40] = 1;
    dst[41] = (uint8_t)nkey;
    const uint64_t cas = (uint64_t)id + 1;
    memcpy(dst + 48, &cas, 8);
    memcpy(dst + 56, key, nkey + 1);
    uint8_t *v = dst + 56 + nkey + 1;
    for (uint32_t i = 0; i < VLEN; i += 8) {
        const uint64_t r = splitmix64();
        memcpy(v + i, &r, 8);
    }
    v[VLEN] = '\r';
    v[VLEN + 1] = '\n';
    return ntotal;
}

static int fails = 0;
#define CHECK(c, ...)                                                  \
    do {                                                               \
        if (!(c)) {                                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);       \
            fprintf(stderr, __VA_ARGS__);                              \
            fprintf(stderr, "\n");                                     \
            ++fails;                                                   \
        }                                                              \
    } while (0)

/* the read-back check of every item: pread(ntotal) + crc32c, returns badcrc */
static uint32_t read_all(int fd, const uint64_t *offs, const uint32_t *ntot, uint32_t *crcs) {
    uint8_t *rb = malloc(8192);
    uint32_t bad = 0;
    for (uint32_t i = 0; i < NITEMS; ++i) {
        if (pread(fd, rb, ntot[i], (off_t)offs[i]) != (ssize_t)ntot[i]) {
            ++bad;
            continue;
        }
        const uint32_t crc = crc32c(0, rb + 32, ntotal_of(rb) - 32);
        if (crcs) crcs[i] = crc;
        bad += crc != rd32(rb + 28);
    }
    free(rb);
    return bad;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <dir> [--gpu]\n", argv[0]);
        return 2;
    }
    const int gpu = argc > 2 && strcmp(argv[2], "--gpu") == 0;
    char path[4096];
    snprintf(path, sizeof path, "%s/extstore.page", argv[1]);
    crc32c_init();

    /* ---- SET + spill: pack into wbufs, CRC into exptime, pwrite full wbufs ---- */
    const uint32_t nwbuf = PAGE / WBUF;
    uint8_t *page = calloc(1, PAGE);
    uint64_t *offs = malloc(sizeof(uint64_t) * NITEMS);
    uint32_t *ntot = malloc(sizeof(uint32_t) * NITEMS), *spill = malloc(sizeof(uint32_t) * NITEMS);
    uint32_t w = 0, used = 0;
    for (uint32_t i = 0; i < NITEMS; ++i) {
        uint8_t img[8192];
        const uint32_t nt = make_item(img, i);
        if (used + nt > WBUF) {  /* extstore.c:627-636: a new wbuf, the tail stays zero */
            ++w;
            used = 0;
        }
        CHECK(w < nwbuf, "page overflow");
        uint8_t *it = page + (uint64_t)w * WBUF + used;
        memcpy(it, img, nt);
        spill[i] = crc32c(0, it + 32, nt - 32); /* storage.c:567 */
        memcpy(it + 28, &spill[i], 4);
        offs[i] = (uint64_t)w * WBUF + used;
        ntot[i] = nt;
        used += nt;
    }
    const uint32_t wbufs_used = w + 1;
    const int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd < 0) {
        perror(path);
        return 2;
    }
    for (uint32_t k = 0; k < wbufs_used; ++k)
        CHECK(pwrite(fd, page + (uint64_t)k * WBUF, WBUF, (off_t)k * WBUF) == (ssize_t)WBUF, "pwrite");

    /* ---- read back: every item, then one torn on disk ---- */
    uint32_t *rcrc = malloc(sizeof(uint32_t) * NITEMS);
    const uint32_t bad = read_all(fd, offs, ntot, rcrc);
    CHECK(bad == 0, "badcrc %u on a clean page", bad);
    for (uint32_t i = 0; i < NITEMS; ++i) CHECK(rcrc[i] == spill[i], "item %u read CRC differs", i);
    const uint64_t torn = offs[4242] + 1000;
    uint8_t b;
    CHECK(pread(fd, &b, 1, (off_t)torn) == 1, "pread");
    b ^= 0x40;
    CHECK(pwrite(fd, &b, 1, (off_t)torn) == 1, "pwrite");
    const uint32_t bad1 = read_all(fd, offs, ntot, NULL);
    CHECK(bad1 == 1, "one torn item: badcrc %u", bad1);
    b ^= 0x40;
    CHECK(pwrite(fd, &b, 1, (off_t)torn) == 1, "pwrite");
    const uint32_t digest = crc32c(0, spill, sizeof(uint32_t) * NITEMS);
    printf("config1: %u written in %u wbufs, %u read, badcrc %u, torn-item badcrc %u, digest %08x\n", NITEMS,
           wbufs_used, NITEMS, bad, bad1, digest);

    if (gpu) {
        /* batched spill: stamp the same wbufs (exptime cleared) in one call */
        uint8_t *bat = crc32c_host_alloc(PAGE);
        CHECK(bat != NULL, "pinned page");
        memcpy(bat, page, PAGE);
        for (uint32_t i = 0; i < NITEMS; ++i) memset(bat + offs[i] + 28, 0, 4);
        uint64_t nbad = 0;
        int rc = crc32c_stamp_items(bat, PAGE, WBUF, offs, NITEMS, NULL, &nbad, 0, NULL);
        CHECK(rc == CRC32C_OK && nbad == 0, "stamp rc %d nbad %llu", rc, (unsigned long long)nbad);
        CHECK(memcmp(bat, page, PAGE) == 0, "batched spill CRCs differ from the per-item crc32c()");
        /* page read back from the file, verified in one call */
        memset(bat, 0, PAGE);
        CHECK(pread(fd, bat, (size_t)wbufs_used * WBUF, 0) == (ssize_t)((size_t)wbufs_used * WBUF), "pread page");
        uint8_t *ok = malloc(NITEMS);
        rc = crc32c_verify_items(bat, PAGE, WBUF, offs, NITEMS, ok, &nbad, 0, NULL);
        CHECK(rc == CRC32C_OK && nbad == 0, "verify rc %d nbad %llu", rc, (unsigned long long)nbad);
        /* the 10 000 reads as one IO batch: spans [off + 32, off + ntotal) */
        uint64_t *so = malloc(sizeof(uint64_t) * NITEMS);
        uint32_t *sl = malloc(sizeof(uint32_t) * NITEMS), *bc = malloc(sizeof(uint32_t) * NITEMS);
        for (uint32_t i = 0; i < NITEMS; ++i) {
            so[i] = offs[i] + 32;
            sl[i] = ntot[i] - 32;
        }
        crc32c_spans s = {bat, PAGE, so, 0, sl, 0, NULL, bc, NITEMS};
        rc = crc32c_batch(&s, 0, NULL);
        CHECK(rc == CRC32C_OK, "read batch rc %d", rc);
        uint32_t diff = 0;
        for (uint32_t i = 0; i < NITEMS; ++i) diff += bc[i] != spill[i];
        CHECK(diff == 0, "%u batched read CRCs differ", diff);
        printf("config1 gpu: stamped == scalar, page verify nbad %llu, read batch mismatches %u\n",
               (unsigned long long)nbad, diff);
        crc32c_host_free(bat);
    }
    close(fd);
    return fails ? 1 : 0;
}
