/* extstore_ref_driver.c -- drives the reference's OWN extstore.c, patched with
 * INTEGRATION.md section 2 (tests/integration/extstore_ref.patch; built by
 * oracle/build_extstore_ref.sh into oracle/_ref/), the way storage.c drives
 * it, with the spill CRC of storage.c:567 deferred to the batched stamp.
 *
 * The patch adds to extstore.c: each wbuf's list of image offsets (recorded by
 * extstore_write, extstore.c:652, under p->mutex), one extstore_stamp_wbuf()
 * call in _submit_wbuf (extstore.c:559, under p->mutex) before the wbuf goes
 * to the flush thread, and the fence -- a read served from the OPEN wbuf
 * (extstore.c:886) stamps its one image with extstore_stamp_one() first.  This
 * file supplies the two hooks: crc32c_stamp_items (libmcrc32c.so) for the
 * wbuf, with the per-item crc32c() of storage.c:567 as the fallback when
 * there is no GPU, and the scalar crc32c() for the fence.
 *
 * Threads: the reference's IO threads and flush (bg) thread; one writer
 * (storage_write, storage.c:499-593, minus the CRC: write_request, copy the
 * image, extstore_write, publish the item); R readers (storage's read path:
 * extstore_submit of an OBJ_IO_READ, then the check of _storage_get_item_cb,
 * storage.c:159-178: crc32c(0, buf + 32, len - 32) against exptime).  Half
 * the reads aim at the newest items, which sit in the open wbuf.
 *
 * After the run the page file is read back and verified on the GPU by
 * crc32c_verify_pages (the device walk of storage.c:950-1072).
 *
 * Usage: extstore_ref <dir> [readers]      (writes <dir>/extstore.file)
 * Prints one line of counts; false_bad counts bad CRCs whose bytes equal the
 * written image (an unstamped image read, the hole the fence closes), corrupt
 * counts reads whose bytes differ from it.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <fcntl.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include "crc32c.h"
#include "crc32c_batch.h"
#include "extstore.h"

#define PAGE_SIZE (8u << 20)
#define WBUF_SIZE (2u << 20)
#define PAGE_COUNT 32
#define NITEMS 40000u
#define VMAX 6000u
#define ITEM_CAS 2u
#define MAX_READERS 32

static uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

/* ITEM_ntotal (memcached.h:149-152) of an image: no client flags here */
static uint32_t ntotal_of(const uint8_t *p) {
    uint16_t flags;
    memcpy(&flags, p + 38, 2);
    return 48 + p[41] + 1 + rd32(p + 32) + ((flags & ITEM_CAS) ? 8 : 0);
}

static uint64_t mix(uint64_t *s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* ---- the hooks the patched extstore.c calls (under p->mutex) ---- */
static atomic_ulong g_batches, g_fallback, g_stamped, g_stamp_bad, g_fence;

void extstore_stamp_wbuf(char *buf, unsigned int size, uint64_t *off, unsigned int n) {
    if (n == 0) return;
    uint64_t nbad = 0;
    if (crc32c_stamp_items(buf, size, size, off, n, NULL, &nbad, 0, NULL) == CRC32C_OK) {
        atomic_fetch_add(&g_batches, 1);
        atomic_fetch_add(&g_stamp_bad, nbad);
    } else {  /* no GPU: storage.c:567 per item */
        for (unsigned int i = 0; i < n; i++) {
            uint8_t *it = (uint8_t *)buf + off[i];
            const uint32_t c = crc32c(0, it + 32, ntotal_of(it) - 32);
            memcpy(it + 28, &c, 4);
        }
        atomic_fetch_add(&g_fallback, 1);
    }
    atomic_fetch_add(&g_stamped, n);
}

void extstore_stamp_one(char *img) {
    uint8_t *it = (uint8_t *)img;
    const uint32_t c = crc32c(0, it + 32, ntotal_of(it) - 32);
    memcpy(it + 28, &c, 4);
    atomic_fetch_add(&g_fence, 1);
}

/* ---- the items ---- */
struct rec {
    uint8_t *img;
    uint32_t len, offset, page_version;
    unsigned short page_id;
};
static struct rec recs[NITEMS];
static atomic_uint g_pub;     /* items published to readers (release) */
static atomic_int g_writer_done;
static void *g_engine;

/* an item image as storage_write copies it (memcached.h:613-636): exptime
 * (the spill CRC) zero until stamped */
static uint8_t *make_image(uint32_t id, uint32_t *len) {
    uint64_t s = 0x5eed0000ull + id;
    const uint32_t v = 100 + (uint32_t)(mix(&s) % VMAX), nbytes = v + 2, nkey = 11;
    const uint32_t n = 48 + 8 + nkey + 1 + nbytes;
    uint8_t *it = calloc(1, n);
    const uint16_t refcount = 1, flags = ITEM_CAS;
    const uint64_t cas = id + 1;
    memcpy(it + 24, &id, 4);                     /* time */
    memcpy(it + 32, &nbytes, 4);
    memcpy(it + 36, &refcount, 2);
    memcpy(it + 38, &flags, 2);
    it[40] = 1;                                  /* slabs_clsid */
    it[41] = (uint8_t)nkey;
    memcpy(it + 48, &cas, 8);
    snprintf((char *)it + 56, nkey + 1, "key%08u", id);
    for (uint32_t k = 0; k < v; k += 8) {
        const uint64_t w = mix(&s);
        memcpy(it + 56 + nkey + 1 + k, &w, v - k < 8 ? v - k : 8);
    }
    memcpy(it + n - 2, "\r\n", 2);
    *len = n;
    return it;
}

static void *writer(void *arg) {
    (void)arg;
    for (uint32_t i = 0; i < NITEMS; i++) {
        uint32_t len;
        uint8_t *img = make_image(i, &len);
        obj_io io;
        memset(&io, 0, sizeof io);
        io.len = len;
        io.mode = OBJ_IO_WRITE;
        /* storage_write gives up and retries later; here: until it fits */
        while (extstore_write_request(g_engine, 0, 0, &io) != 0) {
            const struct timespec d = {0, 20000};
            nanosleep(&d, NULL);
        }
        memcpy(io.buf, img, len);  /* storage.c:561-565; no crc32c() here (deferred) */
        extstore_write(g_engine, &io);
        recs[i] = (struct rec){img, len, io.offset, io.page_version, io.page_id};
        atomic_store_explicit(&g_pub, i + 1, memory_order_release);
        if ((i & 31u) == 31u) {  /* paced, so readers catch images in the open wbuf */
            const struct timespec d = {0, 100000};
            nanosleep(&d, NULL);
        }
    }
    atomic_store(&g_writer_done, 1);
    return NULL;
}

struct waiter {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int done, ret;
};

static void read_cb(void *e, obj_io *io, int ret) {
    (void)e;
    struct waiter *w = io->data;
    pthread_mutex_lock(&w->mu);
    w->ret = ret;
    w->done = 1;
    pthread_cond_signal(&w->cv);
    pthread_mutex_unlock(&w->mu);
}

struct reader {
    pthread_t tid;
    uint64_t seed;
    unsigned long reads, misses, shorts, badcrc, false_bad, corrupt;
};

static void *reader(void *arg) {
    struct reader *r = arg;
    uint8_t *buf = malloc(48 + 8 + 12 + 100 + VMAX + 2);  /* the longest image (make_image) */
    struct waiter w;
    pthread_mutex_init(&w.mu, NULL);
    pthread_cond_init(&w.cv, NULL);
    while (!atomic_load(&g_writer_done) || r->reads < 3000) {
        const uint32_t n = atomic_load_explicit(&g_pub, memory_order_acquire);
        if (n == 0) continue;
        const uint64_t x = mix(&r->seed);
        const uint32_t span = n < 48 ? n : 48;
        const uint32_t idx = (x & 1) ? n - 1 - (uint32_t)((x >> 1) % span) : (uint32_t)((x >> 1) % n);
        const struct rec *c = &recs[idx];
        obj_io io;
        memset(&io, 0, sizeof io);
        io.buf = (char *)buf;
        io.len = c->len;
        io.offset = c->offset;
        io.page_id = c->page_id;
        io.page_version = c->page_version;
        io.mode = OBJ_IO_READ;
        io.cb = read_cb;
        io.data = &w;
        w.done = 0;
        extstore_submit(g_engine, &io);
        pthread_mutex_lock(&w.mu);
        while (!w.done) pthread_cond_wait(&w.cv, &w.mu);
        pthread_mutex_unlock(&w.mu);
        r->reads++;
        if (w.ret < 0) {
            r->misses++;
            continue;
        }
        if ((uint32_t)w.ret != c->len) {
            r->shorts++;
            continue;
        }
        /* _storage_get_item_cb (storage.c:159-178) */
        const bool same = memcmp(buf, c->img, 28) == 0 && memcmp(buf + 32, c->img + 32, c->len - 32) == 0;
        if (!same) r->corrupt++;
        if (crc32c(0, buf + 32, c->len - 32) != rd32(buf + 28)) {
            r->badcrc++;
            if (same) r->false_bad++;
        }
    }
    free(buf);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <dir> [readers]\n", argv[0]);
        return 2;
    }
    int nreaders = argc > 2 ? atoi(argv[2]) : 8;
    if (nreaders < 1 || nreaders > MAX_READERS) nreaders = 8;
    crc32c_init();
    char path[4096];
    snprintf(path, sizeof path, "%s/extstore.file", argv[1]);
    struct extstore_conf_file f;
    memset(&f, 0, sizeof f);
    f.file = path;
    f.page_count = PAGE_COUNT;
    struct extstore_conf cf;
    memset(&cf, 0, sizeof cf);
    cf.page_size = PAGE_SIZE;
    cf.page_count = PAGE_COUNT;
    cf.page_buckets = 1;
    cf.free_page_buckets = 0;
    cf.wbuf_size = WBUF_SIZE;
    cf.wbuf_count = 4;
    cf.io_threadcount = 4;
    cf.io_depth = 1;
    enum extstore_res res;
    g_engine = extstore_init(&f, &cf, &res);
    if (!g_engine) {
        fprintf(stderr, "extstore_init: %s\n", extstore_err(res));
        return 2;
    }
    struct reader rs[MAX_READERS];
    memset(rs, 0, sizeof rs);
    pthread_t wt;
    for (int i = 0; i < nreaders; i++) {
        rs[i].seed = 1000 + i;
        pthread_create(&rs[i].tid, NULL, reader, &rs[i]);
    }
    pthread_create(&wt, NULL, writer, NULL);
    pthread_join(wt, NULL);
    unsigned long reads = 0, misses = 0, shorts = 0, badcrc = 0, false_bad = 0, corrupt = 0;
    for (int i = 0; i < nreaders; i++) {
        pthread_join(rs[i].tid, NULL);
        reads += rs[i].reads;
        misses += rs[i].misses;
        shorts += rs[i].shorts;
        badcrc += rs[i].badcrc;
        false_bad += rs[i].false_bad;
        corrupt += rs[i].corrupt;
    }
    /* the page file: every flushed wbuf verified by the device walk */
    unsigned long vitems = 0, vbad = 0;
    int vrc = CRC32C_ENODEV;
    sleep(1);  /* (the last submitted wbuf's pwrite) */
    const int fd = open(path, O_RDONLY);
    struct stat sb;
    if (fd >= 0 && fstat(fd, &sb) == 0 && sb.st_size > 0) {
        const uint64_t size = (uint64_t)sb.st_size;
        uint8_t *fb = malloc(size);
        uint64_t got = 0;
        while (got < size) {
            const ssize_t k = pread(fd, fb + got, size - got, (off_t)got);
            if (k <= 0) break;
            got += (uint64_t)k;
        }
        const uint64_t cap = size / 50 + size / WBUF_SIZE + 1;
        uint64_t *offs = malloc(cap * 8), nitems = 0, nbad = 0;
        uint8_t *ok = malloc(cap);
        vrc = crc32c_verify_pages(fb, got, WBUF_SIZE, offs, ok, cap, &nitems, &nbad, 0, NULL);
        vitems = nitems;
        vbad = nbad;
        free(offs);
        free(ok);
        free(fb);
    }
    if (fd >= 0) close(fd);
    printf("extstore_ref: written %u reads %lu misses %lu short %lu badcrc %lu false_bad %lu corrupt %lu "
           "open_wbuf_stamps %lu batches %lu fallback_batches %lu stamped %lu stamp_nbad %lu page_verify_rc %d "
           "nitems %lu nbad %lu\n",
           NITEMS, reads, misses, shorts, badcrc, false_bad, corrupt, (unsigned long)atomic_load(&g_fence),
           (unsigned long)atomic_load(&g_batches), (unsigned long)atomic_load(&g_fallback),
           (unsigned long)atomic_load(&g_stamped), (unsigned long)atomic_load(&g_stamp_bad), vrc, vitems, vbad);
    return 0;
}
