/* extstore_sim.c -- the batched spill CRC with its read fence, under
 * concurrency, the way extstore.c / storage.c would run it after integration
 * (INTEGRATION.md section 2).
 *
 * Reference flow.  storage_write (storage.c:499-593) gets a wbuf slot from
 * extstore_write_request (extstore.c:591-646, returns with the page mutex
 * held), copies the image, stores crc32c() in exptime (storage.c:567), calls
 * extstore_write (extstore.c:652-670, unlocks), then links the header item
 * (storage.c:580).  From that moment a GET can read the item; while its wbuf
 * is not flushed (p->active && offset >= p->written) the IO thread copies it
 * straight out of the page's wbuf under p->mutex (extstore.c:885-888,
 * _read_from_wbuf :815-832) -- also while that wbuf is still being filled.
 *
 * Batched flow.  The writer records each image's offset in its wbuf's pending
 * list instead of computing the CRC, and the whole list is stamped by one
 * crc32c_stamp_items call in _submit_wbuf (extstore.c:559, under p->mutex)
 * before the wbuf goes to the flush thread.  The fence: a read served from the
 * OPEN wbuf (not yet submitted) first stamps the image it copies
 * (stamp-on-demand with the scalar crc32c(), under the same p->mutex); the
 * batch stamp at submit rewrites the same value (exptime lies outside the CRC
 * span [32, ntotal), so stamping is idempotent).  Reads of submitted or
 * flushed wbufs need nothing: they were stamped before submit returned.
 *
 * Threads: one writer (storage_write + _submit_wbuf), one flusher
 * (_wbuf_cb: p->written advances), R readers (the IO-thread read + the read
 * callback's CRC check via crc32c_batch on a page-locked read buffer, which
 * goes through the coalescing queue).
 *
 * Usage: extstore_sim [--gpu] [--no-fence] [readers]
 *   --no-fence: the negative control, stamping deferred with no fence; reads
 *   of open-wbuf items must then see false bad CRCs (the hole the fence
 *   closes).  Exit status 0 = the expected outcome.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "crc32c.h"
#include "crc32c_batch.h"

#define WBUF (1u << 20)
#define NWBUF 96
#define NITEMS 12000
#define ITEM_CAS 2u
#define MAX_IMG (48 + 16 + 8 + 12000 + 2)
/* an image is at least 48 + 2 + 1 + 2 bytes: a wbuf holds fewer than WBUF / 48 */
#define PENDING_CAP (WBUF / 48 + 1)

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

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

/* the page (extstore.c:55-72, reduced to what the CRC flow touches) */
static struct {
    pthread_mutex_t mutex;
    uint8_t *buf;              /* NWBUF wbufs back to back: wbuf w at buf + w * WBUF */
    uint32_t cur;              /* the wbuf being filled */
    uint32_t used;             /* bytes of it filled */
    uint64_t written;          /* bytes flushed (extstore.c:538-539) */
    uint64_t pending[PENDING_CAP]; /* unstamped images of wbuf `cur` (offsets from buf) */
    uint32_t npending;
    uint32_t submitted;        /* wbufs handed to the flusher */
    pthread_cond_t flush_cv;
} P = {.mutex = PTHREAD_MUTEX_INITIALIZER, .flush_cv = PTHREAD_COND_INITIALIZER};

static int fence = 1;
static atomic_uint_fast64_t nlinked;  /* items readers may fetch (linked, storage.c:580) */
static uint64_t item_off[NITEMS];
static atomic_int writer_done;
static int stamp_fail;
static uint64_t stamp_nbad;

/* _submit_wbuf (extstore.c:559): called with P.mutex held */
static void submit_wbuf(void) {
    uint8_t *w = P.buf + (uint64_t)P.cur * WBUF;
    uint64_t offs[PENDING_CAP];
    for (uint32_t i = 0; i < P.npending; ++i) offs[i] = P.pending[i] - (uint64_t)P.cur * WBUF;
    uint64_t nbad = 0;
    const int rc = crc32c_stamp_items(w, WBUF, WBUF, offs, P.npending, NULL, &nbad, 0, NULL);
    if (rc != CRC32C_OK) ++stamp_fail;
    stamp_nbad += nbad;
    memset(w + P.used, 0, WBUF - P.used);  /* extstore.c:568 */
    P.npending = 0;
    ++P.submitted;
    ++P.cur;
    P.used = 0;
    pthread_cond_signal(&P.flush_cv);
}

static void *writer(void *arg) {
    (void)arg;
    uint64_t rng = 7;
    static uint8_t src[MAX_IMG];
    for (uint32_t id = 0; id < NITEMS; ++id) {
        /* the item in RAM (items.c), key key%07u, CAS */
        char key[16];
        const int nkey = snprintf(key, sizeof key, "key%07u", id);
        const uint32_t vlen = (uint32_t)(mix(&rng) % 12000), nbytes = vlen + 2;
        const uint32_t nt = 48 + nkey + 1 + nbytes + 8;
        uint16_t refc = 1, flags = ITEM_CAS | 1u /* ITEM_LINKED */;
        memset(src, 0, 48);
        memcpy(src + 32, &nbytes, 4);
        memcpy(src + 36, &refc, 2);
        memcpy(src + 38, &flags, 2);
        src[40] = 3;
        src[41] = (uint8_t)nkey;
        const uint64_t cas = id + 1;
        memcpy(src + 48, &cas, 8);
        memcpy(src + 56, key, nkey + 1);
        for (uint32_t i = 0; i < vlen; ++i) src[56 + nkey + 1 + i] = (uint8_t)mix(&rng);
        src[56 + nkey + 1 + vlen] = '\r';
        src[56 + nkey + 1 + vlen + 1] = '\n';

        pthread_mutex_lock(&P.mutex);               /* extstore_write_request */
        if (P.used + nt > WBUF) {
            if (P.cur + 1 >= NWBUF) {
                pthread_mutex_unlock(&P.mutex);
                break;
            }
            submit_wbuf();                           /* extstore.c:627-629 */
        }
        uint8_t *img = P.buf + (uint64_t)P.cur * WBUF + P.used;
        memcpy(img + 32, src + 32, nt - 32);        /* storage.c:563 */
        memset(img, 0, 32);
        uint16_t f2 = ITEM_CAS;                      /* it_flags &= ~ITEM_LINKED (storage.c:566) */
        memcpy(img + 38, &f2, 2);
        const uint64_t off = (uint64_t)P.cur * WBUF + P.used;
        P.pending[P.npending++] = off;              /* instead of storage.c:567 */
        P.used += nt;                                /* extstore_write (extstore.c:652-670) */
        pthread_mutex_unlock(&P.mutex);
        item_off[id] = off;
        atomic_store_explicit(&nlinked, id + 1, memory_order_release);  /* item_replace, storage.c:580 */
    }
    pthread_mutex_lock(&P.mutex);
    if (P.npending) submit_wbuf();
    pthread_mutex_unlock(&P.mutex);
    atomic_store(&writer_done, 1);
    return NULL;
}

static void *flusher(void *arg) {  /* the bg IO thread's pwrite + _wbuf_cb */
    (void)arg;
    pthread_mutex_lock(&P.mutex);
    for (;;) {
        while (P.written / WBUF >= P.submitted && !atomic_load(&writer_done)) pthread_cond_wait(&P.flush_cv, &P.mutex);
        if (P.written / WBUF >= P.submitted) break;
        pthread_mutex_unlock(&P.mutex);
        struct timespec d = {0, 200000};  /* the pwrite */
        nanosleep(&d, NULL);
        pthread_mutex_lock(&P.mutex);
        P.written += WBUF;
    }
    pthread_mutex_unlock(&P.mutex);
    return NULL;
}

struct reader {
    pthread_t tid;
    int id;
    uint8_t *rbuf;  /* page-locked read buffer (crc32c_host_alloc) */
    uint64_t reads, open_reads, bad, mismatch, rc_fail;
};

static void *reader(void *arg) {
    struct reader *r = arg;
    uint64_t rng = 99 + (uint64_t)r->id;
    while (!atomic_load(&writer_done) || r->reads < 2000) {
        const uint64_t nl = atomic_load_explicit(&nlinked, memory_order_acquire);
        if (nl == 0) continue;
        /* half the reads go to the newest items: those sit in the open wbuf */
        const uint64_t k = mix(&rng) & 1 ? nl - 1 - mix(&rng) % (nl < 32 ? nl : 32) : mix(&rng) % nl;
        const uint64_t off = item_off[k];
        pthread_mutex_lock(&P.mutex);               /* extstore_io_thread, extstore.c:883-898 */
        uint8_t *img = P.buf + off;
        const int open = off / WBUF == P.cur && off >= P.written;
        if (open && fence) {                         /* the fence: stamp on demand */
            const uint32_t crc = crc32c(0, img + 32, ntotal_of(img) - 32);
            memcpy(img + 28, &crc, 4);
        }
        const uint32_t nt = ntotal_of(img);
        memcpy(r->rbuf, img, nt);                    /* _read_from_wbuf / pread */
        pthread_mutex_unlock(&P.mutex);
        r->open_reads += open;
        /* the read callback (storage.c:159-178): CRC via the batch API */
        uint64_t so = 32;
        uint32_t len = nt - 32, crc = 0;
        crc32c_spans s = {r->rbuf, nt, &so, 0, &len, 0, NULL, &crc, 1};
        if (crc32c_batch(&s, 0, NULL) != CRC32C_OK) {
            ++r->rc_fail;
            continue;
        }
        if (crc != crc32c(0, r->rbuf + 32, len)) ++r->mismatch;
        r->bad += crc != rd32(r->rbuf + 28);         /* badcrc_from_extstore */
        ++r->reads;
    }
    return NULL;
}

int main(int argc, char **argv) {
    int gpu = 0, nreaders = 8;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--gpu")) gpu = 1;
        else if (!strcmp(argv[i], "--no-fence")) fence = 0;
        else nreaders = atoi(argv[i]);
    }
    crc32c_init();
    if (!gpu) {
        uint8_t buf[64] = {0};
        uint64_t off = 0, nbad = 0;
        const int rc = crc32c_stamp_items(buf, sizeof buf, 0, &off, 1, NULL, &nbad, 0, NULL);
        printf("extstore_sim: no GPU, stamp reports %s\n", crc32c_strerror(rc));
        return rc == CRC32C_ENODEV ? 0 : 1;
    }
    P.buf = crc32c_host_alloc((size_t)NWBUF * WBUF);  /* pinned wbufs (extstore.c:127-140) */
    uint8_t *rbufs = crc32c_host_alloc((size_t)nreaders * MAX_IMG);
    if (!P.buf || !rbufs) {
        fprintf(stderr, "crc32c_host_alloc failed\n");
        return 1;
    }
    memset(P.buf, 0, (size_t)NWBUF * WBUF);
    struct reader *rs = calloc((size_t)nreaders, sizeof *rs);
    pthread_t wt, ft;
    pthread_create(&ft, NULL, flusher, NULL);
    for (int i = 0; i < nreaders; ++i) {
        rs[i].id = i;
        rs[i].rbuf = rbufs + (uint64_t)i * MAX_IMG;
        pthread_create(&rs[i].tid, NULL, reader, &rs[i]);
    }
    pthread_create(&wt, NULL, writer, NULL);
    pthread_join(wt, NULL);
    for (int i = 0; i < nreaders; ++i) pthread_join(rs[i].tid, NULL);
    pthread_mutex_lock(&P.mutex);
    pthread_cond_signal(&P.flush_cv);
    pthread_mutex_unlock(&P.mutex);
    pthread_join(ft, NULL);

    uint64_t reads = 0, open = 0, bad = 0, mism = 0, fail = 0;
    for (int i = 0; i < nreaders; ++i) {
        reads += rs[i].reads;
        open += rs[i].open_reads;
        bad += rs[i].bad;
        mism += rs[i].mismatch;
        fail += rs[i].rc_fail;
    }
    /* after the last submit every image carries exactly the scalar spill CRC */
    const uint64_t nl = atomic_load(&nlinked);
    uint64_t wrong = 0;
    for (uint64_t k = 0; k < nl; ++k) {
        const uint8_t *img = P.buf + item_off[k];
        wrong += rd32(img + 28) != crc32c(0, img + 32, ntotal_of(img) - 32);
    }
    printf("extstore_sim: fence %s, items %llu in %u wbufs, reads %llu (open wbuf %llu), badcrc %llu, "
           "crc mismatches %llu, rc failures %llu, stamp failures %d, stamp nbad %llu, images wrong after submit %llu\n",
           fence ? "on" : "off", (unsigned long long)nl, P.submitted, (unsigned long long)reads,
           (unsigned long long)open, (unsigned long long)bad, (unsigned long long)mism, (unsigned long long)fail,
           stamp_fail, (unsigned long long)stamp_nbad, (unsigned long long)wrong);
    crc32c_host_free(rbufs);
    crc32c_host_free(P.buf);
    const int base_ok = mism == 0 && fail == 0 && stamp_fail == 0 && stamp_nbad == 0 && wrong == 0 && open > 0;
    return base_ok && (fence ? bad == 0 : bad > 0) ? 0 : 1;
}
