/* queue_sim.c -- the read-verify CRCs of many extstore IO threads through the
 * library's coalescing queue (crc32c_batch_submit / crc32c_batch_wait).
 *
 * Shape (extstore.c:853-945): each IO thread pulls a batch of at most
 * io_depth reads (default io_depth = 1, storage.c:1339), preads every item
 * image into its read buffer and runs the read callback, which checks
 * crc32c(0, buf + 32, len - 32) against the stored exptime (storage.c:159-178).
 * Here each thread copies `depth` random images of a stamped page set into its
 * page-locked read buffer (the pread), submits their CRC spans as one batch,
 * waits, and compares every CRC with the scalar crc32c() and with exptime.
 * Some reads are torn on purpose (one flipped byte) and must be the only
 * mismatches.  The queue's dispatcher packs the batches pending from all
 * threads into shared kernel launches.
 *
 * Usage: queue_sim [--gpu] [threads] [reads_per_thread] [depth]
 * Without --gpu the submit must fail with CRC32C_ENODEV (no CPU fallback).
 * Output: one summary line; exit status 0 = every check passed.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "crc32c.h"
#include "crc32c_batch.h"

#define ITEM_CAS 2u
#define MAX_DEPTH 64
#define MAX_IMG (48 + 16 + 8 + 16384 + 2)

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

static uint32_t ntotal_of(const uint8_t *p) {  /* ITEM_ntotal (memcached.h:149-152) */
    uint16_t flags;
    memcpy(&flags, p + 38, 2);
    return 48 + p[41] + 1 + rd32(p + 32) + ((flags & ITEM_CAS) ? 8 : 0);
}

static uint64_t mix(uint64_t *s) {  /* splitmix64 */
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static uint32_t make_item(uint8_t *dst, uint32_t id, uint32_t vlen, uint64_t *rng) {
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
        const uint64_t r = mix(rng);
        memcpy(v + i, &r, vlen - i < 8 ? vlen - i : 8);
    }
    v[vlen] = '\r';
    v[vlen + 1] = '\n';
    const uint32_t crc = crc32c(0, dst + 32, ntotal - 32);  /* the spill CRC (storage.c:567) */
    memcpy(dst + 28, &crc, 4);
    return ntotal;
}

struct shared {
    const uint8_t *store;
    const uint64_t *offs;
    uint64_t nitems;
    int reads, depth;
};

struct worker {
    pthread_t tid;
    int id;
    const struct shared *sh;
    uint8_t *rbuf;  /* page-locked read buffer: depth slots of MAX_IMG */
    double *lat_us; /* one per submitted batch */
    uint64_t mismatches, torn, detected, false_bad, rc_fail;
};

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void *io_thread(void *arg) {
    struct worker *w = arg;
    const struct shared *sh = w->sh;
    uint64_t rng = 0x1234567ull + (uint64_t)w->id * 0x9e3779b97f4a7c15ull;
    uint64_t off[MAX_DEPTH];
    uint32_t len[MAX_DEPTH], out[MAX_DEPTH];
    int torn[MAX_DEPTH];
    for (int r = 0; r < sh->reads; ++r) {
        for (int k = 0; k < sh->depth; ++k) {  /* the preads of one IO batch */
            const uint8_t *src = sh->store + sh->offs[mix(&rng) % sh->nitems];
            uint8_t *dst = w->rbuf + (uint64_t)k * MAX_IMG;
            const uint32_t nt = ntotal_of(src);
            memcpy(dst, src, nt);
            torn[k] = mix(&rng) % 97 == 0;
            if (torn[k]) dst[32 + mix(&rng) % (nt - 32)] ^= 0x10;
            off[k] = (uint64_t)k * MAX_IMG + 32;
            len[k] = nt - 32;
        }
        crc32c_spans s = {w->rbuf, (uint64_t)sh->depth * MAX_IMG, off, 0, len, 0, NULL, out, (uint64_t)sh->depth};
        crc32c_job_t job;
        const double t0 = now_us();
        int rc = crc32c_batch_submit(&s, 0, &job);
        if (rc == CRC32C_OK) rc = crc32c_batch_wait(job);
        w->lat_us[r] = now_us() - t0;
        if (rc != CRC32C_OK) {
            ++w->rc_fail;
            continue;
        }
        for (int k = 0; k < sh->depth; ++k) {  /* the read callbacks (storage.c:159-178) */
            const uint8_t *it = w->rbuf + (uint64_t)k * MAX_IMG;
            if (out[k] != crc32c(0, it + 32, len[k])) ++w->mismatches;
            const int bad = out[k] != rd32(it + 28);
            w->torn += torn[k];
            w->detected += bad && torn[k];
            w->false_bad += bad && !torn[k];
        }
    }
    return NULL;
}

static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

int main(int argc, char **argv) {
    int gpu = 0, ai = 1;
    if (argc > 1 && strcmp(argv[1], "--gpu") == 0) gpu = 1, ai = 2;
    const int nthreads = argc > ai ? atoi(argv[ai]) : 16;
    const int reads = argc > ai + 1 ? atoi(argv[ai + 1]) : 2000;
    int depth = argc > ai + 2 ? atoi(argv[ai + 2]) : 1;
    if (depth < 1 || depth > MAX_DEPTH || nthreads < 1 || reads < 1) return 2;
    crc32c_init();

    /* the page set the reads come from: ~24 MB of stamped item images of
     * 4 KiB values (the config-1 shape) and some of other sizes */
    const uint64_t nitems = 6000;
    uint8_t *store = malloc(nitems * MAX_IMG);
    uint64_t *offs = malloc(nitems * sizeof(uint64_t));
    uint64_t rng = 42, used = 0;
    for (uint64_t i = 0; i < nitems; ++i) {
        const uint32_t vlen = i % 4 ? 4096 : (uint32_t)(mix(&rng) % 16384);
        offs[i] = used;
        used += make_item(store + used, (uint32_t)i, vlen, &rng);
    }

    if (!gpu) {
        uint32_t len = ntotal_of(store) - 32, out = 0;
        uint64_t off = 32;
        crc32c_spans s = {store, used, &off, 0, &len, 0, NULL, &out, 1};
        crc32c_job_t job;
        const int rc = crc32c_batch_submit(&s, 0, &job);
        printf("queue_sim: no GPU, submit reports %s\n", crc32c_strerror(rc));
        return rc == CRC32C_ENODEV ? 0 : 1;
    }

    /* CPU reference rate of the same callback: one core, scalar crc32c() */
    double t0 = now_us();
    uint32_t sink = 0;
    const int cpu_reads = 20000;
    for (int r = 0; r < cpu_reads; ++r) {
        const uint8_t *it = store + offs[r % nitems];
        sink ^= crc32c(0, it + 32, ntotal_of(it) - 32);
    }
    const double cpu_us = (now_us() - t0) / cpu_reads;

    struct shared sh = {store, offs, nitems, reads, depth};
    struct worker *ws = calloc((size_t)nthreads, sizeof *ws);
    uint8_t *rbufs = crc32c_host_alloc((size_t)nthreads * depth * MAX_IMG);
    if (!rbufs) {
        fprintf(stderr, "crc32c_host_alloc failed\n");
        return 1;
    }
    /* warm-up: device tables, the queue and its dispatcher */
    {
        uint64_t off = 32;
        uint32_t len = ntotal_of(store) - 32, out = 0;
        memcpy(rbufs, store, ntotal_of(store));
        crc32c_spans s = {rbufs, MAX_IMG, &off, 0, &len, 0, NULL, &out, 1};
        if (crc32c_batch(&s, 0, NULL) != CRC32C_OK || out != rd32(store + 28)) {
            fprintf(stderr, "warm-up batch failed\n");
            return 1;
        }
    }
    uint64_t l0, s0, j0, q0;
    crc32c_queue_stats(&l0, &s0, &j0, &q0);
    t0 = now_us();
    for (int t = 0; t < nthreads; ++t) {
        ws[t].id = t;
        ws[t].sh = &sh;
        ws[t].rbuf = rbufs + (uint64_t)t * depth * MAX_IMG;
        ws[t].lat_us = malloc(sizeof(double) * reads);
        pthread_create(&ws[t].tid, NULL, io_thread, &ws[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(ws[t].tid, NULL);
    const double wall_us = now_us() - t0;
    uint64_t l1, s1, j1, q1;
    crc32c_queue_stats(&l1, &s1, &j1, &q1);

    uint64_t mism = 0, torn = 0, det = 0, fbad = 0, fail = 0;
    double *lat = malloc(sizeof(double) * (size_t)nthreads * reads), sum = 0;
    for (int t = 0; t < nthreads; ++t) {
        mism += ws[t].mismatches;
        torn += ws[t].torn;
        det += ws[t].detected;
        fbad += ws[t].false_bad;
        fail += ws[t].rc_fail;
        memcpy(lat + (size_t)t * reads, ws[t].lat_us, sizeof(double) * reads);
    }
    const size_t nl = (size_t)nthreads * reads;
    for (size_t i = 0; i < nl; ++i) sum += lat[i];
    qsort(lat, nl, sizeof(double), cmp_d);
    const uint64_t items = (uint64_t)nthreads * reads * depth;
    const uint64_t launches = l1 - l0, spans = s1 - s0;
    printf("queue_sim: threads %d depth %d reads %llu mismatches %llu torn %llu detected %llu false_bad %llu "
           "rc_fail %llu items_per_s %.0f batch_lat_us mean %.1f p50 %.1f p99 %.1f launches %llu spans %llu "
           "jobs %llu solo %llu spans_per_launch %.1f cpu_us_per_item %.3f (sink %x)\n",
           nthreads, depth, (unsigned long long)items, (unsigned long long)mism, (unsigned long long)torn,
           (unsigned long long)det, (unsigned long long)fbad, (unsigned long long)fail, items / (wall_us * 1e-6),
           sum / nl, lat[nl / 2], lat[(size_t)(nl * 0.99)], (unsigned long long)launches,
           (unsigned long long)spans, (unsigned long long)(j1 - j0), (unsigned long long)(q1 - q0),
           launches ? (double)spans / launches : 0.0, cpu_us, sink & 0xf);
    crc32c_host_free(rbufs);
    return (mism == 0 && fail == 0 && fbad == 0 && det == torn && spans == items) ? 0 : 1;
}
