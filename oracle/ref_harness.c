/* ref_harness.c -- TEST/BASELINE INFRASTRUCTURE ONLY.
 *
 * Linked with the reference crc32c.c (compiled in place from /root/reference by
 * oracle/Makefile into oracle/_ref/libref_crc32c.so).  Exposes the reference
 * crc32c function pointer to ctypes and a pthread timing harness used for the
 * cpu_baseline leg of bench.py: one thread per requested core (optionally
 * pinned to a given CPU list: one logical CPU per physical core), static
 * contiguous split of the item array, each item checksummed with
 * crc32c(0, item, len) exactly as storage.c:567 does.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#include "crc32c.h"

uint32_t ref_crc32c(uint32_t crc, const void *buf, size_t len) { return crc32c(crc, buf, len); }
uint32_t ref_crc32c_sw(uint32_t crc, const void *buf, size_t len) { return crc32c_sw(crc, buf, len); }
void ref_crc32c_init(void) { crc32c_init(); }

struct job {
    const unsigned char *base;
    const uint64_t *offsets; /* NULL: base + i * stride */
    const uint64_t *lens;    /* NULL: every item is `len` bytes */
    uint64_t stride, len, lo, hi;
    uint32_t *out;
};

static void *worker(void *arg) {
    struct job *j = (struct job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const unsigned char *p = j->base + (j->offsets ? j->offsets[i] : i * j->stride);
        j->out[i] = crc32c(0, p, j->lens ? j->lens[i] : j->len);
    }
    return NULL;
}

/* Checksums n items with `threads` threads (thread t pinned to cpus[t] when
 * cpus is not NULL); returns wall seconds. */
double ref_crc32c_batch_timed_cpus(const unsigned char *base, const uint64_t *offsets,
                                   const uint64_t *lens, uint64_t stride, uint64_t len, uint64_t n,
                                   int threads, uint32_t *out, const int *cpus) {
    if (threads < 1) threads = 1;
    pthread_t *tid = calloc((size_t)threads, sizeof *tid);
    struct job *jobs = calloc((size_t)threads, sizeof *jobs);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (struct job){base, offsets, lens, stride, len, n * t / threads,
                               n * (t + 1) / threads, out};
        pthread_attr_t attr;
        pthread_attr_init(&attr);
        if (cpus) {
            cpu_set_t set;
            CPU_ZERO(&set);
            CPU_SET(cpus[t], &set);
            pthread_attr_setaffinity_np(&attr, sizeof set, &set);
        }
        pthread_create(&tid[t], &attr, worker, &jobs[t]);
        pthread_attr_destroy(&attr);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(tid);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

double ref_crc32c_batch_timed(const unsigned char *base, const uint64_t *offsets,
                              const uint64_t *lens, uint64_t stride, uint64_t len, uint64_t n,
                              int threads, uint32_t *out) {
    return ref_crc32c_batch_timed_cpus(base, offsets, lens, stride, len, n, threads, out, NULL);
}

/* NUMA-local form: thread t (pinned to cpus[t]) first copies its contiguous
 * share of the items into memory it allocates itself (so its pages are
 * first-touched on its own node, as a worker-allocated slab would be), then
 * every pass checksums the shares in parallel between two barriers.  Returns
 * the best pass's wall seconds; out[] holds every item's CRC. */
struct ljob {
    const unsigned char *src;
    uint64_t stride, len, lo, hi;
    uint32_t *out;
    int cpu, passes;
    pthread_barrier_t *bar;
    struct timespec *t;  /* per pass: start (thread 0) and end (thread 0) */
};

static void *local_worker(void *arg) {
    struct ljob *j = (struct ljob *)arg;
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    const uint64_t cnt = j->hi - j->lo;
    unsigned char *mine = malloc(cnt * j->stride + 1);
    for (uint64_t i = 0; i < cnt; i++)
        for (uint64_t b = 0; b < j->len; b += 4096) {
            const uint64_t k = j->len - b < 4096 ? j->len - b : 4096;
            __builtin_memcpy(mine + i * j->stride + b, j->src + (j->lo + i) * j->stride + b, k);
        }
    for (int p = 0; p < j->passes; p++) {
        pthread_barrier_wait(j->bar);
        if (j->lo == 0) clock_gettime(CLOCK_MONOTONIC, &j->t[2 * p]);
        for (uint64_t i = 0; i < cnt; i++) j->out[j->lo + i] = crc32c(0, mine + i * j->stride, j->len);
        pthread_barrier_wait(j->bar);
        if (j->lo == 0) clock_gettime(CLOCK_MONOTONIC, &j->t[2 * p + 1]);
    }
    free(mine);
    return NULL;
}

double ref_crc32c_batch_local(const unsigned char *base, uint64_t stride, uint64_t len, uint64_t n, int threads,
                              uint32_t *out, const int *cpus, int passes) {
    if (threads < 1) threads = 1;
    if (passes < 1) passes = 1;
    pthread_t *tid = calloc((size_t)threads, sizeof *tid);
    struct ljob *jobs = calloc((size_t)threads, sizeof *jobs);
    struct timespec *t = calloc((size_t)passes * 2, sizeof *t);
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads);
    for (int k = 0; k < threads; k++) {
        jobs[k] = (struct ljob){base, stride, len, n * k / threads, n * (k + 1) / threads, out,
                                cpus ? cpus[k] : -1, passes, &bar, t};
        pthread_create(&tid[k], NULL, local_worker, &jobs[k]);
    }
    for (int k = 0; k < threads; k++) pthread_join(tid[k], NULL);
    double best = 1e30;
    for (int p = 0; p < passes; p++) {
        const double d = (double)(t[2 * p + 1].tv_sec - t[2 * p].tv_sec) +
                         1e-9 * (double)(t[2 * p + 1].tv_nsec - t[2 * p].tv_nsec);
        if (d < best) best = d;
    }
    pthread_barrier_destroy(&bar);
    free(tid);
    free(jobs);
    free(t);
    return best;
}
