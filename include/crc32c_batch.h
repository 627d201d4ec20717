/* crc32c_batch.h -- batched CRC-32C on AMD Instinct MI355X (gfx950).
 *
 * New surface added next to crc32c.h.  Each entry point
 * replaces a loop of scalar crc32c() calls in the reference:
 *
 *   crc32c_batch           N x crc32c(crc_in[i], base + off[i], len[i]):
 *                          the spill CRC of storage.c:567 gathered per wbuf,
 *                          the read-back CRC of storage.c:172 and
 *                          proxy_internal.c:28 gathered per IO batch
 *                          (extstore.c:853-945).
 *   crc32c_stamp_items     the spill CRC of storage.c:567 for every item image of
 *                          a wbuf, written into exptime.
 *   crc32c_batch_chains    the chained CRC of chunked items over iov lists
 *                          (storage.c:163-170).
 *   crc32c_verify_pages    the same over whole pages, walked on the device as
 *                          storage_compact_readback walks them.
 *   crc32c_verify_items    the read-verify compare of storage.c:159-178 applied
 *                          to every item image of a packed extstore page
 *                          (walk of storage.c:950-960): CRC over
 *                          [off + 32, off + ITEM_ntotal) against the value
 *                          stored in the item's exptime field (byte 28).
 *   crc32c_host_alloc      pinned buffers for wbufs / readback_buf (SURVEY.md 8f
 *                          rank 3).
 *   crc32c_batch_multi     crc32c_batch for host-resident batches split across
 *                          several GPUs by bytes (no collective: items are
 *                          independent); crc32c_shard_cuts is its split.
 *   crc32c_batch_submit    the read-verify CRCs of many IO threads
 *   / crc32c_batch_wait    (extstore.c:853-945, one batch of <= io_depth reads
 *                          per thread) coalesced into one kernel launch per
 *                          dispatch by a per-device queue.
 *
 * Results are bit-identical to the reference crc32c.c.  There is no CPU
 * fallback: without a usable gfx950 device every batch entry point returns
 * CRC32C_ENODEV.  Buffers stay owned by the caller and must stay valid until
 * the call (or crc32c_batch_wait) returns.
 */
#ifndef CRC32C_BATCH_H
#define CRC32C_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRC32C_OK 0
#define CRC32C_ENODEV (-1) /* no gfx950 device visible */
#define CRC32C_EHIP (-2)   /* HIP runtime error */
#define CRC32C_EINVAL (-3) /* bad arguments */
#define CRC32C_ENOMEM (-4) /* device or pinned allocation failed */
#define CRC32C_ERANGE (-5) /* a span lies outside [base, base + base_bytes): it was
                              not read and its out[] entry is 0 */
#define CRC32C_EWALK (-6)  /* crc32c_verify_pages: the device walk's count and emit
                              passes disagreed on some wbuf (an internal invariant;
                              the results are not valid) */

/* flags */
#define CRC32C_DEVICE 0x1u    /* every pointer in the batch is device memory of the
                                 current HIP device */
#define CRC32C_ASYNC 0x2u     /* with CRC32C_DEVICE: enqueue on `stream`, do not wait */
/* (0x4u is reserved: earlier builds named it CRC32C_ALIGNED16, an alignment
   promise no kernel needs -- every span kernel reads the 16-B pieces a span
   overlaps as they lie, at any alignment -- and it is ignored.) */
#define CRC32C_CFLAGS64 0x8u  /* item-image calls: the images come from a build with
                                 --enable-large-client-flags (configure.ac:139-140):
                                 client_flags_t is 8 bytes, so ITEM_CFLAGS adds 8 to
                                 ITEM_ntotal instead of 4 (memcached.h:96-100, :149-152) */

/* Longest span: 2 GiB - 64 KiB, twice the largest item memcached stores
 * (ITEM_SIZE_MAX_UPPER_LIMIT, memcached.h:115).  A device span past it is not
 * read (out[i] = 0, CRC32C_ERANGE; an item image claiming one is malformed);
 * a fixed-length batch or a host batch with one is rejected (CRC32C_EINVAL;
 * host spans are limited to 256 MiB each). */
#define CRC32C_MAX_SPAN 0x7fff0000u

/* A batch of byte spans inside one buffer.
 *   span i = [base + (offsets ? offsets[i] : i * stride),  + (lens ? lens[i] : len))
 *   out[i] = crc32c(crc_in ? crc_in[i] : 0, span i)
 * base_bytes bounds every span: no byte outside [base, base + base_bytes) is
 * read.  A span that does not fit is skipped (out[i] = 0) and the call returns
 * CRC32C_ERANGE (device batches with CRC32C_ASYNC cannot report it: their
 * out-of-range spans still read nothing and get 0).  A batch of equal spans
 * at a fixed stride that overruns base_bytes is rejected up front
 * (CRC32C_EINVAL).  offsets / lens / crc_in / out hold n entries each.
 * Spans may come in any order and may overlap (chunked-item iov lists keep
 * their chain order; host batches are staged in offset order internally). */
typedef struct crc32c_spans {
    const void *base;
    uint64_t base_bytes;
    const uint64_t *offsets;
    uint64_t stride;
    const uint32_t *lens;
    uint32_t len;
    const uint32_t *crc_in;
    uint32_t *out;
    uint64_t n;
} crc32c_spans;

/* Number of usable gfx950 devices (0 when none). */
int crc32c_gpu_count(void);

/* Checksum a batch.  Host batches are staged through pinned memory and the
 * call returns when out[] is filled.  Device batches are enqueued on `stream`
 * (a hipStream_t; NULL = the default stream) and, without CRC32C_ASYNC, the
 * call returns when they are done. */
int crc32c_batch(const crc32c_spans *spans, unsigned flags, void *stream);

/* Host batch split across the first `ngpus` devices by bytes; one host thread
 * per device, pinned H2D / D2H overlapped with the kernels. */
int crc32c_batch_multi(const crc32c_spans *spans, int ngpus);

/* The split crc32c_batch_multi uses: parts + 1 cut points, part g owns spans
 * [cuts[g], cuts[g+1]).  cuts[g] is the first span index i whose byte prefix
 * sum(len[0..i)) reaches total * g / parts (total = every span's bytes), so
 * each part holds about total / parts bytes.  lens == NULL: every span is
 * `len` bytes.  (The Python twin is memcached_amd/shard.py plan().) */
int crc32c_shard_cuts(const uint32_t *lens, uint32_t len, uint64_t n, int parts, uint64_t *cuts);

/* Verify n item images of a packed page buffer (host or device per flags).
 * ok[i] = 1 when item i's CRC matches its stored exptime; *nbad receives the
 * number of mismatching (or malformed) items.  region_bytes is the write
 * buffer size: extstore never lets an item cross a wbuf (extstore.c:627-636),
 * so an image whose header claims to is malformed (0 = bound by base_bytes
 * only). */
int crc32c_verify_items(const void *base, uint64_t base_bytes, uint64_t region_bytes,
                        const uint64_t *item_offsets, uint64_t n, uint8_t *ok, uint64_t *nbad,
                        unsigned flags, void *stream);

/* Chained CRCs over iov lists: the chunked-item read verify of
 * storage.c:163-170, where crc = crc32c(0, hdr + 32, hdr_len - 32) and then
 * crc = crc32c(crc, chunk_x, len_x) for every chunk.  iovs describes every
 * iov of every chain (crc_in must be NULL; iovs->out receives each iov's own
 * CRC and must hold iovs->n entries); chain c is iovs [chain_first[c],
 * chain_first[c+1]) (nchains + 1 entries) and out[c] its chained CRC.  All
 * arrays are host or device memory per flags, as for crc32c_batch. */
int crc32c_batch_chains(const crc32c_spans *iovs, const uint64_t *chain_first, uint64_t nchains,
                        uint32_t *out, unsigned flags, void *stream);

/* Verify whole pages with the walk done on the device: [base, base_bytes) is
 * a sequence of wbuf_bytes reads, each walked as storage_compact_readback does
 * (storage.c:950-1070: items packed from the read's start, nkey == 0 ends it,
 * next item at + ITEM_ntotal, stop when < 48 bytes remain) and every item
 * verified as crc32c_verify_items does (with region_bytes = wbuf_bytes).
 * *nitems = items found; the first min(cap, *nitems) offsets and ok flags are
 * written to offsets[] / ok[], in walk order, and *nbad counts every bad item.
 * cap == 0 is a count-only query: the walk runs, nothing is verified, *nbad =
 * 0 and offsets / ok may be NULL.  An item count is at most
 * base_bytes / 50 + ceil(base_bytes / wbuf_bytes) (an image is >= 50 bytes; a
 * wbuf's last counted image may run past its end).  Device scratch: the walk
 * keeps up to wbuf_bytes / 2048 offsets per wbuf (8 B each, 0.4 % of the
 * walked bytes; grow-only, reused by later calls). */
int crc32c_verify_pages(const void *base, uint64_t base_bytes, uint64_t wbuf_bytes,
                        uint64_t *offsets, uint8_t *ok, uint64_t cap, uint64_t *nitems,
                        uint64_t *nbad, unsigned flags, void *stream);

/* Stamp the spill CRC of n item images (storage.c:567, gathered per wbuf
 * before it is submitted): exptime (bytes 28..31) of image i receives
 * crc32c(0, image + 32, ITEM_ntotal - 32).  Host or device per flags; with
 * CRC32C_DEVICE | CRC32C_ASYNC and nbad == NULL the call returns once the
 * kernels are enqueued on `stream` (the caller fences reads of the wbuf on
 * that stream).  ok (optional) marks stamped images;
 * malformed images are left untouched and counted in *nbad.  region_bytes as
 * for crc32c_verify_items.  Images are expected not to overlap (extstore
 * packs them back to back); where one image's span covers another's exptime,
 * its CRC may or may not include that image's new stamp. */
int crc32c_stamp_items(void *base, uint64_t base_bytes, uint64_t region_bytes,
                       const uint64_t *item_offsets, uint64_t n, uint8_t *ok, uint64_t *nbad,
                       unsigned flags, void *stream);

/* Asynchronous form of crc32c_batch: returns at once with a job handle;
 * crc32c_batch_wait blocks until out[] is filled and frees the handle.
 *
 * Jobs go to the current device's queue.  Host jobs whose buffer is
 * device-visible (crc32c_host_alloc, crc32c_host_register) and whose spans are
 * at most 256 KiB are coalesced: the queue's dispatcher packs every such job
 * pending at that moment (up to 8192 spans) into one kernel launch that reads
 * the spans straight from host memory, while the previous launch runs.  Many
 * IO threads that each submit their few reads (storage.c:172 per io_depth
 * batch) thus share launches; crc32c_batch itself takes this path for such
 * batches.  Other jobs (pageable host memory, long spans, CRC32C_DEVICE
 * batches) run one by one on the dispatcher.  A CRC32C_DEVICE job runs on the
 * queue's own stream after the work the submitting thread had enqueued on its
 * device's default (NULL) stream when it submitted (an event recorded there
 * at submit time): a batch filled by work on another stream must be complete
 * when submitted.  The caller's arrays must stay valid until
 * crc32c_batch_wait returns. */
typedef struct crc32c_job *crc32c_job_t;
int crc32c_batch_submit(const crc32c_spans *spans, unsigned flags, crc32c_job_t *job);
int crc32c_batch_wait(crc32c_job_t job);

/* Queue counters of the current device since the first submit: coalesced
 * kernel launches, the spans and jobs they carried, and jobs run alone.  Any
 * pointer may be NULL. */
int crc32c_queue_stats(uint64_t *launches, uint64_t *spans, uint64_t *jobs, uint64_t *solo_jobs);

/* Page-locked host memory for extstore's wbufs (extstore.c:127-140) and the
 * compaction readback_buf (storage.c:1120): host batches over such buffers
 * are copied by one DMA per pipeline slot with no staging copy.  NULL when
 * there is no gfx950 device or the allocation fails; free with
 * crc32c_host_free. */
void *crc32c_host_alloc(size_t bytes);
void crc32c_host_free(void *p);

/* Page-lock and map an existing host range (e.g. the slab arena that read
 * buffers come from, storage.c:264-337) so host batches over it are read by
 * the GPU in place: coalesced by the queue and copied without staging. */
int crc32c_host_register(void *p, size_t bytes);
int crc32c_host_unregister(void *p);

/* Tuning, for tests and benchmarks: batches of at most n spans (default 8192,
 * the kernel's limit) take the single-launch small-batch kernel; 0 sends every
 * batch through the planned multi-launch path.  Process-wide; returns the
 * previous value. */
uint64_t crc32c_set_small_max(uint64_t n);

const char *crc32c_strerror(int err);

/* Duration of this thread's last synchronous device batch (milliseconds,
 * hipEvent-measured on its stream); -1 before the first one. */
float crc32c_last_kernel_ms(void);

#ifdef __cplusplus
}
#endif

#endif /* CRC32C_BATCH_H */
