// crc32c_shim.hip -- the C-ABI library (libmcrc32c.so): memcached's crc32c.h
// surface plus the batched gfx950 entry points of crc32c_batch.h.
//
// Host side of the drop-in boundary.  The scalar symbols replace crc32c.c
// (crc32c.c:47, :266-275, :507-513); the batch symbols replace loops of those
// calls in storage.c / proxy_internal.c (see include/crc32c_batch.h).
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/crc32c.h"
#include "../../include/crc32c_batch.h"
#include "crc32c_gf2.h"
#include "crc32c_host.h"
#include "crc32c_kernels.hip"

// ---------------------------------------------------------------------------
// Scalar drop-in (crc32c.h)
// ---------------------------------------------------------------------------
extern "C" {

crc_func crc32c = nullptr;

void crc32c_init(void) {
    mcrc::host_tables_init();
    crc32c = mcrc::host_has_hw_crc() ? mcrc::crc32c_host_hw : mcrc::crc32c_host_sw;
}

uint32_t crc32c_sw(uint32_t crc, void const *buf, size_t len) { return mcrc::crc32c_host_sw(crc, buf, len); }

uint32_t crc32c_sw_little(uint32_t crc, void const *buf, size_t len) {
    return mcrc::crc32c_host_sw(crc, buf, len);
}

uint32_t crc32c_sw_big(uint32_t crc, void const *buf, size_t len) {
    return mcrc::crc32c_host_sw_big(crc, buf, len);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Per-device state
// ---------------------------------------------------------------------------
namespace {

constexpr int kBlock = 1024;                    // 16 waves, 32 lane groups
constexpr uint32_t kItemsPerBlockStep = 32;     // one span per 32-lane group
constexpr uint32_t kFixedLen = mcrc_dev::kK1Bytes;  // K1: 8 pieces x 32 lanes x 16 B

thread_local float g_last_kernel_ms = -1.0f;

struct Queue;
enum {
    kScrWalkCnt, kScrWalkPrefix, kScrWalkOffs, kScrWalkOk, kScrWalkScan, kScrStage, kScrItemOffs, kScrItemOut,
    kScrFb, kScrFbOffs, kScrFbOk, kScrRt, kScrWalkSlots, kScrCount
};

struct Device {
    int id = -1;
    int cus = 0;
    bool ok = false;
    uint4 *img = nullptr;       // LDS table image of every table kernel (build_lds_image_span, chunk 16)
    uint32_t *tab8 = nullptr;   // byte-wise table (k_count / k_final: a span's head fragment and foreign bytes)
    uint32_t *xpow = nullptr;   // x^(8n) table (layout mcrc_dev::kXpow*)
    uint32_t xm128 = 0;         // k_lines / k_fix: x^(-8 * 128)
    uint4 *zero = nullptr;      // kZeroBytes of zeros (one 4 KiB line set per CU slot)
    unsigned long long *nbad = nullptr;  // [0]: bad / out-of-range count, [1]: walk invariant failures
    unsigned long long *hbad = nullptr;  // pinned twin of nbad[0..1] (a D2H copy into pageable memory is a slow path)
    // k_small's own counters for calls that take the count from hbad (item
    // images): zero between calls, kept so by the kernel's last workgroup
    unsigned long long *small_nbad = nullptr;
    uint32_t *small_done = nullptr;
    uint32_t *nfb = nullptr;    // k_lines' fallback count (device)
    uint32_t *route = nullptr;  // k_census's verdict: K5 (1) or the planned path (0)
    hipStream_t stream = nullptr, copy = nullptr;
    // a stamp's k_fix runs on `side` beside the damaged images' planned path
    // (fork: after k_lines on the caller's stream; join: the caller's stream
    // waits for it before the call's last kernel)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t copied[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};  // host-batch pipeline slots
    std::mutex mu;              // serialises the entry points that use the scratch below
    std::atomic<Queue *> queue{nullptr};  // coalescing queue (crc32c_batch_submit), created on first use
    // Shared device scratch (plan buffers, nbad, walk buffers) is owned in
    // stream order: a launch on stream B waits for the last use on stream A.
    hipEvent_t busy = nullptr;
    hipStream_t busy_stream = nullptr;
    bool busy_valid = false;
    void acquire(hipStream_t st) {
        if (busy_valid && busy_stream != st) (void)hipStreamWaitEvent(st, busy, 0);
    }
    void release(hipStream_t st) {
        if (hipEventRecord(busy, st) == hipSuccess) {
            busy_stream = st;
            busy_valid = true;
        }
    }
    // host-batch staging: two device slots + two pinned slots
    uint8_t *dbuf[2] = {nullptr, nullptr};
    uint8_t *pin[2] = {nullptr, nullptr};
    uint64_t slot_bytes = 0;
    uint64_t *doffs[2] = {nullptr, nullptr};
    uint32_t *dlens[2] = {nullptr, nullptr}, *dcin[2] = {nullptr, nullptr}, *dout[2] = {nullptr, nullptr};
    uint64_t *hoffs[2] = {nullptr, nullptr};  // pinned twins of the descriptor slots
    uint32_t *hlens[2] = {nullptr, nullptr}, *hcin[2] = {nullptr, nullptr}, *hout[2] = {nullptr, nullptr};
    uint64_t slot_items = 0;
    // work-unit planning for long / variable spans (grow-only)
    uint64_t *nunit = nullptr;  // per span: units | blocks << 32
    mcrc_dev::PlanSum *tile_sum = nullptr, *tile_pre = nullptr;  // per kPlanTile spans: sums, exclusive scan (+ total)
    uint32_t *span_acc = nullptr, *counters = nullptr;
    uint32_t *starts = nullptr;  // balanced plan: first record of each span-kernel group (groups + 1)
    uint32_t *segpow = nullptr;  // rows x^i * x^(8*4096*k): k < 256, then k = 256 j
    mcrc_dev::UnitRec *units = nullptr, *whole = nullptr;
    uint4 *irec = nullptr;  // per-span record written by k_count
    uint8_t *fast = nullptr;     // per span: its unit is one whole block (k_blocks takes it)
    uint32_t *fastidx = nullptr; // the fast spans' indices, compacted (k_expand)
    uint4 *big = nullptr;  // spans expanded by k_expand_big: {span, p0, b0}
    uint64_t plan_items = 0, plan_units = 0;
    // grow-only scratch for the page walk and staged item batches
    struct Scratch {
        void *p = nullptr;
        size_t bytes = 0;
    } scratch[kScrCount];
    void *grow(int slot, size_t bytes) {
        Scratch &s = scratch[slot];
        if (s.bytes < bytes) {
            if (s.p) (void)hipFree(s.p);
            s.p = nullptr;
            s.bytes = 0;
            if (hipMalloc(&s.p, bytes) != hipSuccess) {
                s.p = nullptr;
                (void)hipGetLastError();  // (not left pending for a later launch check)
                return nullptr;
            }
            s.bytes = bytes;
        }
        return s.p;
    }
    // grow-only pinned, device-mapped scratch of the host item-image calls:
    // host address in *h, the address kernels use in *dv
    struct Pinned {
        void *h = nullptr, *d = nullptr;
        size_t bytes = 0;
    } pinned[4];
    bool grow_pinned(int slot, size_t bytes, void **h, void **dv) {
        Pinned &s = pinned[slot];
        if (s.bytes < bytes) {
            if (s.h) (void)hipHostFree(s.h);
            s = Pinned{};
            if (hipHostMalloc(&s.h, bytes, hipHostMallocDefault) != hipSuccess) return false;
            if (hipHostGetDevicePointer(&s.d, s.h, 0) != hipSuccess) {
                (void)hipHostFree(s.h);
                s = Pinned{};
                return false;
            }
            s.bytes = bytes;
        }
        *h = s.h;
        *dv = s.d;
        return true;
    }
};
enum { kPinStage, kPinOffs, kPinOk, kPinCrc };

std::mutex g_dev_mu;  // device discovery and first initialisation only
// Device state by HIP ordinal (every visible device; only gfx950 ones are
// ever initialised), and the library's device index -> HIP ordinal map: the
// gfx950 ordinals in order.  crc32c_gpu_count() is that map's size and
// crc32c_batch_multi's part g runs on HIP ordinal g_gfx[g], so a node whose
// first ordinals are other parts still shards over its gfx950 devices.
std::vector<std::unique_ptr<Device>> g_devs;
std::vector<int> g_gfx;
int g_nhip = -1;
// Initialised devices by ordinal, published once (release) after init_device:
// the per-call lookup reads them without g_dev_mu, so threads driving
// different devices (crc32c_batch_multi, IO threads on several GPUs) never
// serialise on a process-wide lock after the first call.
constexpr int kMaxDevices = 64;
std::atomic<Device *> g_ready[kMaxDevices];
std::atomic<int> g_ngfx_pub{-1};

// MCRC_DEBUG=1 in the environment: report the failing HIP call on stderr.
bool debug_on() {
    static const bool on = getenv("MCRC_DEBUG") != nullptr;
    return on;
}
#define HIP_OK(x)                                                                                  \
    do {                                                                                           \
        const hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                                    \
            if (debug_on()) fprintf(stderr, "mcrc: %s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return CRC32C_EHIP;                                                                    \
        }                                                                                          \
    } while (0)

bool is_gfx950(int ordinal) {
    hipDeviceProp_t p;
    return hipGetDeviceProperties(&p, ordinal) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

int init_device(Device &d, int id) {
    d.id = id;
    HIP_OK(hipSetDevice(id));
    hipDeviceProp_t p;
    HIP_OK(hipGetDeviceProperties(&p, id));
    if (strncmp(p.gcnArchName, "gfx950", 6) != 0) return CRC32C_ENODEV;
    d.cus = p.multiProcessorCount;
    // the table image of every table kernel: slice-by-4 tables replicated per
    // bank, the lane tree on 16-B granules, the half-item fold M_2048 and the
    // shifted last steps (crc32c_gf2.h build_lds_image_span at chunk 16)
    std::vector<uint32_t> img(mcrc::kImageK1Dwords);
    mcrc::build_lds_image_span(img.data(), mcrc_dev::kK1LaneBytes);
    std::vector<uint32_t> tab8(mcrc_dev::kTab8Dwords);  // [k][b]: the byte-wise table followed by k zero bytes
    mcrc::build_t0(tab8.data());
    for (uint32_t k = 1; k < 16; ++k) {
        const mcrc::Gf2Op zk = mcrc::Gf2Op::zeros(k);
        for (uint32_t b = 0; b < 256; ++b) tab8[256 * k + b] = zk.apply(tab8[b]);
    }
    const mcrc::Gf2Op z4k = mcrc::Gf2Op::zeros(mcrc_dev::kBlockBytes);  // tables 16..19: M_4096 by byte slice
    for (uint32_t k = 0; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) tab8[256 * (16 + k) + b] = z4k.apply(b << (8 * k));
    std::vector<uint32_t> xp(mcrc_dev::kXpowDwords);
    for (uint32_t j = 0; j < 1024; ++j) {
        xp[j] = mcrc::xpow8n(j);
        xp[1024 + j] = mcrc::xpow8n((uint64_t)j << 10);
        xp[2048 + j] = mcrc::xpow8n((uint64_t)j << 20);
    }
    for (uint32_t t = 0; t < mcrc_dev::kGridAlign; ++t) xp[mcrc_dev::kXpowInv + t] = mcrc::xpow8n_inv(t);
    for (uint32_t j = 0; j < 8; ++j) xp[mcrc_dev::kXpowL3 + j] = mcrc::xpow8n((uint64_t)j << 30);
    HIP_OK(hipMalloc(&d.img, img.size() * 4));
    HIP_OK(hipMemcpy(d.img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMalloc(&d.tab8, tab8.size() * 4));
    HIP_OK(hipMemcpy(d.tab8, tab8.data(), tab8.size() * 4, hipMemcpyHostToDevice));
    // rows k (k < kSegpowLo) and kSegpowLo + j (x^(8 * 4096 * kSegpowLo j))
    // for every block shift in a 4 GiB span (a unit's shift: the blocks from
    // its end to the span's end)
    constexpr uint32_t lo = mcrc_dev::kSegpowLo;
    const uint32_t nhi = (uint32_t)((((1ull << 32) + 16) / mcrc_dev::kBlockBytes + 1 + lo - 1) / lo);
    std::vector<uint32_t> sp((lo + nhi) * 32);
    for (uint32_t k = 0; k < lo + nhi; ++k) {
        const uint64_t blocks = k < lo ? k : (uint64_t)lo * (k - lo);
        const uint32_t y = mcrc::xpow8n((uint64_t)mcrc_dev::kBlockBytes * blocks);
        for (uint32_t i = 0; i < 32; ++i) sp[k * 32 + i] = mcrc::mulmodp(0x80000000u >> i, y);
    }
    HIP_OK(hipMalloc(&d.segpow, sp.size() * 4));
    HIP_OK(hipMemcpy(d.segpow, sp.data(), sp.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMalloc(&d.xpow, xp.size() * 4));
    HIP_OK(hipMemcpy(d.xpow, xp.data(), xp.size() * 4, hipMemcpyHostToDevice));
    d.xm128 = mcrc::xpow8n_inv(128);
    HIP_OK(hipMalloc(&d.zero, mcrc_dev::kZeroBytes));
    HIP_OK(hipMemset(d.zero, 0, mcrc_dev::kZeroBytes));
    HIP_OK(hipMalloc(&d.nbad, 2 * sizeof(unsigned long long)));
    HIP_OK(hipHostMalloc(&d.hbad, 2 * sizeof(unsigned long long), hipHostMallocDefault));
    HIP_OK(hipMalloc(&d.small_nbad, 16));
    HIP_OK(hipMemset(d.small_nbad, 0, 16));
    d.small_done = reinterpret_cast<uint32_t *>(d.small_nbad + 1);
    HIP_OK(hipMalloc(&d.nfb, 2 * sizeof(uint32_t)));
    d.route = d.nfb + 1;
    HIP_OK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&d.side, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&d.fork, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&d.join, hipEventDisableTiming));
    HIP_OK(hipEventCreate(&d.ev0));
    HIP_OK(hipEventCreate(&d.ev1));
    HIP_OK(hipEventCreateWithFlags(&d.busy, hipEventDisableTiming));
    for (int k = 0; k < 2; ++k) {
        HIP_OK(hipEventCreateWithFlags(&d.copied[k], hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&d.done[k], hipEventDisableTiming));
    }
    const void *k160[] = {
        (const void *)mcrc_dev::k_fixed<false, true>,
        (const void *)mcrc_dev::k_fixed<true, true>,
        (const void *)mcrc_dev::k_fixed<false, false>,
        (const void *)mcrc_dev::k_fixed<true, false>,
        (const void *)mcrc_dev::k_spans<false>,
        (const void *)mcrc_dev::k_spans<true>,
        (const void *)mcrc_dev::k_small<0>,
        (const void *)mcrc_dev::k_small<1>,
        (const void *)mcrc_dev::k_small<2>,
        (const void *)mcrc_dev::k_blocks<false, true>,
        (const void *)mcrc_dev::k_blocks<true, true>,
        (const void *)mcrc_dev::k_blocks<true, false>,
        (const void *)mcrc_dev::k_lines<0, true>,
        (const void *)mcrc_dev::k_lines<0, false>,
        (const void *)mcrc_dev::k_lines<1, true>,
        (const void *)mcrc_dev::k_lines<2, true>,
    };
    for (const void *k : k160)
        HIP_OK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mcrc_dev::kLdsImageK1Bytes));
    d.ok = true;
    return CRC32C_OK;
}

int ensure_devices() {  // (call with g_dev_mu held): the number of gfx950 devices
    if (g_nhip < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) {
            (void)hipGetLastError();
            n = 0;
        }
        g_nhip = std::min(n, kMaxDevices);
        for (int i = 0; i < g_nhip; ++i) {
            g_devs.emplace_back(new Device());
            if (is_gfx950(i)) g_gfx.push_back(i);
        }
        g_ngfx_pub.store((int)g_gfx.size(), std::memory_order_release);
    }
    return (int)g_gfx.size();
}

int gfx_ordinal(int index) {  // library device index -> HIP ordinal (-1: none)
    std::lock_guard<std::mutex> lk(g_dev_mu);
    ensure_devices();
    return index >= 0 && index < (int)g_gfx.size() ? g_gfx[index] : -1;
}

// Device state for the calling thread's current HIP device.  After a
// device's first call this is hipGetDevice plus one acquire load.
int current_device(Device **out) {
    int id = 0;
    if (hipGetDevice(&id) != hipSuccess) return CRC32C_ENODEV;
    if (id >= 0 && id < kMaxDevices) {
        if (Device *r = g_ready[id].load(std::memory_order_acquire)) {
            *out = r;
            return CRC32C_OK;
        }
    }
    std::lock_guard<std::mutex> lk(g_dev_mu);
    ensure_devices();
    if (id < 0 || id >= g_nhip) return CRC32C_ENODEV;
    Device &d = *g_devs[id];
    if (!d.ok) {
        const int rc = init_device(d, id);
        if (rc != CRC32C_OK) return rc;
        g_ready[id].store(&d, std::memory_order_release);
    }
    *out = &d;
    return CRC32C_OK;
}

int grid_for(const Device &d, uint64_t n) {
    const uint64_t want = (n + kItemsPerBlockStep - 1) / kItemsPerBlockStep;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)d.cus));
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// Planned batches split their blocks evenly over the span kernel's 32-lane
// groups (k_expand's balanced plan; round robin over units was the round-3
// A/B baseline, profiles/r03_ablations/k2_balanced_plan_ab.jsonl).
constexpr bool kSpanBalance = true;
uint32_t span_groups(const Device &d) { return (uint32_t)d.cus * (mcrc_dev::kSpanBlock / 32); }
// Rounds of the balanced plan (k_spans): one per kRoundBytes of the batch's
// buffer, at most kMaxRounds, so the span kernel's groups stream through
// about 8 GiB of it at a time (round 5: the mixed pages at 300 pages -2 % in
// three sessions, config 3 and 1000 pages within noise; 1-4 GiB rounds'
// pipeline restarts cost as much as their locality gained at 1000 pages;
// profiles/r05_ablations/plan_rounds_ab.txt).
constexpr uint64_t kRoundBytes = 8ull << 30;
constexpr uint32_t kMaxRounds = 16;
uint32_t plan_rounds(const mcrc_dev::SpanArgs &a) {
    return (uint32_t)std::min<uint64_t>(kMaxRounds, std::max<uint64_t>(1, (a.base_bytes + kRoundBytes - 1) / kRoundBytes));
}

int ensure_plan(Device &d, uint64_t n, uint64_t cap) {
    if (d.plan_items < n) {
        (void)hipFree(d.nunit);
        (void)hipFree(d.tile_sum);
        (void)hipFree(d.tile_pre);
        (void)hipFree(d.whole);
        (void)hipFree(d.irec);
        (void)hipFree(d.span_acc);
        (void)hipFree(d.big);
        (void)hipFree(d.fast);
        (void)hipFree(d.fastidx);
        d.plan_items = 0;
        const uint64_t ntiles = (n + mcrc_dev::kPlanTile - 1) / mcrc_dev::kPlanTile;
        if (hipMalloc(&d.nunit, n * 8) != hipSuccess ||
            hipMalloc(&d.tile_sum, ntiles * sizeof(mcrc_dev::PlanSum)) != hipSuccess ||
            hipMalloc(&d.tile_pre, (ntiles + 1) * sizeof(mcrc_dev::PlanSum)) != hipSuccess ||
            hipMalloc(&d.whole, n * sizeof(mcrc_dev::UnitRec)) != hipSuccess ||
            hipMalloc(&d.irec, n * sizeof(uint4)) != hipSuccess || hipMalloc(&d.span_acc, n * 4) != hipSuccess ||
            hipMalloc(&d.big, n * sizeof(uint4)) != hipSuccess || hipMalloc(&d.fast, n) != hipSuccess ||
            hipMalloc(&d.fastidx, n * 4) != hipSuccess)
            return CRC32C_ENOMEM;
        d.plan_items = n;
    }
    if (d.plan_units < cap) {
        (void)hipFree(d.units);
        d.plan_units = 0;
        // (+ one record per share boundary of the balanced plan)
        if (hipMalloc(&d.units, (cap + (uint64_t)kMaxRounds * span_groups(d)) * sizeof(mcrc_dev::UnitRec)) != hipSuccess)
            return CRC32C_ENOMEM;
        d.plan_units = cap;
    }
    if (!d.counters && hipMalloc(&d.counters, 16) != hipSuccess) return CRC32C_ENOMEM;
    if (!d.starts && hipMalloc(&d.starts, ((uint64_t)kMaxRounds * span_groups(d) + 1) * 4) != hipSuccess)
        return CRC32C_ENOMEM;
    return CRC32C_OK;
}

// Every span of `len` bytes is one whole block at its G1 (mcrc_dev::one_block)
// whatever its alignment (p mod 128, the grid's line): the identity batch can
// go to k_blocks.
bool one_block_len(uint32_t len) {
    for (uint32_t al = 0; al < mcrc_dev::kGridAlign; ++al) {
        const uint32_t kh = al & 15u;
        const uint32_t vlen = len + ((0u - al - len) & (mcrc_dev::kGridAlign - 1)), x = vlen + kh;
        const uint32_t g1o = x - mcrc_dev::kBlockBytes * ((x - 1) / mcrc_dev::kBlockBytes) - kh;
        const bool drop = len && (g1o <= mcrc_dev::kFragMax || vlen <= mcrc_dev::kWholeMax);  // frag_drop
        if (!(drop ? vlen - g1o == mcrc_dev::kBlockBytes : len && x == mcrc_dev::kBlockBytes)) return false;
    }
    return true;
}

// Every span of `len` bytes, at any alignment, has K5's fused shape: K5 takes
// the batch whole (config 2r: 4133-B spans).  k_lines: 31 or 32 whole lines
// after a 4..131-B head, at every 128-B alignment.
bool fused_len(uint32_t len) {
    constexpr uint32_t L = mcrc_dev::kLineBytes;
    for (uint32_t al = 0; al < L; ++al) {
        const int64_t A = (al + 4 + L - 1) / L * L, B = (al + (int64_t)len) / L * L;
        if (len < 4 || !mcrc_dev::lines_fused(B - A)) return false;
    }
    return true;
}

// K5's kernel for a batch of n spans or images (k_lines: runs of 2 nsr
// consecutive images per wave, nsr up to kEpoch, enough runs for every wave).
template <int MODE, bool OFFS>
void launch_k5(const Device &d, const mcrc_dev::SpanArgs &a, mcrc_dev::ItemsOut io, hipStream_t st) {
    const int grid = grid_for(d, a.n);
    const uint64_t waves = (uint64_t)grid * (1024 / 64);
    io.xm128 = d.xm128;
    io.nsr = (uint32_t)std::min<uint64_t>(mcrc_dev::kEpoch, std::max<uint64_t>(1, (a.n + 2 * waves - 1) / (2 * waves)));
    hipLaunchKernelGGL((mcrc_dev::k_lines<MODE, OFFS>), dim3(grid), dim3(1024), mcrc_dev::kLdsImageK1Bytes, st, a,
                       d.img, io);
}

// Large item batches go through launch_items, where k_census samples their
// headers on the device and routes them to K5 (one-block images: 4 KiB
// values, configs 1 and 5) or to the planned path.
bool items_fused(const mcrc_dev::SpanArgs &a) { return a.n >= 4096; }

// Batches of at most g_small_max spans take the single-launch k_small
// (crc32c_set_small_max changes it; the parity tests run every case through
// both paths).
constexpr uint64_t kSmallSpanMax = 1 << 20;   // fixed-length batches: spans up to 1 MiB
constexpr uint64_t kSmallBaseMax = 8ull << 20;  // else: a buffer of at most 8 MiB (a wbuf, an IO batch)
std::atomic<uint64_t> g_small_max{mcrc_dev::kSmallMax};

// One launch (k_small) for small batches whose spans are bounded: a group
// reads its whole span alone, so a batch of a few multi-MiB spans is left to
// the planned path (segments over the whole grid).  Decided once per call.
template <int MODE>
bool takes_small(const mcrc_dev::SpanArgs &a) {
    const bool bounded = MODE == 0 && a.lens == nullptr ? a.len <= kSmallSpanMax : a.base_bytes <= kSmallBaseMax;
    return a.n <= g_small_max.load(std::memory_order_relaxed) && bounded;
}

// k_small over a's spans on st.  Spans per workgroup: enough workgroups to
// reach every CU (one fits a CU: 160 KiB of tables), at least 8 so that each
// workgroup's table copy stays a few round trips (2-32 measured,
// DESIGN.md section 3).  host_counted: a.nbad / host_nbad / done are k_small's
// own counters and the count arrives in *host_nbad.
template <int MODE>
int launch_small(const Device &d, const mcrc_dev::SpanArgs &a, hipStream_t st) {
    const uint64_t n = a.n;
    uint64_t per = (n + d.cus - 1) / std::max(d.cus, 1);
    per = std::min<uint64_t>(32, std::max<uint64_t>(8, (per + 1) & ~1ull));
    hipLaunchKernelGGL((mcrc_dev::k_small<MODE>), dim3((unsigned)((n + per - 1) / per)), dim3((unsigned)(32 * per)),
                       mcrc_dev::kLdsImageK1Bytes, st, a, d.img);
    HIP_OK(hipGetLastError());
    return CRC32C_OK;
}

// Unit capacity of a planned batch: units fit whenever the spans do not
// overlap; overlapping long spans past it are processed whole by the second
// span pass.
uint64_t plan_cap(const mcrc_dev::SpanArgs &a) {
    return std::min<uint64_t>(a.n + a.base_bytes / mcrc_dev::kSegBytes + 1 + a.n / 4096, 0xfffffff0ull);
}

// How a batch runs, decided once by the caller:
//   small:        one k_small launch (takes_small);
//   host_counted: (small only) k_small counts into d.small_nbad and its last
//                 workgroup hands the count to the pinned word d.hbad (no
//                 memset, no copy); else the caller zeroes and reads d.nbad;
//   counted:      the plan entries of k_count are already written (the page
//                 walk's second pass).
struct Path {
    bool small = false, host_counted = false, counted = false;
};

template <int MODE>
int launch_units(Device &d, mcrc_dev::SpanArgs a, hipStream_t st, Path path) {
    const uint64_t n = a.n;
    const bool identity = MODE == 0 && a.lens == nullptr && a.len <= mcrc_dev::kSegBytes;
    auto spans = [&](const mcrc_dev::SpanArgs &x, int grid) {
        if (x.units)
            hipLaunchKernelGGL((mcrc_dev::k_spans<true>), dim3(grid), dim3(mcrc_dev::kSpanBlock),
                               mcrc_dev::kLdsImageK1Bytes, st, x, d.img);
        else
            hipLaunchKernelGGL((mcrc_dev::k_spans<false>), dim3(grid), dim3(mcrc_dev::kSpanBlock),
                               mcrc_dev::kLdsImageK1Bytes, st, x, d.img);
    };
    const int g1 = (int)std::min<uint64_t>((n + 255) / 256, 2048);
    // k_final: 1024 workgroups (it adds its bad count once per workgroup: 4096
    // groups cost 30 us of same-address atomics per 4.8 M verified items, 64 Ki
    // groups 190 us); k_count: 2048 (round 5: config 3 and the mixed pages
    // 0.2-1.2 % faster than 4096, 1024 no better and config 5 +1.3 %;
    // profiles/r05_ablations/k_count_grid_ab.txt; round 4 measured 1024 25 %
    // slower than 4096 on config 3 before the whole spans went wave-wide).
    const int gf = (int)std::min<uint64_t>((n + 255) / 256, 1024);
    if (path.small) {
        if (path.host_counted) {
            a.nbad = d.small_nbad;
            a.host_nbad = d.hbad;
            a.done = d.small_done;
        }
        return launch_small<MODE>(d, a, st);
    }
    if (identity && fused_len(a.len) && n < 0xffffffffull) {  // K5: one block after a head fragment
        mcrc_dev::ItemsOut io{};  // (MODE 0: K5 stores every CRC itself)
        if (a.offsets) launch_k5<0, true>(d, a, io, st);
        else launch_k5<0, false>(d, a, io, st);
        HIP_OK(hipGetLastError());
        return CRC32C_OK;
    }
    if (identity) {
        // (spans of at most kWholeMax - (kGridAlign - 1) bytes are all their threads' in k_final)
        if (a.len + mcrc_dev::kGridAlign - 1 > mcrc_dev::kWholeMax) {
            if (one_block_len(a.len) && a.offsets)
                hipLaunchKernelGGL((mcrc_dev::k_blocks<true, true>), dim3(grid_for(d, n)), dim3(1024),
                                   mcrc_dev::kLdsImageK1Bytes, st, a, d.img, (const uint4 *)nullptr,
                                   (const uint32_t *)nullptr, (const uint32_t *)nullptr);
            else if (one_block_len(a.len))
                hipLaunchKernelGGL((mcrc_dev::k_blocks<true, false>), dim3(grid_for(d, n)), dim3(1024),
                                   mcrc_dev::kLdsImageK1Bytes, st, a, d.img, (const uint4 *)nullptr,
                                   (const uint32_t *)nullptr, (const uint32_t *)nullptr);
            else
                spans(a, grid_for(d, n));
        }
        hipLaunchKernelGGL((mcrc_dev::k_final<0, false>), dim3(gf), dim3(256), 0, st, a, nullptr);
        HIP_OK(hipGetLastError());
        return CRC32C_OK;
    }
    if (n >= 0xffffffffull) return CRC32C_EINVAL;
    const uint64_t cap = plan_cap(a);
    int rc = ensure_plan(d, n, cap);
    if (rc) return rc;
    uint32_t *nvalid = d.counters, *nwhole = d.counters + 1, *nbig = d.counters + 2;
    HIP_OK(hipMemsetAsync(nvalid, 0, 12, st));  // nvalid, nwhole, nbig
    // the balanced plan's shares: rounds x the span kernel's groups
    const uint32_t rounds = kSpanBalance ? plan_rounds(a) : 1u;
    const uint32_t shares = rounds * span_groups(d);
    if (kSpanBalance) HIP_OK(hipMemsetAsync(d.starts, 0xff, ((uint64_t)shares + 1) * 4, st));
    a.span_acc = d.span_acc;
    if (!path.counted)
        hipLaunchKernelGGL((mcrc_dev::k_count<MODE>), dim3(g1), dim3(256), 0, st, a, d.nunit, d.irec, d.fast);
    // prefix sums of the plan (units, blocks, one-block spans): tile sums, one
    // workgroup over them, then each tile rescanned where k_expand uses it
    const uint64_t ntiles = (n + mcrc_dev::kPlanTile - 1) / mcrc_dev::kPlanTile;
    const int gt = (int)std::min<uint64_t>(ntiles, 4096);
    // (a.dn: n is the list's upper bound and its length is read on the device)
    hipLaunchKernelGGL(mcrc_dev::k_plan_tiles, dim3(gt), dim3(mcrc_dev::kPlanThreads), 0, st,
                       (const uint64_t *)d.nunit, (const uint8_t *)d.fast, n, a.dn, d.tile_sum);
    mcrc_dev::PlanSum *total = d.tile_pre + ntiles;
    hipLaunchKernelGGL(mcrc_dev::k_plan_scan, dim3(1), dim3(mcrc_dev::kPlanThreads), 0, st,
                       (const mcrc_dev::PlanSum *)d.tile_sum, n, a.dn, d.tile_pre, total);
    const uint32_t *nfast = &total->fast;
    uint32_t *const starts = kSpanBalance ? d.starts : nullptr;
    hipLaunchKernelGGL(mcrc_dev::k_expand, dim3(gt), dim3(mcrc_dev::kPlanThreads), 0, st, a.base,
                       (const uint64_t *)d.nunit, (const uint8_t *)d.fast, (const mcrc_dev::PlanSum *)d.tile_pre,
                       (const mcrc_dev::PlanSum *)total, (const uint4 *)d.irec, n, a.dn, d.units, cap, nvalid, d.whole,
                       nwhole, d.big, nbig, d.fastidx, shares, starts);
    hipLaunchKernelGGL(mcrc_dev::k_expand_big, dim3(1024), dim3(256), 0, st, a.base, (const uint64_t *)d.nunit,
                       (const mcrc_dev::PlanSum *)total, (const uint4 *)d.irec, d.units, (const uint4 *)d.big,
                       (const uint32_t *)nbig, n, a.dn, shares, starts);
    mcrc_dev::SpanArgs u = a;
    u.units = d.units;
    u.nunits = nvalid;
    u.span_acc = d.span_acc;
    u.segpow = d.segpow;
    u.starts = starts;
    u.rounds = rounds;
    // spans whose unit is one whole block: k_blocks over the compacted list;
    // the other spans' units: the span kernel
    hipLaunchKernelGGL((mcrc_dev::k_blocks<false, true>), dim3(grid_for(d, n)), dim3(1024), mcrc_dev::kLdsImageK1Bytes, st,
                       u, d.img, (const uint4 *)d.irec, (const uint32_t *)d.fastidx, (const uint32_t *)nfast);
    spans(u, d.cus);
    mcrc_dev::SpanArgs w = u;  // (every table pointer set, even those whole units do not use)
    w.units = d.whole;
    w.nunits = nwhole;
    w.starts = nullptr;
    spans(w, d.cus);
    hipLaunchKernelGGL((mcrc_dev::k_final<MODE, true>), dim3(gf), dim3(256), 0, st, u, d.irec);
    HIP_OK(hipGetLastError());
    return CRC32C_OK;
}

// K5 over the item images of a (MODE 1 verify, MODE 2 stamp; device memory,
// a.nbad zeroed by the caller): k_census routes the batch on the device,
// k_lines checksums the one-block images (+ k_fix for stamps) and lists the
// others, and the planned path takes that list with its length read on the
// device (a.dn).  Nothing is read back: an async stamp stays async.
template <int MODE>
int launch_items(Device &d, mcrc_dev::SpanArgs a, hipStream_t st) {
    const uint64_t n = a.n;
    if (n >= 0xffffffffull) return CRC32C_EINVAL;
    mcrc_dev::ItemsOut io{};
    io.fb = (uint32_t *)d.grow(kScrFb, n * 4);
    io.nfb = d.nfb;
    io.route = d.route;
    if (MODE == 2) io.rt = (uint2 *)d.grow(kScrRt, n * 8);
    uint64_t *fo = (uint64_t *)d.grow(kScrFbOffs, n * 8);
    uint8_t *fok = (uint8_t *)d.grow(kScrFbOk, n);
    if (!io.fb || (MODE == 2 && !io.rt) || !fo || !fok) return CRC32C_ENOMEM;
    HIP_OK(hipMemsetAsync(d.nfb, 0, 4, st));
    hipLaunchKernelGGL(mcrc_dev::k_census<MODE>, dim3(1), dim3(mcrc_dev::kCensus), 0, st, a, d.route);
    launch_k5<MODE, true>(d, a, io, st);
    const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 1024);
    // Once k_fix is forked, every exit joins it back into st, error exits
    // included: the caller's busy event (recorded on st after this returns)
    // must cover k_fix's writes to the images and its reads of io.rt.
    struct Join {
        hipStream_t st;
        hipEvent_t ev;
        bool armed = false;
        ~Join() {
            if (armed) (void)hipStreamWaitEvent(st, ev, 0);
        }
    } join{st, d.join};
    if (MODE == 2) {
        // k_fix (the stamps of the images k_lines checksummed) on the side
        // stream, beside the planned path of the images it listed: its
        // scattered partial-sector writes and that path's small launches
        // overlap.  They touch disjoint bytes unless images overlap
        // (crc32c_batch.h: then an image's CRC may or may not see another
        // image's new stamp).
        HIP_OK(hipEventRecord(d.fork, st));
        HIP_OK(hipStreamWaitEvent(d.side, d.fork, 0));
        hipLaunchKernelGGL(mcrc_dev::k_fix, dim3(g), dim3(256), 0, d.side, a, (const uint2 *)io.rt,
                           (const uint32_t *)d.route, d.xm128);
        HIP_OK(hipEventRecord(d.join, d.side));
        join.armed = true;
    }
    hipLaunchKernelGGL(mcrc_dev::k_gather_offs, dim3(g), dim3(256), 0, st, a.offsets, (const uint32_t *)io.fb,
                       (const uint32_t *)d.nfb, fo, (const uint32_t *)d.route);
    HIP_OK(hipGetLastError());
    mcrc_dev::SpanArgs f = a;
    const bool want_ok = MODE == 1 || a.ok;
    f.offsets = fo;
    f.dn = d.nfb;  // (f.n = n: the list's upper bound)
    f.ok = want_ok ? fok : nullptr;
    int rc = launch_units<MODE>(d, f, st, Path{});
    if (MODE == 2) {
        join.armed = false;
        HIP_OK(hipStreamWaitEvent(st, d.join, 0));  // (also when the planned path failed)
    }
    if (rc) return rc;
    if (want_ok)
        hipLaunchKernelGGL(mcrc_dev::k_scatter_ok, dim3(g), dim3(256), 0, st, (const uint8_t *)fok,
                           (const uint32_t *)io.fb, (const uint32_t *)d.nfb, a.ok, (const uint32_t *)d.route);
    HIP_OK(hipGetLastError());
    return CRC32C_OK;
}

// Enqueue the kernels for a device-resident batch on `st`.
// Equal spans at a fixed stride must fit [base, base + base_bytes): checked
// here (the kernels read them unchecked).  Spans given by device offsets or
// lengths are checked by the span kernels (out-of-range ones are not read).
bool fixed_spans_fit(const crc32c_spans &s) {
    if (!s.lens && s.len > mcrc_dev::kMaxSpan) return false;
    if (s.offsets || s.lens) return true;
    if (s.len > s.base_bytes) return false;
    if (s.n <= 1 || s.stride == 0) return true;
    return (s.n - 1) <= (s.base_bytes - s.len) / s.stride;
}

mcrc_dev::SpanArgs span_args(const Device &d, const crc32c_spans &s) {
    mcrc_dev::SpanArgs a{};
    a.base = (const uint8_t *)s.base;
    a.base_bytes = s.base_bytes;
    a.offsets = s.offsets;
    a.stride = s.stride;
    a.lens = s.lens;
    a.len = s.len;
    a.crc_in = s.crc_in;
    a.out = s.out;
    a.nbad = d.nbad;  // spans outside the buffer
    a.n = s.n;
    a.segpow = d.segpow;
    a.xpow = d.xpow;
    a.tab8 = d.tab8;
    a.zero = d.zero;
    a.cfl = 4;
    return a;
}

// want_host_count (synchronous callers only): a small batch's out-of-range
// count comes back in d.hbad from k_small itself (no memset, no copy);
// *host_counted says whether that happened.
// K1's batch shape: equal 4 KiB spans at a 16-B aligned base and stride (the
// lane offset within a step, item * stride, is 32-bit in K1).
bool k1_shape(const crc32c_spans &s) {
    return s.offsets == nullptr && s.lens == nullptr && s.len == kFixedLen && aligned16(s.base) &&
           (s.stride & 15u) == 0 && s.stride < (1ull << 31);
}

// K1 touches no shared scratch, counter or event of the device: callers may
// enqueue it without d.mu.
// Non-temporal loads only when every 128-B line belongs to one item.
int launch_k1(const Device &d, const crc32c_spans &s, hipStream_t st) {
    const bool nt = ((uintptr_t)s.base & 127u) == 0 && (s.stride & 127u) == 0;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid_for(d, s.n)), dim3(kBlock), mcrc_dev::kLdsImageK1Bytes, st,
                           (const uint8_t *)s.base, s.stride, s.n, (const uint4 *)d.img, (const uint32_t *)s.crc_in,
                           s.out);
    };
    if (s.crc_in) nt ? go(mcrc_dev::k_fixed<true, true>) : go(mcrc_dev::k_fixed<true, false>);
    else nt ? go(mcrc_dev::k_fixed<false, true>) : go(mcrc_dev::k_fixed<false, false>);
    HIP_OK(hipGetLastError());
    return CRC32C_OK;
}

int enqueue_device(Device &d, const crc32c_spans &s, hipStream_t st, bool want_host_count = false,
                   bool *host_counted = nullptr) {
    if (host_counted) *host_counted = false;
    if (s.n == 0) return CRC32C_OK;
    if (!fixed_spans_fit(s)) return CRC32C_EINVAL;
    if (k1_shape(s)) return launch_k1(d, s, st);
    const mcrc_dev::SpanArgs a = span_args(d, s);
    Path path;
    path.small = takes_small<0>(a);
    path.host_counted = path.small && want_host_count;
    if (!path.host_counted) HIP_OK(hipMemsetAsync(d.nbad, 0, sizeof(unsigned long long), st));
    if (host_counted) *host_counted = path.host_counted;
    return launch_units<0>(d, a, st, path);
}

// [p, p + bytes) lies inside one device allocation (so no kernel read bounded
// by it can fault).  Memory the runtime cannot describe (e.g. host-registered
// or managed) is not checked.
bool device_range_ok(const void *p, uint64_t bytes) {
    hipDeviceptr_t lo = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&lo, &size, (hipDeviceptr_t)p) != hipSuccess || lo == nullptr) {
        (void)hipGetLastError();
        return true;
    }
    const uint64_t skip = (uint64_t)((const uint8_t *)p - (const uint8_t *)lo);
    return skip <= size && bytes <= size - skip;
}

const uint8_t *device_view_range(const void *p, uint64_t bytes);

// [p, p + bytes) can be the source of one DMA as it lies: device or managed
// memory, or host memory page-locked over the whole range.
bool is_pinned_or_device(const void *p, uint64_t bytes) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type == hipMemoryTypeHost) return device_view_range(p, bytes) != nullptr;
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

// The address a kernel reads host memory p at, when p is page-locked and
// mapped (crc32c_host_alloc, hipHostMalloc, crc32c_host_register); nullptr for
// pageable memory.
const uint8_t *device_view(const void *p) {
    hipPointerAttribute_t at;
    if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost) return nullptr;
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, const_cast<void *>(p), 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return (const uint8_t *)dp;
}

// The device address of the whole host range [p, p + bytes) when every byte
// of it is page-locked and mapped as one contiguous range, else nullptr (the
// caller then stages the batch).  A caller may have registered only part of
// an arena, or pass a base_bytes past the end of its hipHostMalloc buffer: a
// kernel reading such a range in place would page-fault.  The runtime's
// record of the allocation or registration holding p must cover the range;
// where the runtime cannot describe it, both ends must map, to addresses
// bytes - 1 apart.
const uint8_t *device_view_range(const void *p, uint64_t bytes) {
    const uint8_t *dv = device_view(p);
    if (!dv || bytes <= 1) return dv;
    const uint8_t *h = (const uint8_t *)p;
    hipDeviceptr_t lo = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&lo, &size, (hipDeviceptr_t)p) == hipSuccess && lo) {
        // (the base comes back as the host or as the device address of the range)
        for (const uint8_t *q : {h, dv}) {
            const uint8_t *b = (const uint8_t *)lo;
            if (q >= b && (uint64_t)(q - b) <= size) return bytes <= size - (uint64_t)(q - b) ? dv : nullptr;
        }
        return nullptr;
    }
    (void)hipGetLastError();
    return device_view(h + bytes - 1) == dv + (bytes - 1) ? dv : nullptr;
}

uint64_t span_off(const crc32c_spans &s, uint64_t i) { return s.offsets ? s.offsets[i] : i * s.stride; }
uint64_t span_len(const crc32c_spans &s, uint64_t i) { return s.lens ? s.lens[i] : s.len; }

int ensure_slots(Device &d, uint64_t bytes, uint64_t items) {
    if (d.slot_bytes < bytes) {
        for (int k = 0; k < 2; ++k) {
            if (d.dbuf[k]) (void)hipFree(d.dbuf[k]);
            if (d.pin[k]) (void)hipHostFree(d.pin[k]);
            d.dbuf[k] = nullptr;
            d.pin[k] = nullptr;
            if (hipMalloc(&d.dbuf[k], bytes) != hipSuccess) return CRC32C_ENOMEM;
            if (hipHostMalloc(&d.pin[k], bytes, hipHostMallocDefault) != hipSuccess) return CRC32C_ENOMEM;
        }
        d.slot_bytes = bytes;
    }
    if (d.slot_items < items) {
        for (int k = 0; k < 2; ++k) {
            (void)hipFree(d.doffs[k]);
            (void)hipFree(d.dlens[k]);
            (void)hipFree(d.dcin[k]);
            (void)hipFree(d.dout[k]);
            (void)hipHostFree(d.hoffs[k]);
            (void)hipHostFree(d.hlens[k]);
            (void)hipHostFree(d.hcin[k]);
            (void)hipHostFree(d.hout[k]);
            if (hipMalloc(&d.doffs[k], items * 8) != hipSuccess || hipMalloc(&d.dlens[k], items * 4) != hipSuccess ||
                hipMalloc(&d.dcin[k], items * 4) != hipSuccess || hipMalloc(&d.dout[k], items * 4) != hipSuccess ||
                hipHostMalloc(&d.hoffs[k], items * 8, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc(&d.hlens[k], items * 4, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc(&d.hcin[k], items * 4, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc(&d.hout[k], items * 4, hipHostMallocDefault) != hipSuccess)
                return CRC32C_ENOMEM;
        }
        d.slot_items = items;
    }
    return CRC32C_OK;
}

constexpr uint64_t kSlotBytes = 256ull << 20;  // bytes of span data per pipeline stage
constexpr uint64_t kSlotItems = 1ull << 20;

// Host spans must lie in [base, base + base_bytes) and fit a pipeline slot.
bool host_spans_ok(const crc32c_spans &s) {
    for (uint64_t i = 0; i < s.n; ++i) {
        const uint64_t off = span_off(s, i), len = span_len(s, i);
        if (off > s.base_bytes || len > s.base_bytes - off || len > kSlotBytes - 16) return false;
    }
    return true;
}

// Host-resident batch on one device.  Spans are staged in offset order (a
// permutation when the caller's order is not sorted: chunked-item iov lists
// keep their chain order) in chunks that go through two pipeline slots: while
// chunk c is checksummed, chunk c+1 is staged into pinned memory (unless the
// caller's buffer is already pinned) and copied H2D on the copy stream.
// Descriptors and results travel through pinned twins so no copy touches
// pageable memory; results are scattered back to the caller's order.
int run_host_batch(Device &d, const crc32c_spans &s) {
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_OK(hipSetDevice(d.id));
    if (s.n == 0) return CRC32C_OK;
    if (!host_spans_ok(s)) return CRC32C_EINVAL;
    std::vector<uint64_t> order;  // staging order -> caller index (empty: identity)
    for (uint64_t i = 1; i < s.n; ++i)
        if (span_off(s, i) < span_off(s, i - 1)) {
            order.resize(s.n);
            for (uint64_t k = 0; k < s.n; ++k) order[k] = k;
            std::stable_sort(order.begin(), order.end(),
                             [&](uint64_t x, uint64_t y) { return span_off(s, x) < span_off(s, y); });
            break;
        }
    auto idx = [&](uint64_t k) { return order.empty() ? k : order[k]; };
    int rc = ensure_slots(d, kSlotBytes, kSlotItems);
    if (rc) return rc;
    d.acquire(d.stream);
    d.acquire(d.copy);
    // Every exit waits for both streams (an H2D copy may still be reading the
    // caller's pinned buffer after an error) and hands the scratch on.
    struct Guard {
        Device &d;
        ~Guard() {
            (void)hipStreamSynchronize(d.copy);
            (void)hipStreamSynchronize(d.stream);
            d.release(d.stream);
        }
    } guard{d};
    const bool src_pinned = is_pinned_or_device(s.base, s.base_bytes);
    const uint8_t *src = (const uint8_t *)s.base;
    uint64_t pend_k0[2] = {0, 0}, pend_n[2] = {0, 0};  // results waiting in hout[slot]
    auto drain = [&](int k) -> int {
        if (!pend_n[k]) return CRC32C_OK;
        HIP_OK(hipEventSynchronize(d.done[k]));
        if (order.empty()) memcpy(s.out + pend_k0[k], d.hout[k], pend_n[k] * 4);
        else
            for (uint64_t i = 0; i < pend_n[k]; ++i) s.out[order[pend_k0[k] + i]] = d.hout[k][i];
        pend_n[k] = 0;
        return CRC32C_OK;
    };
    uint64_t k0 = 0;
    int slot = 0;
    while (k0 < s.n) {
        const uint64_t lo = span_off(s, idx(k0)) & ~15ull;
        uint64_t k1 = k0, hi = lo;
        while (k1 < s.n && k1 - k0 < kSlotItems) {
            const uint64_t e = span_off(s, idx(k1)) + span_len(s, idx(k1));
            if (std::max(hi, e) - lo > kSlotBytes) break;
            hi = std::max(hi, e);
            ++k1;
        }
        const uint64_t bytes = hi - lo, cnt = k1 - k0;
        if ((rc = drain(slot))) return rc;  // slot free: its kernel and D2H are done
        const uint8_t *h2d_src = src + lo;
        if (!src_pinned) {
            memcpy(d.pin[slot], src + lo, bytes);
            h2d_src = d.pin[slot];
        }
        for (uint64_t i = 0; i < cnt; ++i) {
            const uint64_t c = idx(k0 + i);
            d.hoffs[slot][i] = span_off(s, c) - lo;
            if (s.lens) d.hlens[slot][i] = s.lens[c];
            if (s.crc_in) d.hcin[slot][i] = s.crc_in[c];
        }
        HIP_OK(hipMemcpyAsync(d.dbuf[slot], h2d_src, bytes, hipMemcpyHostToDevice, d.copy));
        HIP_OK(hipMemcpyAsync(d.doffs[slot], d.hoffs[slot], cnt * 8, hipMemcpyHostToDevice, d.copy));
        if (s.lens) HIP_OK(hipMemcpyAsync(d.dlens[slot], d.hlens[slot], cnt * 4, hipMemcpyHostToDevice, d.copy));
        if (s.crc_in) HIP_OK(hipMemcpyAsync(d.dcin[slot], d.hcin[slot], cnt * 4, hipMemcpyHostToDevice, d.copy));
        HIP_OK(hipEventRecord(d.copied[slot], d.copy));
        HIP_OK(hipStreamWaitEvent(d.stream, d.copied[slot], 0));
        crc32c_spans sub{};
        sub.base = d.dbuf[slot];
        sub.base_bytes = bytes;
        sub.offsets = d.doffs[slot];
        sub.lens = s.lens ? d.dlens[slot] : nullptr;
        sub.len = s.len;
        sub.crc_in = s.crc_in ? d.dcin[slot] : nullptr;
        sub.out = d.dout[slot];
        sub.n = cnt;
        if ((rc = enqueue_device(d, sub, d.stream))) return rc;
        HIP_OK(hipMemcpyAsync(d.hout[slot], d.dout[slot], cnt * 4, hipMemcpyDeviceToHost, d.stream));
        HIP_OK(hipEventRecord(d.done[slot], d.stream));
        pend_k0[slot] = k0;
        pend_n[slot] = cnt;
        k0 = k1;
        slot ^= 1;
    }
    if ((rc = drain(slot)) || (rc = drain(slot ^ 1))) return rc;
    return CRC32C_OK;
}

// Synchronous device batch on `st` (the body of crc32c_batch for
// CRC32C_DEVICE): records the kernel time; ERANGE when a span lay outside the
// buffer.
int device_batch(Device &d, const crc32c_spans &s, unsigned flags, hipStream_t st) {
    if (s.n && !device_range_ok(s.base, s.base_bytes)) return CRC32C_EINVAL;
    // an asynchronous K1 batch needs nothing the lock guards (no scratch, no
    // timing events): IO or device threads enqueue it concurrently
    if ((flags & CRC32C_ASYNC) && s.n && k1_shape(s))
        return fixed_spans_fit(s) ? launch_k1(d, s, st) : CRC32C_EINVAL;
    std::lock_guard<std::mutex> lk(d.mu);
    const bool timed = !(flags & CRC32C_ASYNC);
    d.acquire(st);
    if (timed) HIP_OK(hipEventRecord(d.ev0, st));
    bool host_counted = false;
    int rc = enqueue_device(d, s, st, timed, &host_counted);
    if (rc) {
        d.release(st);
        return rc;
    }
    if (!timed) {
        d.release(st);
        return CRC32C_OK;
    }
    HIP_OK(hipEventRecord(d.ev1, st));
    // spans given by offsets / lengths are range-checked on the device
    unsigned long long nrange = 0;
    const bool checked = s.n && (s.offsets || s.lens);
    if (checked && !host_counted) HIP_OK(hipMemcpyAsync(d.hbad, d.nbad, sizeof nrange, hipMemcpyDeviceToHost, st));
    d.release(st);
    HIP_OK(hipEventSynchronize(d.ev1));
    if (checked) {
        HIP_OK(hipStreamSynchronize(st));
        nrange = *d.hbad;
    }
    (void)hipEventElapsedTime(&g_last_kernel_ms, d.ev0, d.ev1);
    return nrange ? CRC32C_ERANGE : CRC32C_OK;
}

// Item-image batches (verify: MODE 1, stamp: MODE 2) over a packed buffer of
// item images at item_offsets.
//   device: in place on the caller's stream;
//   host, small (at most 8 MiB, a wbuf or an IO batch): one k_small launch on
//     the library stream that reads the images where they are when the buffer
//     is page-locked (crc32c_host_alloc / _register; stamps are written into
//     it in place), else from a pinned copy; descriptors and results through
//     pinned mapped scratch -- no device allocation, no copy engine;
//   host, large: staged into grow-only device scratch, planned kernels.
template <int MODE>
int item_images(void *base, uint64_t base_bytes, uint64_t region_bytes, const uint64_t *item_offsets, uint64_t n,
                uint8_t *ok, uint64_t *nbad, unsigned flags, void *stream) {
    if (!base || !item_offsets || (MODE == 1 && !ok)) return CRC32C_EINVAL;
    Device *d = nullptr;
    int rc = current_device(&d);
    if (rc) return rc;
    if (n == 0) {
        if (nbad) *nbad = 0;
        return CRC32C_OK;
    }
    const bool dev = flags & CRC32C_DEVICE;
    if (dev && !device_range_ok(base, base_bytes)) return CRC32C_EINVAL;
    mcrc_dev::SpanArgs a{};
    a.base = (const uint8_t *)base;
    a.base_bytes = base_bytes;
    a.offsets = item_offsets;
    a.nbad = d->nbad;
    a.n = n;
    a.xpow = d->xpow;
    a.tab8 = d->tab8;
    a.zero = d->zero;
    a.region = region_bytes;
    a.cfl = (flags & CRC32C_CFLAGS64) ? 8u : 4u;
    Path path;
    path.small = takes_small<MODE>(a);
    std::lock_guard<std::mutex> lk(d->mu);
    if (dev) {
        hipStream_t st = (hipStream_t)stream;  // NULL: the default stream
        a.ok = ok;
        a.out = nullptr;  // stamp: write into the images
        path.host_counted = path.small;
        // large batches: K5 or the planned path, routed on the device
        const bool k5 = !path.small && items_fused(a);
        d->acquire(st);
        if (!path.host_counted) (void)hipMemsetAsync(d->nbad, 0, sizeof(unsigned long long), st);
        rc = k5 ? launch_items<MODE>(*d, a, st) : launch_units<MODE>(*d, a, st, path);
        if (!rc && !path.host_counted)
            rc = hipMemcpyAsync(d->hbad, d->nbad, sizeof(unsigned long long), hipMemcpyDeviceToHost, st) == hipSuccess
                     ? CRC32C_OK
                     : CRC32C_EHIP;
        d->release(st);
        if (rc) return rc;
        if ((flags & CRC32C_ASYNC) && !nbad) return CRC32C_OK;  // fire and forget
        HIP_OK(hipStreamSynchronize(st));
        if (nbad) *nbad = *d->hbad;
        return CRC32C_OK;
    }
    hipStream_t st = d->stream;
    HIP_OK(hipSetDevice(d->id));
    d->acquire(st);
    struct Release {
        Device *d;
        hipStream_t st;
        ~Release() {
            (void)hipStreamSynchronize(st);
            d->release(st);
        }
    } release_on_exit{d, st};
    void *h_offs, *v_offs, *h_ok, *v_ok, *h_crc = nullptr, *v_crc = nullptr;
    if (!d->grow_pinned(kPinOffs, n * 8, &h_offs, &v_offs) || !d->grow_pinned(kPinOk, n, &h_ok, &v_ok))
        return CRC32C_ENOMEM;
    memcpy(h_offs, item_offsets, n * 8);
    const uint8_t *mapped = device_view_range(base, base_bytes);
    // stamp results come back as CRCs (scattered into the caller's images
    // here) unless the kernel stamps the caller's page-locked buffer itself
    const bool crcs_back = MODE == 2 && !(path.small && mapped);
    if (crcs_back && !d->grow_pinned(kPinCrc, n * 4, &h_crc, &v_crc)) return CRC32C_ENOMEM;
    a.ok = (uint8_t *)v_ok;
    a.out = (uint32_t *)v_crc;
    if (path.small) {
        if (!mapped) {  // a pinned copy the kernel reads
            void *h_stage, *v_stage;
            if (!d->grow_pinned(kPinStage, base_bytes, &h_stage, &v_stage)) return CRC32C_ENOMEM;
            memcpy(h_stage, base, base_bytes);
            mapped = (const uint8_t *)v_stage;
        }
        a.base = mapped;
        a.offsets = (const uint64_t *)v_offs;
        path.host_counted = true;
        if ((rc = launch_units<MODE>(*d, a, st, path))) return rc;
    } else {
        uint8_t *b = (uint8_t *)d->grow(kScrStage, base_bytes);
        uint64_t *o = (uint64_t *)d->grow(kScrItemOffs, n * 8);
        uint8_t *r = (uint8_t *)d->grow(kScrItemOut, n * 5 + 4);  // ok[n], then (4-B aligned) crc[n]
        if (!b || !o || !r) return CRC32C_ENOMEM;
        HIP_OK(hipMemcpyAsync(b, base, base_bytes, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(o, h_offs, n * 8, hipMemcpyHostToDevice, st));
        a.base = b;
        a.offsets = o;
        a.ok = r;
        a.out = crcs_back ? (uint32_t *)(r + ((n + 3) & ~3ull)) : nullptr;
        HIP_OK(hipMemsetAsync(d->nbad, 0, sizeof(unsigned long long), st));
        if ((rc = launch_units<MODE>(*d, a, st, path))) return rc;
        HIP_OK(hipMemcpyAsync(h_ok, a.ok, n, hipMemcpyDeviceToHost, st));
        if (crcs_back) HIP_OK(hipMemcpyAsync(h_crc, a.out, n * 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipMemcpyAsync(d->hbad, d->nbad, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    const uint8_t *oks = (const uint8_t *)h_ok;
    if (crcs_back) {
        uint8_t *bb = (uint8_t *)base;
        const uint32_t *crcs = (const uint32_t *)h_crc;
        for (uint64_t i = 0; i < n; ++i)
            if (oks[i]) memcpy(bb + item_offsets[i] + 28, &crcs[i], 4);  // exptime (storage.c:567)
    }
    if (ok) memcpy(ok, oks, n);
    if (nbad) *nbad = *d->hbad;
    return CRC32C_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// Coalescing queue (crc32c_batch_submit / _wait)
// ---------------------------------------------------------------------------
// The read-verify CRCs arrive from many IO threads, each with a batch of at
// most io_depth reads (extstore.c:853-945; io_depth = 1 by default,
// storage.c:1339).  One synchronous GPU call per such batch costs a launch and
// a round trip per thread; the queue instead lets every thread enqueue its
// spans and a per-device dispatcher packs whatever is pending into one k_small
// launch, reading the spans where they lie in page-locked host memory
// (group commit: while one launch runs, the next batch accumulates).
struct crc32c_job {
    crc32c_spans s;
    unsigned flags = 0;
    // CRC32C_DEVICE jobs: recorded on the submitter's default stream, waited
    // for by the queue's stream before the job runs (work the caller queued on
    // the default stream, e.g. the copy filling the spans, stays ordered first)
    hipEvent_t after = nullptr;
    const uint8_t *dbase = nullptr;  // coalesced jobs: the device view of s.base
    bool coalesce = false;
    int rc = CRC32C_OK;
    std::atomic<int> done{0};
    Queue *q = nullptr;
};

namespace {

constexpr uint64_t kQueueSpanMax = 256u << 10;  // longer spans: the job runs alone (planned path)
static_assert(sizeof(std::atomic<int>) == sizeof(int) && std::atomic<int>::is_always_lock_free,
              "crc32c_job::done is waited on as a futex word");

struct Queue {
    Device *d = nullptr;
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<crc32c_job *> pending;
    hipStream_t st = nullptr;
    // Two launch slots: while one launch runs, the next (whatever was pending
    // when it started) is queued behind it on the stream.  Each slot has
    // pinned, mapped descriptors for kSmallMax spans and its event.
    struct Slot {
        uint64_t *addr = nullptr;
        uint32_t *len = nullptr, *cin = nullptr, *out = nullptr;
        void *v_addr = nullptr, *v_len = nullptr, *v_cin = nullptr, *v_out = nullptr;
        hipEvent_t done = nullptr;
        std::vector<crc32c_job *> jobs;  // empty: the slot is free
    } slot[2];
    unsigned long long *dnbad = nullptr;  // (spans are absolute: never out of range)
    std::atomic<uint64_t> launches{0}, spans{0}, jobs{0}, solo{0};

    int init(Device &dev) {
        d = &dev;
        HIP_OK(hipSetDevice(dev.id));
        HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        const uint64_t n = mcrc_dev::kSmallMax;
        for (Slot &l : slot) {
            HIP_OK(hipHostMalloc((void **)&l.addr, n * 8, hipHostMallocDefault));
            HIP_OK(hipHostMalloc((void **)&l.len, n * 4, hipHostMallocDefault));
            HIP_OK(hipHostMalloc((void **)&l.cin, n * 4, hipHostMallocDefault));
            HIP_OK(hipHostMalloc((void **)&l.out, n * 4, hipHostMallocDefault));
            HIP_OK(hipHostGetDevicePointer(&l.v_addr, l.addr, 0));
            HIP_OK(hipHostGetDevicePointer(&l.v_len, l.len, 0));
            HIP_OK(hipHostGetDevicePointer(&l.v_cin, l.cin, 0));
            HIP_OK(hipHostGetDevicePointer(&l.v_out, l.out, 0));
            HIP_OK(hipEventCreateWithFlags(&l.done, hipEventDisableTiming));
        }
        HIP_OK(hipMalloc(&dnbad, sizeof(unsigned long long)));
        HIP_OK(hipMemset(dnbad, 0, sizeof(unsigned long long)));
        // the dispatcher runs until process exit: an atexit hook (registered
        // after the HIP runtime initialised, so it runs before HIP's static
        // destructors) stops it once the queue has drained and joins it
        worker = std::thread([this] { run(); });
        return CRC32C_OK;
    }

    std::thread worker;
    bool stop = false;  // (under mu)

    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv_work.notify_one();
        if (worker.joinable()) worker.join();
    }

    // false once the dispatcher is stopping (process exit): a job queued
    // then might never run, so it is refused instead
    bool submit(crc32c_job *j) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (stop) return false;
            pending.push_back(j);
        }
        cv_work.notify_one();
        return true;
    }

    // Completion wakes exactly the job's own waiter (a futex on j->done): with
    // many IO threads a shared condition variable woke every waiter per launch,
    // and spinning waiters starved the dispatcher of CPU time.
    // (A spinning waiter can see done == 1, return and free the job before
    // the FUTEX_WAKE below runs.  The wake only hashes the address: on
    // reused memory it at most wakes another job's waiter, which re-checks
    // its word and sleeps again; on unmapped memory it fails with EFAULT.
    // Neither writes memory, so the job is not touched after the store.)
    static void complete(crc32c_job *j, int rc) {
        j->rc = rc;
        j->done.store(1, std::memory_order_release);
        syscall(SYS_futex, reinterpret_cast<int *>(&j->done), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
    }

    static int wait(crc32c_job *j) {
        // a launch completes within tens of microseconds: spin briefly first
        const auto t0 = std::chrono::steady_clock::now();
        while (!j->done.load(std::memory_order_acquire) &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(10))
            __builtin_ia32_pause();
        while (!j->done.load(std::memory_order_acquire))
            syscall(SYS_futex, reinterpret_cast<int *>(&j->done), FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
        return j->rc;
    }

    // The jobs of slot l in one k_small launch over absolute span addresses
    // (enqueued, not waited for).
    int launch(Slot &l) {
        uint64_t k = 0;
        for (crc32c_job *j : l.jobs) {
            const crc32c_spans &s = j->s;
            for (uint64_t i = 0; i < s.n; ++i, ++k) {
                l.addr[k] = (uint64_t)(uintptr_t)(j->dbase + span_off(s, i));
                l.len[k] = (uint32_t)span_len(s, i);
                l.cin[k] = s.crc_in ? s.crc_in[i] : 0u;
            }
        }
        mcrc_dev::SpanArgs a{};
        a.base = nullptr;  // spans at absolute addresses
        a.base_bytes = ~0ull;
        a.offsets = (const uint64_t *)l.v_addr;
        a.lens = (const uint32_t *)l.v_len;
        a.crc_in = (const uint32_t *)l.v_cin;
        a.out = (uint32_t *)l.v_out;
        a.nbad = dnbad;
        a.n = k;
        a.xpow = d->xpow;
        a.tab8 = d->tab8;
        a.zero = d->zero;
        a.cfl = 4;
        int rc = launch_small<0>(*d, a, st);
        if (rc) return rc;
        HIP_OK(hipEventRecord(l.done, st));
        launches.fetch_add(1, std::memory_order_relaxed);
        spans.fetch_add(k, std::memory_order_relaxed);
        jobs.fetch_add(l.jobs.size(), std::memory_order_relaxed);
        return CRC32C_OK;
    }

    // Wait for slot l's launch, hand out the CRCs, wake the waiters.
    void finish(Slot &l, int rc) {
        if (!rc && hipEventSynchronize(l.done) != hipSuccess) rc = CRC32C_EHIP;
        uint64_t k = 0;
        for (crc32c_job *j : l.jobs) {
            if (!rc) memcpy(j->s.out, l.out + k, j->s.n * 4);
            k += j->s.n;
            complete(j, rc);
        }
        l.jobs.clear();
    }

    int run_solo(crc32c_job *j) {
        solo.fetch_add(1, std::memory_order_relaxed);
        if (j->flags & CRC32C_DEVICE) {
            if (j->after) {
                const hipError_t e = hipStreamWaitEvent(st, j->after, 0);
                (void)hipEventDestroy(j->after);
                j->after = nullptr;
                if (e != hipSuccess) return CRC32C_EHIP;
            }
            return device_batch(*d, j->s, j->flags & ~(unsigned)CRC32C_ASYNC, st);
        }
        return run_host_batch(*d, j->s);
    }

    void run() {
        (void)hipSetDevice(d->id);
        int cur = 0;              // slot of the launch in flight (if it has jobs)
        int rcs[2] = {0, 0};      // launch status of each slot
        for (;;) {
            Slot &busy = slot[cur], &next = slot[cur ^ 1];
            crc32c_job *solo_job = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu);
                if (busy.jobs.empty()) {
                    cv_work.wait(lk, [&] { return !pending.empty() || stop; });
                    if (pending.empty()) return;  // stop, and nothing in flight
                }
                if (!pending.empty() && !pending.front()->coalesce) {
                    solo_job = pending.front();
                    pending.pop_front();
                } else {
                    uint64_t ns = 0;
                    while (!pending.empty() && pending.front()->coalesce &&
                           ns + pending.front()->s.n <= mcrc_dev::kSmallMax) {
                        ns += pending.front()->s.n;
                        next.jobs.push_back(pending.front());
                        pending.pop_front();
                    }
                }
            }
            if (!next.jobs.empty()) rcs[cur ^ 1] = launch(next);  // queued behind the busy slot
            if (!busy.jobs.empty()) finish(busy, rcs[cur]);
            if (solo_job) {  // (the stream is drained first: solo jobs use it too)
                if (!next.jobs.empty()) finish(next, rcs[cur ^ 1]);
                complete(solo_job, run_solo(solo_job));
            }
            cur ^= 1;
        }
    }
};

// Every device's dispatcher stops (after its pending jobs) at process exit.
void stop_queues() {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    for (auto &d : g_devs)
        if (Queue *q = d->queue.load(std::memory_order_acquire)) q->shutdown();
}

int queue_of(Device &d, Queue **out) {
    static std::mutex mu;
    static bool hooked = false;
    std::lock_guard<std::mutex> lk(mu);
    Queue *q = d.queue.load(std::memory_order_acquire);
    if (!q) {
        q = new Queue();
        const int rc = q->init(d);
        if (rc) return rc;  // (a partly initialised queue is leaked, not reused)
        if (!hooked) hooked = std::atexit(stop_queues) == 0;
        d.queue.store(q, std::memory_order_release);
    }
    *out = q;
    return CRC32C_OK;
}

// A new job for the current device's queue; *coalesce says whether it can
// share a launch (host spans, device-visible buffer, short spans).
int make_job(const crc32c_spans &s, unsigned flags, crc32c_job **out) {
    if (s.n && (!s.base || !s.out)) return CRC32C_EINVAL;
    Device *d = nullptr;
    int rc = current_device(&d);
    if (rc) return rc;
    Queue *q = nullptr;
    if ((rc = queue_of(*d, &q))) return rc;
    crc32c_job *j = new crc32c_job();
    j->s = s;
    j->flags = flags & ~(unsigned)CRC32C_ASYNC;
    j->q = q;
    if (flags & CRC32C_DEVICE) {
        // order the job after the submitter's default stream (its work so far)
        if (hipEventCreateWithFlags(&j->after, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(j->after, nullptr) != hipSuccess) {
            if (j->after) (void)hipEventDestroy(j->after);
            delete j;
            return CRC32C_EHIP;
        }
    } else {
        if (!host_spans_ok(s)) {
            delete j;
            return CRC32C_EINVAL;
        }
        bool short_spans = s.n >= 1 && s.n <= mcrc_dev::kSmallMax;
        for (uint64_t i = 0; short_spans && i < s.n; ++i) short_spans = span_len(s, i) <= kQueueSpanMax;
        if (short_spans && (j->dbase = device_view_range(s.base, s.base_bytes)) != nullptr) j->coalesce = true;
    }
    *out = j;
    return CRC32C_OK;
}

// crc32c_batch_multi's workers: one persistent thread per gfx950 device,
// bound to its HIP ordinal once (hipSetDevice) when first needed and kept for
// the life of the process (detached; idle ones sleep on their condition
// variable), so a call costs one hand-off per device rather than a thread
// creation and a device bind (round 5 spawned a std::thread per device per
// call).  Each worker runs its parts in the order they were posted; several
// callers may use the pool at once.
struct MultiDone {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
    void add() {
        std::lock_guard<std::mutex> lk(mu);
        ++left;
    }
    void finish() {
        std::lock_guard<std::mutex> lk(mu);
        if (--left == 0) cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left == 0; });
    }
};
struct MultiJob {
    crc32c_spans part;
    int *rc;
    MultiDone *done;
};
struct MultiWorker {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<MultiJob> q;
    void post(const MultiJob &j) {
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(j);
        }
        cv.notify_one();
    }
    void run(int ordinal) {
        const bool bound = hipSetDevice(ordinal) == hipSuccess;
        for (;;) {
            MultiJob j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !q.empty(); });
                j = q.front();
                q.pop_front();
            }
            *j.rc = bound ? crc32c_batch(&j.part, 0, nullptr) : CRC32C_EHIP;
            j.done->finish();
        }
    }
};
std::mutex g_multi_mu;
MultiWorker *g_multi[kMaxDevices];

MultiWorker *multi_worker(int index) {
    if (index < 0 || index >= kMaxDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_multi_mu);
    if (!g_multi[index]) {
        const int ordinal = gfx_ordinal(index);
        if (ordinal < 0) return nullptr;
        MultiWorker *w = new MultiWorker();  // (lives for the process)
        std::thread([w, ordinal] { w->run(ordinal); }).detach();
        g_multi[index] = w;
    }
    return g_multi[index];
}

}  // namespace

// ---------------------------------------------------------------------------
// Batch C ABI
// ---------------------------------------------------------------------------
extern "C" {

int crc32c_gpu_count(void) {
    const int n = g_ngfx_pub.load(std::memory_order_acquire);
    if (n >= 0) return n;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    return ensure_devices();
}

void *crc32c_host_alloc(size_t bytes) {
    if (bytes == 0 || crc32c_gpu_count() <= 0) return nullptr;
    void *p = nullptr;
    // portable: usable by every device's copy engine (crc32c_batch_multi)
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) return nullptr;
    return p;
}

void crc32c_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int crc32c_host_register(void *p, size_t bytes) {
    if (!p || !bytes) return CRC32C_EINVAL;
    if (crc32c_gpu_count() <= 0) return CRC32C_ENODEV;
    HIP_OK(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    return CRC32C_OK;
}

int crc32c_host_unregister(void *p) {
    if (!p) return CRC32C_EINVAL;
    if (crc32c_gpu_count() <= 0) return CRC32C_ENODEV;
    HIP_OK(hipHostUnregister(p));
    return CRC32C_OK;
}

uint64_t crc32c_set_small_max(uint64_t n) {
    return g_small_max.exchange(std::min<uint64_t>(n, mcrc_dev::kSmallMax));
}

const char *crc32c_strerror(int err) {
    switch (err) {
        case CRC32C_OK: return "ok";
        case CRC32C_ENODEV: return "no gfx950 device";
        case CRC32C_EHIP: return "HIP runtime error";
        case CRC32C_EINVAL: return "invalid argument";
        case CRC32C_ENOMEM: return "out of device or pinned memory";
        case CRC32C_ERANGE: return "span outside [base, base + base_bytes) (not read)";
        case CRC32C_EWALK: return "device page walk passes disagreed (results not valid)";
        default: return "unknown error";
    }
}

float crc32c_last_kernel_ms(void) { return g_last_kernel_ms; }

int crc32c_batch_submit(const crc32c_spans *s, unsigned flags, crc32c_job_t *job) {
    if (!s || !job) return CRC32C_EINVAL;
    crc32c_job *j = nullptr;
    const int rc = make_job(*s, flags, &j);
    if (rc) return rc;
    if (!j->q->submit(j)) {
        if (j->after) (void)hipEventDestroy(j->after);
        delete j;
        return CRC32C_EHIP;
    }
    *job = j;
    return CRC32C_OK;
}

int crc32c_batch_wait(crc32c_job_t j) {
    if (!j) return CRC32C_EINVAL;
    const int rc = j->q->wait(j);
    delete j;
    return rc;
}

int crc32c_queue_stats(uint64_t *launches, uint64_t *spans, uint64_t *jobs, uint64_t *solo_jobs) {
    Device *d = nullptr;
    const int rc = current_device(&d);
    if (rc) return rc;
    const Queue *q = d->queue.load(std::memory_order_acquire);
    if (launches) *launches = q ? q->launches.load() : 0;
    if (spans) *spans = q ? q->spans.load() : 0;
    if (jobs) *jobs = q ? q->jobs.load() : 0;
    if (solo_jobs) *solo_jobs = q ? q->solo.load() : 0;
    return CRC32C_OK;
}

int crc32c_batch(const crc32c_spans *s, unsigned flags, void *stream) {
    if (!s || (s->n && (!s->base || !s->out))) return CRC32C_EINVAL;
    Device *d = nullptr;
    int rc = current_device(&d);
    if (rc) return rc;
    if (!(flags & CRC32C_DEVICE)) {
        // short spans in page-locked memory share the queue's launches with
        // other threads' batches; anything else is staged on its own
        crc32c_job *j = nullptr;
        if ((rc = make_job(*s, flags, &j))) return rc;
        if (!j->coalesce) {
            delete j;
            return run_host_batch(*d, *s);
        }
        rc = j->q->submit(j) ? j->q->wait(j) : CRC32C_EHIP;
        delete j;
        return rc;
    }
    // Device batches run on the caller's stream; NULL is the default stream, so
    // the kernel is ordered after whatever produced the buffers there.
    return device_batch(*d, *s, flags, (hipStream_t)stream);
}

int crc32c_batch_chains(const crc32c_spans *iovs, const uint64_t *chain_first, uint64_t nchains, uint32_t *out,
                        unsigned flags, void *stream) {
    if (!iovs || !chain_first || (nchains && !out) || iovs->crc_in) return CRC32C_EINVAL;
    if (nchains == 0) return CRC32C_OK;
    Device *d = nullptr;
    int rc = current_device(&d);
    if (rc) return rc;
    const bool dev = flags & CRC32C_DEVICE;
    if (!dev) {  // per-iov CRCs through the staged host path, then the fold on the device
        for (uint64_t c = 0; c < nchains; ++c)
            if (chain_first[c + 1] < chain_first[c] || chain_first[c + 1] > iovs->n) return CRC32C_EINVAL;
        rc = run_host_batch(*d, *iovs);
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> lk(d->mu);
    hipStream_t st = dev ? (hipStream_t)stream : d->stream;
    d->acquire(st);
    struct Release {
        Device *d;
        hipStream_t st;
        ~Release() { d->release(st); }
    } release_on_exit{d, st};
    const uint32_t *crcs = iovs->out, *lens = iovs->lens;
    const uint64_t *first = chain_first;
    uint32_t *dout = out;
    unsigned long long nrange = 0;
    bool nrange_copied = false;
    if (dev) {
        if (!device_range_ok(iovs->base, iovs->base_bytes)) return CRC32C_EINVAL;
        rc = enqueue_device(*d, *iovs, st);
        if (rc) return rc;
        if (!(flags & CRC32C_ASYNC) && (iovs->offsets || iovs->lens)) {  // range-checked on the device
            HIP_OK(hipMemcpyAsync(d->hbad, d->nbad, sizeof nrange, hipMemcpyDeviceToHost, st));
            nrange_copied = true;
        }
    } else {  // stage the fold's inputs (small: 4-8 B per iov / chain)
        const uint64_t n = iovs->n;
        uint8_t *buf = (uint8_t *)d->grow(kScrStage, n * 8 + (nchains + 1) * 8 + nchains * 4 + 64);
        if (!buf) return CRC32C_ENOMEM;
        uint32_t *c_d = (uint32_t *)buf, *l_d = lens ? c_d + n : nullptr;
        uint64_t *f_d = (uint64_t *)(buf + ((n * 8 + 7) & ~7ull));
        uint32_t *o_d = (uint32_t *)(f_d + nchains + 1);
        HIP_OK(hipMemcpyAsync(c_d, iovs->out, n * 4, hipMemcpyHostToDevice, st));
        if (lens) HIP_OK(hipMemcpyAsync(l_d, lens, n * 4, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(f_d, chain_first, (nchains + 1) * 8, hipMemcpyHostToDevice, st));
        crcs = c_d;
        lens = l_d;
        first = f_d;
        dout = o_d;
    }
    const int g = (int)std::min<uint64_t>((nchains + 255) / 256, 4096);
    hipLaunchKernelGGL(mcrc_dev::k_chain, dim3(g), dim3(256), 0, st, crcs, lens, iovs->len, first, nchains, dout,
                       (const uint32_t *)d->xpow);
    HIP_OK(hipGetLastError());
    if (!dev) HIP_OK(hipMemcpyAsync(out, dout, nchains * 4, hipMemcpyDeviceToHost, st));
    if (!dev || !(flags & CRC32C_ASYNC)) HIP_OK(hipStreamSynchronize(st));
    if (nrange_copied) nrange = *d->hbad;
    return nrange ? CRC32C_ERANGE : CRC32C_OK;
}

int crc32c_verify_items(const void *base, uint64_t base_bytes, uint64_t region_bytes, const uint64_t *item_offsets,
                        uint64_t n, uint8_t *ok, uint64_t *nbad, unsigned flags, void *stream) {
    if (!nbad) return CRC32C_EINVAL;
    return item_images<1>(const_cast<void *>(base), base_bytes, region_bytes, item_offsets, n, ok, nbad,
                          flags & ~(unsigned)CRC32C_ASYNC, stream);
}

int crc32c_stamp_items(void *base, uint64_t base_bytes, uint64_t region_bytes, const uint64_t *item_offsets,
                       uint64_t n, uint8_t *ok, uint64_t *nbad, unsigned flags, void *stream) {
    return item_images<2>(base, base_bytes, region_bytes, item_offsets, n, ok, nbad, flags, stream);
}

int crc32c_verify_pages(const void *base, uint64_t base_bytes, uint64_t wbuf_bytes, uint64_t *offsets, uint8_t *ok,
                        uint64_t cap, uint64_t *nitems, uint64_t *nbad, unsigned flags, void *stream) {
    if (!base || !wbuf_bytes || !nitems || !nbad || (cap && (!offsets || !ok))) return CRC32C_EINVAL;
    Device *d = nullptr;
    int rc = current_device(&d);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const bool dev = flags & CRC32C_DEVICE;
    if (dev && !device_range_ok(base, base_bytes)) return CRC32C_EINVAL;
    std::lock_guard<std::mutex> lk(d->mu);
    const uint64_t nw = (base_bytes + wbuf_bytes - 1) / wbuf_bytes;
    d->acquire(st);
    struct Release {
        Device *d;
        hipStream_t st;
        ~Release() { d->release(st); }
    } release_on_exit{d, st};
    if (nw == 0 || nw >= 0x7fffffffull) {
        *nitems = *nbad = 0;
        return nw ? CRC32C_EINVAL : CRC32C_OK;
    }
    const uint8_t *dbase = (const uint8_t *)base;
    if (!dev) {
        uint8_t *b = (uint8_t *)d->grow(kScrStage, base_bytes);
        if (!b) return CRC32C_ENOMEM;
        HIP_OK(hipMemcpyAsync(b, base, base_bytes, hipMemcpyHostToDevice, st));
        dbase = b;
    }
    // counts of nw wbufs and a zero: the exclusive scan's last entry is the total
    uint32_t *cnt = (uint32_t *)d->grow(kScrWalkCnt, (nw + 1) * 4);
    uint32_t *prefix = (uint32_t *)d->grow(kScrWalkPrefix, (nw + 2) * 4);
    if (!cnt || !prefix) return CRC32C_ENOMEM;
    mcrc_dev::SpanArgs a{};
    a.base = dbase;
    a.base_bytes = base_bytes;
    a.nbad = d->nbad;
    a.xpow = d->xpow;
    a.tab8 = d->tab8;
    a.zero = d->zero;
    a.region = wbuf_bytes;
    a.cfl = (flags & CRC32C_CFLAGS64) ? 8u : 4u;
    // one walking wave per wbuf, kWalkWaves per workgroup
    const int gw = (int)std::min<uint64_t>((nw + mcrc_dev::kWalkWaves - 1) / mcrc_dev::kWalkWaves, 65535);
    const dim3 bw(64 * mcrc_dev::kWalkWaves);
    mcrc_dev::WalkOut wo{};
    wo.cnt = cnt;
    // the count pass keeps each wbuf's first offsets (one per 2 KiB of wbuf:
    // every 4 MiB wbuf of items of at least 2 KiB; 8 B per 2 KiB, 0.4 % of the
    // walked bytes), so a K5 verify's emit pass copies them instead of walking
    // again.  Wbufs under 16 KiB keep none (walked twice), and so does a walk
    // whose slot buffer cannot be allocated.
    wo.kslot = (uint32_t)std::min<uint64_t>(wbuf_bytes / 2048, 8192);
    if (wo.kslot < 8) wo.kslot = 0;
    wo.slots = wo.kslot ? (uint64_t *)d->grow(kScrWalkSlots, (size_t)nw * wo.kslot * 8) : nullptr;
    if (!wo.slots) wo.kslot = 0;
    HIP_OK(hipMemsetAsync(cnt + nw, 0, 4, st));
    hipLaunchKernelGGL(mcrc_dev::k_walk<false>, dim3(gw), bw, 0, st, a, nw, wo);
    hipLaunchKernelGGL(mcrc_dev::k_scan32, dim3(1), dim3(1024), 0, st, (const uint32_t *)cnt, nw + 1, prefix);
    uint32_t total = 0;
    HIP_OK(hipMemcpyAsync(&total, prefix + nw, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    *nitems = total;
    if (total == 0 || cap == 0) {  // cap == 0: count-only query (no verify)
        *nbad = 0;
        return CRC32C_OK;
    }
    const bool direct = dev && cap >= total;  // caller's device arrays take the results
    uint64_t *doffs = direct ? offsets : (uint64_t *)d->grow(kScrWalkOffs, (size_t)total * 8);
    uint8_t *dok = direct ? ok : (uint8_t *)d->grow(kScrWalkOk, total);
    if (!doffs || !dok) return CRC32C_ENOMEM;
    a.offsets = doffs;
    a.ok = dok;
    a.n = total;
    // The emit pass writes the offsets: copied from the count pass's slots,
    // or for a wbuf of more items than those (or with no slots kept) by
    // walking it again.  A planned verify then reads the headers in k_count,
    // in parallel (round 6; the emit pass used to walk again and write
    // k_count's entries itself, one header per round trip on mixed pages);
    // only when no slots are kept does the second walk write the entries
    // too (the headers are then read once more, not twice).
    Path path;
    path.small = takes_small<1>(a);
    const bool k5 = !path.small && items_fused(a);  // (then the walk writes offsets only)
    path.counted = !path.small && !k5 && wo.kslot == 0;
    if (path.counted) {
        rc = ensure_plan(*d, total, plan_cap(a));
        if (rc) return rc;
        a.span_acc = d->span_acc;
    }
    wo.prefix = prefix;
    wo.offs = doffs;
    wo.err = d->nbad + 1;
    wo.nunit = path.counted ? d->nunit : nullptr;
    wo.irec = path.counted ? d->irec : nullptr;
    wo.fast = path.counted ? d->fast : nullptr;
    HIP_OK(hipMemsetAsync(d->nbad, 0, 2 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(mcrc_dev::k_walk<true>, dim3(gw), bw, 0, st, a, nw, wo);
    rc = k5 ? launch_items<1>(*d, a, st) : launch_units<1>(*d, a, st, path);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(d->hbad, d->nbad, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    const uint64_t k = std::min<uint64_t>(cap, total);
    if (!direct && k) {
        const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        HIP_OK(hipMemcpyAsync(offsets, doffs, k * 8, kind, st));
        HIP_OK(hipMemcpyAsync(ok, dok, k, kind, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    *nbad = d->hbad[0];
    return d->hbad[1] ? CRC32C_EWALK : CRC32C_OK;
}

int crc32c_shard_cuts(const uint32_t *lens, uint32_t len, uint64_t n, int parts, uint64_t *cuts) {
    if (parts < 1 || !cuts) return CRC32C_EINVAL;
    unsigned __int128 total = 0;
    for (uint64_t i = 0; i < n; ++i) total += lens ? lens[i] : len;
    cuts[0] = 0;
    uint64_t i = 0;
    unsigned __int128 acc = 0;
    for (int g = 1; g < parts; ++g) {
        const unsigned __int128 target = total * (unsigned)g / (unsigned)parts;
        for (; i < n && acc < target; ++i) acc += lens ? lens[i] : len;
        cuts[g] = i;
    }
    cuts[parts] = n;
    return CRC32C_OK;
}

int crc32c_batch_multi(const crc32c_spans *s, int ngpus) {
    if (!s) return CRC32C_EINVAL;
    const int avail = crc32c_gpu_count();
    if (avail <= 0) return CRC32C_ENODEV;
    if (ngpus <= 0 || ngpus > avail) ngpus = avail;
    std::vector<uint64_t> cut(ngpus + 1);
    int rc = crc32c_shard_cuts(s->lens, s->len, s->n, ngpus, cut.data());
    if (rc) return rc;
    std::vector<int> rcs(ngpus, CRC32C_OK);
    MultiDone done;
    for (int g = 0; g < ngpus; ++g) {
        const uint64_t a0 = cut[g], a1 = cut[g + 1];
        if (a1 == a0) continue;
        crc32c_spans sub = *s;
        sub.n = a1 - a0;
        if (s->offsets) sub.offsets = s->offsets + a0;
        else {
            sub.base = (const uint8_t *)s->base + a0 * s->stride;
            sub.base_bytes = s->base_bytes - a0 * s->stride;
        }
        if (s->lens) sub.lens = s->lens + a0;
        if (s->crc_in) sub.crc_in = s->crc_in + a0;
        sub.out = s->out + a0;
        MultiWorker *w = multi_worker(g);
        if (!w) {
            rcs[g] = CRC32C_ENODEV;
            continue;
        }
        done.add();
        w->post(MultiJob{sub, &rcs[g], &done});
    }
    done.wait();
    for (int r : rcs)
        if (r) return r;
    return CRC32C_OK;
}

}  // extern "C"
