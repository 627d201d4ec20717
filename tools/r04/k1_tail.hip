// k1_tail.hip -- dev experiment (not part of the library): how much of a K1
// launch is the start (table copy) and the end (waves finishing at different
// times under the static grid-stride split)?
//
//   1. K1 (the product kernel, included) timed with events at 1, 2, 4 Mi
//      items: T(n) = a + b n gives the fixed cost a per launch.
//   2. A copy of K1 that stamps, per wave, s_memrealtime (100 MHz) at entry,
//      after the table copy and at exit, plus its XCC / SE / CU: the spread of
//      the exit stamps is the tail a dynamic split could recover.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/k1_tail.hip -o /tmp/k1_tail
//   /tmp/k1_tail [REPS]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "crc32c_gf2.h"
#include "crc32c_kernels.hip"

using namespace mcrc_dev;

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

struct Stamp {
    uint64_t t0, t1, t2, id;
};

// k_fixed<false> with per-wave stamps (same loop, same loads).
__global__ __launch_bounds__(1024) void k_fixed_ts(const uint8_t *__restrict__ base, uint64_t stride, uint64_t nitems,
                                                   const uint4 *__restrict__ img, uint32_t *__restrict__ out,
                                                   Stamp *st) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    using Regs = ItemRegs<32, kK1CH, kK1Rows>;
    constexpr uint32_t IPW = 2;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t li = lane & 31u;
    const uint32_t g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t gstep = gridDim.x * waves;
    const uint64_t ngroups = (nitems + IPW - 1) / IPW;
    const uint32_t wid = blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6);
    uint64_t grp = __builtin_amdgcn_readfirstlane(wid);
    if (grp < ngroups) {
        auto item_of = [&](uint64_t gi) { return gi * IPW + g; };
        Regs ra, rb;
        auto ld = [&](Regs &r, uint64_t gi) {
            const uint64_t gu = gi < ngroups ? gi : gi - gstep < ngroups ? gi - gstep : ngroups - 1;
            const uint64_t first = gu * IPW;
            const uint8_t *wb = base + first * stride;
            const uint32_t gl = first + g < nitems ? g : (uint32_t)(nitems - 1 - first);
            r.cin = 0u;
            r.load_at(wb, gl * (uint32_t)stride + li * kK1CH);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto part0 = [&](Regs &m) {
            if (li == 0) m.d[0][0].x ^= ~m.cin;
            return reduce_level<0>(lane_partial_x3s<kK1CH>(m, c), (lane & 1u) == 0u);
        };
        const uint64_t nsteps = (ngroups - grp + gstep - 1) / gstep;
        ld(ra, grp);
        uint64_t k = 0;
        for (; k + 4 <= nsteps; k += 4) {
            ld(rb, grp + gstep);
            const uint32_t va = part0(ra);
            ld(ra, grp + 2 * gstep);
            const uint32_t vb = part0(rb);
            const uint32_t vab = group_pair_level1(va, vb, lane);
            ld(rb, grp + 3 * gstep);
            const uint32_t vc = part0(ra);
            ld(ra, grp + 4 * gstep);
            const uint32_t vd = part0(rb);
            const uint32_t raw = group_reduce32_quad(vab, group_pair_level1(vc, vd, lane), lane);
            const uint64_t item = item_of(grp + (li & 3u) * gstep);
            if (li < 4 && item < nitems) out[item] = ~raw;
            grp += 4 * gstep;
        }
        for (; k + 2 <= nsteps; k += 2) {
            ld(rb, grp + gstep);
            const uint32_t va = part0(ra);
            ld(ra, grp + 2 * gstep);
            const uint32_t vb = part0(rb);
            const uint32_t raw = group_reduce32_pair(va, vb, lane);
            const uint64_t item = item_of(li == 0 ? grp : grp + gstep);
            if (li < 2 && item < nitems) out[item] = ~raw;
            grp += 2 * gstep;
        }
        if (nsteps & 1) {
            const uint32_t raw = group_reduce32_dpp(lane_partial_x3s<kK1CH>(ra, c), lane);
            const uint64_t item = item_of(grp);
            if (li == 0 && item < nitems) out[item] = ~raw;
        }
    }
    // out[] stores drained before the exit stamp
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    if (lane == 0) st[wid] = Stamp{t0, t1, t2, hw | ((uint64_t)xcc << 32)};
}

// Dynamic split.  Chunks of kCG groups (4 steps of a wave, 8 items, 32 KiB)
// in P <= 8 pools of contiguous chunks; pool p is pulled by the workgroups
// labelled b % P == p (which share an XCD in practice).  A wave's first chunk
// is static (its rank in the pool); the next one is claimed with one
// returning atomic on the pool's head at the top of the current chunk and used
// for the prefetch at its last step; an exhausted pool sends the wave to the
// other pools (read the head, claim only if not exhausted).  The last
// workgroup to finish zeroes the heads for the next launch.
// every counter on its own 256-B line (atomics on one line serialise like
// atomics on one word)
struct Line {
    uint32_t v;
    uint32_t pad[63];
};
struct DynCtl {
    Line head[8];
    Line lab_done[8];
    Line all_done;
};

__device__ __forceinline__ uint32_t ld_agent(uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t *p) {
    return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool TS, uint32_t kCG>
__global__ __launch_bounds__(1024) void k_fixed_dyn(const uint8_t *__restrict__ base, uint64_t stride, uint64_t nitems,
                                                    const uint4 *__restrict__ img, uint32_t *__restrict__ out,
                                                    Stamp *st, DynCtl *ctl) {
    const uint64_t t0 = TS ? __builtin_amdgcn_s_memrealtime() : 0;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
    const uint64_t t1 = TS ? __builtin_amdgcn_s_memrealtime() : 0;
    using Regs = ItemRegs<32, kK1CH, kK1Rows>;
    constexpr uint32_t IPW = 2;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t li = lane & 31u;
    const uint32_t g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    constexpr uint32_t waves = 16;
    const uint64_t ngroups = (nitems + IPW - 1) / IPW;
    const uint32_t nch = (uint32_t)((ngroups + kCG - 1) / kCG);
    const uint32_t P = gridDim.x < 8 ? gridDim.x : 8;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * waves + (threadIdx.x >> 6));
    const uint32_t b = blockIdx.x;
    auto pool_lo = [&](uint32_t p) { return (uint32_t)((uint64_t)nch * p / P); };
    // workgroups with label p: ceil((grid - p) / P); waves pulling pool p statically
    auto pool_w = [&](uint32_t p) { return (gridDim.x - p + P - 1) / P * waves; };
    uint32_t pool = b % P;
    uint32_t cur = pool_lo(pool) + (b / P) * waves + (threadIdx.x >> 6);
    uint32_t tried = 0;  // pools seen exhausted (bit mask)
    // claim: a chunk of pool q from its head, or ~0u if q is exhausted
    auto claim_in = [&](uint32_t q) -> uint32_t {
        const uint32_t lo = pool_lo(q), sz = pool_lo(q + 1) - lo, w0 = pool_w(q);
        uint32_t h = 0;
        if (lane == 0) h = ld_agent(&ctl->head[q].v);
        h = __builtin_amdgcn_readfirstlane(h);
        if (w0 + h >= sz) return ~0u;
        if (lane == 0) h = add_agent(&ctl->head[q].v);
        h = __builtin_amdgcn_readfirstlane(h);
        return w0 + h < sz ? lo + w0 + h : ~0u;
    };
    // after the own claim failed: the other pools in turn
    auto steal = [&]() -> uint32_t {
        tried |= 1u << pool;
        for (uint32_t k = 1; k < P; ++k) {
            const uint32_t q = (pool + k) % P;
            if (tried & (1u << q)) continue;
            const uint32_t x = claim_in(q);
            if (x != ~0u) {
                pool = q;
                return x;
            }
            tried |= 1u << q;
        }
        return ~0u;
    };
    if (cur >= pool_lo(pool + 1)) cur = steal();
    if (cur != ~0u) {
        Regs ra, rb;
        auto ld = [&](Regs &r, uint64_t gi) {
            const uint64_t gu = gi < ngroups ? gi : ngroups - 1;
            const uint64_t first = gu * IPW;
            const uint8_t *wb = base + first * stride;
            const uint32_t gl = first + g < nitems ? g : (uint32_t)(nitems - 1 - first);
            r.cin = 0u;
            r.load_at(wb, gl * (uint32_t)stride + li * kK1CH);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto part0 = [&](Regs &m) {
            if (li == 0) m.d[0][0].x ^= ~m.cin;
            return reduce_level<0>(lane_partial_x3s<kK1CH>(m, c), (lane & 1u) == 0u);
        };
        ld(ra, (uint64_t)cur * kCG);
        for (;;) {
            const uint64_t grp0 = (uint64_t)cur * kCG;
            uint32_t h = 0, nxt = ~0u;
#pragma unroll
            for (uint32_t q = 0; q < kCG / 4; ++q) {
                const uint64_t grp = grp0 + 4 * q;
                ld(rb, grp + 1);
                if (q == 0 && lane == 0) h = add_agent(&ctl->head[pool].v);
                const uint32_t va = part0(ra);
                ld(ra, grp + 2);
                const uint32_t vb = part0(rb);
                const uint32_t vab = group_pair_level1(va, vb, lane);
                ld(rb, grp + 3);
                const uint32_t vc = part0(ra);
                if (q + 1 == kCG / 4) {
                    h = __builtin_amdgcn_readfirstlane(h);
                    const uint32_t lo = pool_lo(pool), sz = pool_lo(pool + 1) - lo, w0 = pool_w(pool);
                    nxt = w0 + h < sz ? lo + w0 + h : steal();
                    ld(ra, nxt != ~0u ? (uint64_t)nxt * kCG : grp + 3);
                } else {
                    ld(ra, grp + 4);
                }
                const uint32_t vd = part0(rb);
                const uint32_t raw = group_reduce32_quad(vab, group_pair_level1(vc, vd, lane), lane);
                const uint64_t item = (grp + (li & 3u)) * IPW + g;
                if (li < 4 && item < nitems) out[item] = ~raw;
            }
            if (nxt == ~0u) break;
            cur = nxt;
        }
    }
    if (TS) {
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        if (lane == 0) st[wid] = Stamp{t0, t1, t2, hw | ((uint64_t)xcc << 32)};
    }
    // the last workgroup zeroes the heads (every claim of this launch is done)
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t lab = b % P, nlab = (gridDim.x - lab + P - 1) / P;
        if (add_agent(&ctl->lab_done[lab].v) == nlab - 1 && add_agent(&ctl->all_done.v) == P - 1) {
            for (uint32_t q = 0; q < 8; ++q) {
                __hip_atomic_store(&ctl->head[q].v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctl->lab_done[q].v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __hip_atomic_store(&ctl->all_done.v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void k_fill(uint32_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull;
        z = (z ^ (z >> 31)) * 0xbf58476d1ce4e5b9ull;
        p[i] = (uint32_t)(z ^ (z >> 29));
    }
}

static double pct(std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t maxn = 4ull << 20, stride = 4096;
    uint8_t *base;
    uint32_t *out, *out2;
    uint4 *img;
    Stamp *st;
    DynCtl *ctl;
    CHECK(hipMalloc(&base, maxn * stride));
    CHECK(hipMalloc(&out, maxn * 4));
    CHECK(hipMalloc(&out2, maxn * 4));
    CHECK(hipMalloc(&st, sizeof(Stamp) * cus * 16));
    CHECK(hipMalloc(&ctl, sizeof(DynCtl)));
    CHECK(hipMemset(ctl, 0, sizeof(DynCtl)));
    CHECK(hipMalloc(&img, kLdsImageK1Bytes));
    std::vector<uint32_t> h(kLdsImageK1Bytes / 4);
    mcrc::build_lds_image_k1(h.data(), kK1CH);
    CHECK(hipMemcpy(img, h.data(), kLdsImageK1Bytes, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)base, maxn * stride / 4);
    for (const void *k : {(const void *)k_fixed<false>, (const void *)k_fixed_ts, (const void *)k_fixed_dyn<false, 4>,
                          (const void *)k_fixed_dyn<true, 4>, (const void *)k_fixed_dyn<false, 8>,
                          (const void *)k_fixed_dyn<false, 16>, (const void *)k_fixed_dyn<true, 16>})
        CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageK1Bytes));
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // 0 k_fixed, 1 stamped copy, 2 dynamic, 3 dynamic stamped
    auto run = [&](uint64_t n, int v, uint32_t *o, int grid) {
        if (v == 0)
            hipLaunchKernelGGL(k_fixed<false>, dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n, img,
                               (const uint32_t *)nullptr, o);
        else if (v == 1)
            hipLaunchKernelGGL(k_fixed_ts, dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n, img, o, st);
        else if (v == 2)
            hipLaunchKernelGGL((k_fixed_dyn<false, 4>), dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n,
                               img, o, st, ctl);
        else if (v == 3)
            hipLaunchKernelGGL((k_fixed_dyn<true, 4>), dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n,
                               img, o, st, ctl);
        else if (v == 4)
            hipLaunchKernelGGL((k_fixed_dyn<false, 8>), dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n,
                               img, o, st, ctl);
        else if (v == 5)
            hipLaunchKernelGGL((k_fixed_dyn<false, 16>), dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n,
                               img, o, st, ctl);
        else
            hipLaunchKernelGGL((k_fixed_dyn<true, 16>), dim3(grid), dim3(1024), kLdsImageK1Bytes, 0, base, stride, n,
                               img, o, st, ctl);
    };
    if (argc > 2 && !strcmp(argv[2], "block")) {  // K1 with fewer waves per CU (one workgroup per CU)
        for (int i = 0; i < 300; ++i) run(1ull << 20, 0, out, cus);
        for (int round = 0; round < 3; ++round)
            for (int bs : {1024, 896, 768, 640, 512}) {
                std::vector<double> ms;
                for (int r = 0; r < reps; ++r) {
                    CHECK(hipEventRecord(e0));
                    hipLaunchKernelGGL(k_fixed<false>, dim3(cus), dim3(bs), kLdsImageK1Bytes, 0, base, stride,
                                       1ull << 20, img, (const uint32_t *)nullptr, out2);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float x;
                    CHECK(hipEventElapsedTime(&x, e0, e1));
                    ms.push_back(x);
                }
                printf("round %d block %4d: median %.4f ms min %.4f max %.4f\n", round, bs, pct(ms, .5), pct(ms, 0),
                       pct(ms, 1));
                fflush(stdout);
            }
        return 0;
    }
    // exactness of the dynamic split (and of its head reset across launches):
    // sizes around the chunk and pool edges, small grids
    {
        long bad = 0;
        const uint64_t ns[] = {1, 2, 3, 7, 8, 9, 63, 64, 65, 1000, 8191, 8192, 8193, 65537, 1048576, 1048575, 4194304};
        for (uint64_t n : ns) {
            for (int grid : {1, 3, 8, 9, cus}) {
                const int gr = std::min<uint64_t>(grid, (n + 31) / 32) > 0 ? std::min<uint64_t>(grid, (n + 31) / 32) : 1;
                CHECK(hipMemset(out, 0, n * 4));
                run(n, 0, out, gr);
                for (int v : {2, 4, 5}) {
                    CHECK(hipMemset(out2, 0xff, n * 4));
                    run(n, v, out2, gr);
                    run(n, v, out2, gr);
                    CHECK(hipDeviceSynchronize());
                    std::vector<uint32_t> a(n), b2(n);
                    CHECK(hipMemcpy(a.data(), out, n * 4, hipMemcpyDeviceToHost));
                    CHECK(hipMemcpy(b2.data(), out2, n * 4, hipMemcpyDeviceToHost));
                    long d = 0;
                    for (uint64_t i = 0; i < n; ++i) d += a[i] != b2[i];
                    DynCtl hc;
                    CHECK(hipMemcpy(&hc, ctl, sizeof hc, hipMemcpyDeviceToHost));
                    uint32_t left = hc.all_done.v;
                    for (int q = 0; q < 8; ++q) left |= hc.head[q].v | hc.lab_done[q].v;
                    if (d || left)
                        printf("MISMATCH v %d n %llu grid %d: %ld CRCs differ, ctl left %u\n", v, (unsigned long long)n, gr,
                               d, left);
                    bad += d + (left != 0);
                }
            }
        }
        printf("dynamic split exactness: %s\n", bad ? "FAILED" : "all equal to k_fixed, heads reset");
        if (bad) return 1;
    }
    // settle the clock
    for (int i = 0; i < 300; ++i) run(1ull << 20, 0, out, cus);
    CHECK(hipDeviceSynchronize());
    for (int round = 0; round < 3; ++round) {
        for (uint64_t n : {1ull << 20, 4ull << 20}) {
            for (int v : {0, 2, 4, 5}) {
                std::vector<double> ms;
                for (int r = 0; r < reps; ++r) {
                    CHECK(hipEventRecord(e0));
                    run(n, v, out, cus);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float x;
                    CHECK(hipEventElapsedTime(&x, e0, e1));
                    ms.push_back(x);
                }
                static const char *nm[] = {"k_fixed", "stamped", "dyn4", "dyn4+st", "dyn8", "dyn16", "dyn16+st"};
                printf("round %d n %7llu %-10s: median %.4f ms  min %.4f  max %.4f  (%.1f %% of 8 TB/s at median)\n",
                       round, (unsigned long long)n, nm[v], pct(ms, 0.5), pct(ms, 0), pct(ms, 1),
                       100.0 * n * stride / (pct(ms, 0.5) * 1e-3) / 8e12);
            }
        }
    }
    // per-wave stamps of one stamped launch, static and dynamic
    for (int v : {1, 3, 6})
        for (uint64_t n : {1ull << 20}) {
            run(n, v, out, cus);
            CHECK(hipDeviceSynchronize());
            std::vector<Stamp> s(cus * 16);
            CHECK(hipMemcpy(s.data(), st, sizeof(Stamp) * s.size(), hipMemcpyDeviceToHost));
            uint64_t tmin = ~0ull, tmax = 0;
            for (auto &x : s) tmin = std::min(tmin, x.t0), tmax = std::max(tmax, x.t2);
            std::vector<double> start, tab, end;
            std::vector<double> xend[16];
            for (auto &x : s) {
                start.push_back((x.t0 - tmin) * 0.01);
                tab.push_back((x.t1 - x.t0) * 0.01);
                end.push_back((x.t2 - tmin) * 0.01);
                xend[(x.id >> 32) & 15].push_back((x.t2 - tmin) * 0.01);
            }
            printf("\n%s n %llu: span %.1f us; wave start p0/p50/p100 %.1f/%.1f/%.1f us; table copy p50/p100 %.1f/%.1f us\n",
                   v == 1 ? "static" : v == 3 ? "dyn4" : "dyn16", (unsigned long long)n, (tmax - tmin) * 0.01, pct(start, 0),
                   pct(start, .5), pct(start, 1), pct(tab, .5), pct(tab, 1));
            printf("wave end p0 %.1f p1 %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f p100 %.1f us\n", pct(end, 0),
                   pct(end, .01), pct(end, .1), pct(end, .5), pct(end, .9), pct(end, .99), pct(end, 1));
            for (int x = 0; x < 16; ++x)
                if (!xend[x].empty())
                    printf("  xcc %d: %zu waves, end p0 %.1f p50 %.1f p100 %.1f us\n", x, xend[x].size(),
                           pct(xend[x], 0), pct(xend[x], .5), pct(xend[x], 1));
            std::vector<double> wg(cus, 0);
            for (int b = 0; b < cus; ++b) {
                double m = 0;
                for (int w = 0; w < 16; ++w) m = std::max(m, end[b * 16 + w]);
                wg[b] = m;
            }
            printf("workgroup end (last wave) p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f us\n", pct(wg, 0),
                   pct(wg, .1), pct(wg, .5), pct(wg, .9), pct(wg, 1));
        }
    return 0;
}
