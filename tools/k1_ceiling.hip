// k1_ceiling.hip -- dev experiment (not part of the library): K1's read
// ceiling on the box it runs on, in one session (round-5 review item 4).
//
// Over the headline batch (1 Mi x 4096 B, device-resident), each timed with
// events (median of REPS launches after a 300 ms clock settle):
//   k_fixed   the product kernel (included from crc32c_kernels.hip; since
//             round 5 the coalesced non-temporal K1, k1c<true> below)
//   k1nt      round 4's K1 (32-B lane rows) with non-temporal loads
//   k1c<NT>   the coalesced K1 (16-B lane pieces at 512-B spacing)
//   k1load    K1's grid, wave ranges and scrambled range order, K1's loads
//             (lane i: bytes [32i, 32i + 32) of each 1 KiB row, two dwordx4,
//             double-buffered, sched_barrier-fenced) -- the CRC chains
//             replaced by an XOR of the loaded dwords
//   coalesced the same ranges, each dwordx4 wave-instruction one contiguous
//             1 KiB (lane i: bytes [16i, 16i + 16)), double-buffered
//   glds<W,S,B,NT>  the same ranges through LDS-DMA (global_load_lds_dwordx4:
//             1 KiB per wave-instruction into a wave-private ring of B slots of
//             S bytes; counted vmcnt waits, then ds_read_b128 + XOR), W waves
//             per CU, default or non-temporal policy
// Every mode writes each item's XOR of its 1024 dwords; the load-only modes
// must agree item for item (they read the same bytes).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/k1_ceiling.hip -o tools/k1_ceiling
//   tools/k1_ceiling [REPS]     (REPS 1: no settle, one launch of each -- for rocprofv3 --pmc)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
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

constexpr uint64_t kItems = 1ull << 20, kItemBytes = 4096;

// Round 4's K1 pieces, removed from the product in round 5 and kept here for
// k1load / k1nt: a lane's 32 contiguous bytes of each 1 KiB row, four row
// chains, the tree on 32-B granules (the row image build_lds_image_k1 at
// chunk 32, level 4 at tables 16..19).
constexpr uint32_t kK1Rows = 4, kK1CH = 32;
template <int LPI, int CH, int R>
struct ItemRegs {
    static constexpr int Q = CH / 16;
    uint4 d[R][Q];
    uint32_t cin;
};
template <int CH>
__device__ __forceinline__ uint32_t lane_partial_x3s(const ItemRegs<32, CH, 4> &it, const LaneCtx &c) {
    constexpr int N = 4 * (CH / 16);
    constexpr uint32_t kShift[3] = {kAuxShift0, kAuxShift1, kAuxShift2};
    uint32_t x[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = it.d[r][0].x;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            x[r] = i + 1 < N ? step4_next(x[r], dw4(it.d[r][(i + 1) >> 2], (i + 1) & 3), c)
                             : (r < 3 ? step4_last_shifted(x[r], kShift[r]) : step4_next(x[r], 0u, c));
    return xor3(x[0], x[1], x[2]) ^ x[3];
}
__device__ __forceinline__ uint32_t group_reduce32_quad(uint32_t ab, uint32_t cd, uint32_t lane) {
    const uint32_t cs = __builtin_amdgcn_update_dpp(0u, cd, 0x112, 0xf, 0xf, false);  // row_shr:2
    uint32_t v = (lane & 2u) ? cs : ab;
    v = reduce_level<2>(v, (lane & 7u) < 4u);
    v = reduce_level<3>(v, (lane & 15u) < 4u);
    return reduce_level<4>(v, (lane & 31u) < 4u);
}
__device__ __forceinline__ uint32_t group_reduce32_pair(uint32_t a, uint32_t b, uint32_t lane) {
    const uint32_t bs = __builtin_amdgcn_update_dpp(0u, b, 0x111, 0xf, 0xf, false);  // row_shr:1
    uint32_t v = (lane & 1u) ? bs : a;
    v = reduce_level<1>(v, (lane & 3u) < 2u);
    v = reduce_level<2>(v, (lane & 7u) < 2u);
    v = reduce_level<3>(v, (lane & 15u) < 2u);
    return reduce_level<4>(v, (lane & 31u) < 2u);
}
__device__ __forceinline__ uint32_t group_reduce32_dpp(uint32_t v, uint32_t lane) {
    v = reduce_level<0>(v, (lane & 1u) == 0u);
    v = reduce_level<1>(v, (lane & 3u) == 0u);
    v = reduce_level<2>(v, (lane & 7u) == 0u);
    v = reduce_level<3>(v, (lane & 15u) == 0u);
    return reduce_level<4>(v, (lane & 31u) == 0u);
}

// K1's wave -> contiguous range of item pairs (crc32c_kernels.hip k_fixed)
struct Range {
    uint64_t g0, g1;
};
__device__ __forceinline__ Range k1_range(uint64_t ngroups) {
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t gstep = gridDim.x * waves;
    uint64_t grp = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6));
    if (gstep % 65521u) grp = (grp * 65521u) % gstep;
    const uint64_t cg = (ngroups + gstep - 1) / gstep;
    return Range{grp * cg, min((grp + 1) * cg, ngroups)};
}

__device__ __forceinline__ uint32_t xor4(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }
// 16-B register load, default or non-temporal policy
template <bool NT>
__device__ __forceinline__ uint4 ldp(const uint8_t *p) {
    const u32x4 v = NT ? __builtin_nontemporal_load((const u32x4 *)p) : *(const u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t wave_xor32(uint32_t v) {  // over each 32-lane half
    v ^= __shfl_xor(v, 1);
    v ^= __shfl_xor(v, 2);
    v ^= __shfl_xor(v, 4);
    v ^= __shfl_xor(v, 8);
    v ^= __shfl_xor(v, 16);
    return v;
}

// K1's loads, XOR instead of the chains.
template <bool NT>
__global__ __launch_bounds__(1024) void k1load(const uint8_t *__restrict__ base, uint32_t *__restrict__ out) {
    using Regs = ItemRegs<32, kK1CH, kK1Rows>;
    const uint32_t lane = threadIdx.x & 63u, li = lane & 31u, g = lane >> 5;
    const uint64_t ngroups = kItems / 2;
    const Range rg = k1_range(ngroups);
    if (rg.g0 >= ngroups) return;
    Regs ra, rb;
    auto ld = [&](Regs &r, uint64_t gi) {
        const uint64_t gu = gi < rg.g1 ? gi : rg.g1 - 1;
        const uint8_t *wb = base + gu * 2 * kItemBytes + g * (uint32_t)kItemBytes + li * kK1CH;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int q = 0; q < 2; ++q) r.d[i][q] = ldp<NT>(wb + i * 1024 + 16 * q);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto fold = [&](const Regs &r) {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int q = 0; q < 2; ++q) x ^= xor4(r.d[i][q]);
        return wave_xor32(x);
    };
    uint64_t grp = rg.g0;
    ld(ra, grp);
    for (; grp + 2 <= rg.g1; grp += 2) {
        ld(rb, grp + 1);
        const uint32_t a = fold(ra);
        if (li == 0) out[grp * 2 + g] = a;
        ld(ra, grp + 2);
        const uint32_t b = fold(rb);
        if (li == 0) out[(grp + 1) * 2 + g] = b;
    }
    if (grp < rg.g1) {
        const uint32_t a = fold(ra);
        if (li == 0) out[grp * 2 + g] = a;
    }
}

// Each wave-instruction reads one contiguous KiB; a step is one item pair.
struct Pair {
    uint4 v[8];
};
template <bool NT>
__global__ __launch_bounds__(1024) void coalesced(const uint8_t *__restrict__ base, uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t ngroups = kItems / 2;
    const Range rg = k1_range(ngroups);
    if (rg.g0 >= ngroups) return;
    Pair ra, rb;
    auto ld = [&](Pair &r, uint64_t gi) {
        const uint64_t gu = gi < rg.g1 ? gi : rg.g1 - 1;
        const uint8_t *wb = base + gu * 2 * kItemBytes;
#pragma unroll
        for (int j = 0; j < 8; ++j) r.v[j] = ldp<NT>(wb + j * 1024 + lane * 16);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto fold = [&](const Pair &r, uint32_t &a, uint32_t &b) {
        uint32_t x = 0, y = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) x ^= xor4(r.v[j]);
#pragma unroll
        for (int j = 4; j < 8; ++j) y ^= xor4(r.v[j]);
        x = wave_xor32(x);
        y = wave_xor32(y);
        a = x ^ __shfl_xor(x, 32);
        b = y ^ __shfl_xor(y, 32);
    };
    uint64_t grp = rg.g0;
    ld(ra, grp);
    uint32_t a, b;
    for (; grp + 2 <= rg.g1; grp += 2) {
        ld(rb, grp + 1);
        fold(ra, a, b);
        if (lane == 0) out[grp * 2] = a, out[grp * 2 + 1] = b;
        ld(ra, grp + 2);
        fold(rb, a, b);
        if (lane == 0) out[grp * 2 + 2] = a, out[grp * 2 + 3] = b;
    }
    if (grp < rg.g1) {
        fold(ra, a, b);
        if (lane == 0) out[grp * 2] = a, out[grp * 2 + 1] = b;
    }
}

// k_fixed<false> with non-temporal item loads (the product's loop, its loads
// through ldp<true>)
__global__ __launch_bounds__(1024) void k1nt(const uint8_t *__restrict__ base, const uint4 *__restrict__ img,
                                             uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
    using Regs = ItemRegs<32, kK1CH, kK1Rows>;
    const uint32_t lane = threadIdx.x & 63u, li = lane & 31u, g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t ngroups = kItems / 2;
    const Range rg = k1_range(ngroups);
    if (rg.g0 >= ngroups) return;
    Regs ra, rb;
    auto ld = [&](Regs &r, uint64_t gi) {
        const uint64_t gu = gi < rg.g1 ? gi : rg.g1 - 1;
        const uint8_t *wb = base + gu * 2 * kItemBytes + g * (uint32_t)kItemBytes + li * kK1CH;
        r.cin = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int q = 0; q < 2; ++q) r.d[i][q] = ldp<true>(wb + i * 1024 + 16 * q);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto part0 = [&](Regs &m) {
        if (li == 0) m.d[0][0].x ^= ~m.cin;
        return reduce_level<0>(lane_partial_x3s<kK1CH>(m, c), (lane & 1u) == 0u);
    };
    uint64_t grp = rg.g0;
    const uint64_t nsteps = rg.g1 - rg.g0;
    ld(ra, grp);
    uint64_t k = 0;
    for (; k + 4 <= nsteps; k += 4) {
        ld(rb, grp + 1);
        const uint32_t va = part0(ra);
        ld(ra, grp + 2);
        const uint32_t vb = part0(rb);
        const uint32_t vab = group_pair_level1(va, vb, lane);
        ld(rb, grp + 3);
        const uint32_t vc = part0(ra);
        ld(ra, grp + 4);
        const uint32_t vd = part0(rb);
        const uint32_t raw = group_reduce32_quad(vab, group_pair_level1(vc, vd, lane), lane);
        if (li < 4) out[(grp + li) * 2 + g] = ~raw;
        grp += 4;
    }
    for (; k + 2 <= nsteps; k += 2) {
        ld(rb, grp + 1);
        const uint32_t va = part0(ra);
        ld(ra, grp + 2);
        const uint32_t vb = part0(rb);
        const uint32_t raw = group_reduce32_pair(va, vb, lane);
        if (li < 2) out[(li == 0 ? grp : grp + 1) * 2 + g] = ~raw;
        grp += 2;
    }
    if (nsteps & 1) {
        if (li == 0) ra.d[0][0].x ^= ~ra.cin;
        const uint32_t raw = group_reduce32_dpp(lane_partial_x3s<kK1CH>(ra, c), lane);
        if (li == 0) out[grp * 2 + g] = ~raw;
    }
}

// K1c: K1 with coalesced loads.  A 32-lane group still owns one item, but
// lane i holds the 16-B pieces at 512 k + 16 i (k = 0..7): each load
// instruction reads 512 contiguous bytes per group (1 KiB per wave, two
// items).  Chains: one per piece (4 dwords); the pieces of each half item
// fold into the lane value through the shifted last steps (M_1536, M_1024,
// M_512; slots 156, 24, 20 of build_lds_image_span at chunk 16), the first
// half is moved up by M_2048 (tables 16..19), and the lane tree runs on
// 16-B granules (levels M_16 .. M_128, level 4 = level 3 twice).
struct K1cRegs {
    uint4 d[8];
    uint32_t cin;
};
__device__ __forceinline__ uint32_t k1c_partial(const K1cRegs &r, const LaneCtx &c) {
    constexpr uint32_t kShift[3] = {kAuxShift0, kAuxShift1, kAuxShift2};
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = r.d[k].x;
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = step4_next(x[k], dw4(r.d[k], i), c);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (k & 3) < 3 ? step4_last_shifted(x[k], kShift[k & 3]) : step4_next(x[k], 0u, c);
    const uint32_t ua = xor3(x[0], x[1], x[2]) ^ x[3], ub = xor3(x[4], x[5], x[6]) ^ x[7];
    return apply_op<4>(kAuxSpanFold, ua) ^ ub;
}
template <bool NT>
__global__ __launch_bounds__(1024) void k1c(const uint8_t *__restrict__ base, const uint4 *__restrict__ img,
                                            uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
    const uint32_t lane = threadIdx.x & 63u, li = lane & 31u, g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t ngroups = kItems / 2;
    const Range rg = k1_range(ngroups);
    if (rg.g0 >= ngroups) return;
    K1cRegs ra, rb;
    auto ld = [&](K1cRegs &r, uint64_t gi) {
        const uint64_t gu = gi < rg.g1 ? gi : rg.g1 - 1;
        const uint8_t *wb = base + gu * 2 * kItemBytes + g * (uint32_t)kItemBytes + li * 16;
        r.cin = 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) r.d[k] = ldp<NT>(wb + 512 * k);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto part0 = [&](K1cRegs &m) {
        if (li == 0) m.d[0].x ^= ~m.cin;
        return reduce_level<0>(k1c_partial(m, c), (lane & 1u) == 0u);
    };
    uint64_t grp = rg.g0;
    const uint64_t nsteps = rg.g1 - rg.g0;
    ld(ra, grp);
    uint64_t k = 0;
    for (; k + 4 <= nsteps; k += 4) {
        ld(rb, grp + 1);
        const uint32_t va = part0(ra);
        ld(ra, grp + 2);
        const uint32_t vb = part0(rb);
        const uint32_t vab = group_pair_level1(va, vb, lane);
        ld(rb, grp + 3);
        const uint32_t vc = part0(ra);
        ld(ra, grp + 4);
        const uint32_t vd = part0(rb);
        const uint32_t raw = group_reduce32_quad_span(vab, group_pair_level1(vc, vd, lane), lane);
        if (li < 4) out[(grp + li) * 2 + g] = ~raw;
        grp += 4;
    }
    for (; k + 2 <= nsteps; k += 2) {
        ld(rb, grp + 1);
        const uint32_t va = part0(ra);
        ld(ra, grp + 2);
        const uint32_t vb = part0(rb);
        const uint32_t raw = group_reduce32_pair_span(va, vb, lane);
        if (li < 2) out[(li == 0 ? grp : grp + 1) * 2 + g] = ~raw;
        grp += 2;
    }
    if (nsteps & 1) {
        if (li == 0) ra.d[0].x ^= ~ra.cin;
        uint32_t v = reduce_level<0>(k1c_partial(ra, c), (lane & 1u) == 0u);
        v = reduce_level<1>(v, (lane & 3u) == 0u);
        v = reduce_level<2>(v, (lane & 7u) == 0u);
        v = reduce_level<3>(v, (lane & 15u) == 0u);
        const uint32_t raw = reduce_level4_span(v, (lane & 31u) == 0u);
        if (li == 0) out[grp * 2 + g] = ~raw;
    }
}

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14, others at max)
template <int N>
__device__ __forceinline__ void wait_vm() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

// LDS-DMA stream: a step = S bytes of the wave's range (S / 1024 wave
// instructions) into slot (step % B) of the wave's ring; B - 1 steps in flight.
template <int S, int B, bool NT>
__global__ void glds(const uint8_t *__restrict__ base, uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int J = S / 1024;  // wave instructions per step
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    // steps over the same item-pair ranges as K1 (a pair is 8 KiB)
    const uint64_t ngroups = kItems / 2;
    const Range rg = k1_range(ngroups);
    if (rg.g0 >= ngroups) return;
    const uint64_t b0 = rg.g0 * 8192, nsteps = (rg.g1 - rg.g0) * 8192 / S;
    __attribute__((address_space(3))) char *ring = (__attribute__((address_space(3))) char *)smem + wave * (S * B);
    auto issue = [&](uint64_t s) {
        const uint64_t su = s < nsteps ? s : nsteps - 1;
        const uint8_t *src = base + b0 + su * S + lane * 16;
        __attribute__((address_space(3))) char *dst = ring + (s % B) * S;
#pragma unroll
        for (int j = 0; j < J; ++j)
            __builtin_amdgcn_global_load_lds((const void *)(src + j * 1024), (__attribute__((address_space(3))) void *)(dst + j * 1024), 16, 0, NT ? 2 : 0);
    };
#pragma unroll
    for (int s = 0; s < B - 1; ++s) issue(s);
    uint32_t acc = 0;  // XOR of this lane's 16 B of the current item, all its KiB
    for (uint64_t s = 0; s < nsteps; ++s) {
        issue(s + B - 1);
        wait_vm<J * (B - 1)>();  // step s landed (the B - 1 younger steps may be in flight)
        const __attribute__((address_space(3))) char *src = ring + (s % B) * S;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const u32x4 v = *(const __attribute__((address_space(3))) u32x4 *)(src + j * 1024 + lane * 16);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
            const uint64_t kib = s * J + j;  // KiB index in the range
            if ((kib & 3) == 3) {            // the item's last KiB
                uint32_t x = wave_xor32(acc);
                x ^= __shfl_xor(x, 32);
                if (lane == 0) out[rg.g0 * 2 + kib / 4] = x;
                acc = 0;
            }
        }
        // (the slot is rewritten B - 1 steps later, after this wave's reads:
        // ds_reads retire in order before the next DMA into it is issued)
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    }
    wait_vm<0>();
}

__global__ void fill(uint32_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9e3779b97f4a7c15ull;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        p[i] = (uint32_t)(z ^ (z >> 31));
    }
}

template <typename F>
float time_median(F launch, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a, 0));
        launch();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("device %s  CUs %d  reps %d\n", p.gcnArchName, cus, reps);
    const uint64_t bytes = kItems * kItemBytes;
    uint8_t *d;
    uint32_t *out, *ref;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&out, kItems * 4));
    CHECK(hipMalloc(&ref, kItems * 4));
    fill<<<4096, 256>>>((uint32_t *)d, bytes / 4);
    std::vector<uint32_t> img(mcrc::kImageK1Dwords);
    mcrc::build_lds_image_k1(img.data(), kK1CH);
    uint4 *dimg;
    CHECK(hipMalloc(&dimg, img.size() * 4));
    CHECK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> img_c(mcrc::kImageK1Dwords);
    mcrc::build_lds_image_span(img_c.data(), 16);
    uint4 *dimg_c;
    CHECK(hipMalloc(&dimg_c, img_c.size() * 4));
    CHECK(hipMemcpy(dimg_c, img_c.data(), img_c.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipFuncSetAttribute((const void *)k_fixed<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageK1Bytes));
    auto run_k1 = [&] {
        hipLaunchKernelGGL((k_fixed<false, true>), dim3(cus), dim3(1024), kLdsImageK1Bytes, 0, d, kItemBytes, kItems, dimg_c,
                           nullptr, out);
    };
    // clock settle: 300 ms of K1 launches (not for a counter pass: REPS 1)
    if (reps > 1) {
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(300)) {
            for (int i = 0; i < 20; ++i) run_k1();
            CHECK(hipDeviceSynchronize());
        }
    }
    std::vector<uint32_t> h_ref(kItems), h(kItems);
    auto report = [&](const char *name, float ms, bool check) {
        bool same = true;
        if (check) {
            CHECK(hipMemcpy(h.data(), out, kItems * 4, hipMemcpyDeviceToHost));
            same = memcmp(h.data(), h_ref.data(), kItems * 4) == 0;
        }
        printf("%-28s %.4f ms  %7.1f GB/s  %5.1f %% of 8 TB/s%s\n", name, ms, bytes / (ms * 1e-3) / 1e9,
               bytes / (ms * 1e-3) / 8e12 * 100, check ? (same ? "  xor ok" : "  XOR MISMATCH") : "");
        fflush(stdout);
    };
    CHECK(hipFuncSetAttribute((const void *)k1nt, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageK1Bytes));
    CHECK(hipFuncSetAttribute((const void *)k1c<false>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageK1Bytes));
    CHECK(hipFuncSetAttribute((const void *)k1c<true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageK1Bytes));

    std::vector<uint32_t> h_crc(kItems);
    for (int round = 0; round < 2; ++round) {
        printf("-- round %d\n", round);
        const float t_k1 = time_median(run_k1, reps);
        CHECK(hipMemcpy(h_crc.data(), out, kItems * 4, hipMemcpyDeviceToHost));
        report("k_fixed (product)", t_k1, false);
        CHECK(hipMemset(out, 0, kItems * 4));
        const float t_k1nt = time_median([&] { hipLaunchKernelGGL(k1nt, dim3(cus), dim3(1024), kLdsImageK1Bytes, 0, d, dimg, out); }, reps);
        CHECK(hipMemcpy(h.data(), out, kItems * 4, hipMemcpyDeviceToHost));
        printf("%-28s %.4f ms  %7.1f GB/s  %5.1f %% of 8 TB/s  %s\n", "k1nt (K1, nt loads)", t_k1nt,
               bytes / (t_k1nt * 1e-3) / 1e9, bytes / (t_k1nt * 1e-3) / 8e12 * 100,
               memcmp(h.data(), h_crc.data(), kItems * 4) == 0 ? "crc = k_fixed" : "CRC MISMATCH");
        for (int nt = 0; nt < 2; ++nt) {
            CHECK(hipMemset(out, 0, kItems * 4));
            const float t = time_median([&] {
                if (nt) hipLaunchKernelGGL(k1c<true>, dim3(cus), dim3(1024), kLdsImageK1Bytes, 0, d, dimg_c, out);
                else hipLaunchKernelGGL(k1c<false>, dim3(cus), dim3(1024), kLdsImageK1Bytes, 0, d, dimg_c, out);
            }, reps);
            CHECK(hipMemcpy(h.data(), out, kItems * 4, hipMemcpyDeviceToHost));
            printf("%-28s %.4f ms  %7.1f GB/s  %5.1f %% of 8 TB/s  %s\n", nt ? "k1c nt (coalesced K1)" : "k1c (coalesced K1)", t,
                   bytes / (t * 1e-3) / 1e9, bytes / (t * 1e-3) / 8e12 * 100,
                   memcmp(h.data(), h_crc.data(), kItems * 4) == 0 ? "crc = k_fixed" : "CRC MISMATCH");
        }
        CHECK(hipMemset(out, 0, kItems * 4));
        const float t_load = time_median([&] { hipLaunchKernelGGL(k1load<false>, dim3(cus), dim3(1024), 0, 0, d, out); }, reps);
        if (round == 0) CHECK(hipMemcpy(h_ref.data(), out, kItems * 4, hipMemcpyDeviceToHost));
        report("k1load (K1 loads, XOR)", t_load, round > 0);
        CHECK(hipMemset(out, 0, kItems * 4));
        report("k1load nt",
               time_median([&] { hipLaunchKernelGGL(k1load<true>, dim3(cus), dim3(1024), 0, 0, d, out); }, reps), true);
        CHECK(hipMemset(out, 0, kItems * 4));
        report("coalesced (1 KiB / instr)",
               time_median([&] { hipLaunchKernelGGL(coalesced<false>, dim3(cus), dim3(1024), 0, 0, d, out); }, reps), true);
        CHECK(hipMemset(out, 0, kItems * 4));
        report("coalesced nt",
               time_median([&] { hipLaunchKernelGGL(coalesced<true>, dim3(cus), dim3(1024), 0, 0, d, out); }, reps), true);
#define GLDS(W, S, B, NT)                                                                                     \
    {                                                                                                         \
        CHECK(hipFuncSetAttribute((const void *)glds<S, B, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (W) * (S) * (B)));                                                          \
        CHECK(hipMemset(out, 0, kItems * 4));                                                                 \
        report("glds W" #W " S" #S " B" #B " nt" #NT,                                                          \
               time_median([&] { hipLaunchKernelGGL((glds<S, B, NT>), dim3(cus), dim3(64 * (W)), (W) * (S) * (B), 0, d, out); }, \
                           reps),                                                                             \
               true);                                                                                         \
    }
        GLDS(16, 2048, 4, false)
        GLDS(16, 2048, 4, true)
        GLDS(8, 8192, 2, true)
        GLDS(8, 4096, 4, true)
        GLDS(8, 4096, 2, true)
        GLDS(16, 1024, 4, true)
        GLDS(4, 8192, 4, true)
    }
    CHECK(hipFree(d));
    return 0;
}
