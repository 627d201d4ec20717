// k1_ring.hip -- dev experiment (not part of the library), round 6 review
// item 4.  tools/k1_waves.hip found the plain register stream at 85 % with
// two item pairs in flight per wave (16 waves) against 83.5 % with one, and
// the product K1 (16 waves, three half-steps = 12 KiB in flight per wave) at
// 79-80 %, 81 % with 8 waves.  Here K1 with a ring of 8 half-steps (7 in
// flight, 28 KiB per wave) at 8 waves per CU (256 VGPRs per wave allowed),
// against the product at 16 and 8 waves, in one session.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/k1_ring.hip -o tools/k1_ring
//   tools/k1_ring [REPS]
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

// k_fixed<CRCIN, NT> with an NH-slot ring of half-steps (NH - 1 in flight);
// NH divides 8, so a 4-step body (8 halves) maps halves to slots statically.
template <bool CRCIN, int NH, int THREADS>
__global__ __launch_bounds__(THREADS) void k1_ring(const uint8_t *__restrict__ base, uint64_t stride, uint64_t nitems,
                                                   const uint4 *__restrict__ img, const uint32_t *__restrict__ crc_in,
                                                   uint32_t *__restrict__ out) {
    static_assert(8 % NH == 0 && NH >= 4, "NH divides the 8 halves of a 4-step body");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
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
    uint64_t grp = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6));
    if (gstep % 65521u) grp = (grp * 65521u) % gstep;
    const uint64_t cg = (ngroups + gstep - 1) / gstep;
    const uint64_t gend = min((grp + 1) * cg, ngroups);
    grp *= cg;
    if (grp >= ngroups) return;
    const uint64_t glast = gend - 1;
    auto item_of = [&](uint64_t gi) { return gi * IPW + g; };
    auto ldh = [&](K1Half &r, uint64_t gi, int q) {
        const bool real = gi < gend;
        const uint64_t gu = real ? gi : glast;
        const uint64_t first = gu * IPW;
        const uint8_t *wb = real ? base + first * stride : reinterpret_cast<const uint8_t *>(img);
        const uint32_t gl = first + g < nitems ? g : (uint32_t)(nitems - 1 - first);
        if (q == 0) {
            if constexpr (CRCIN) r.cin = crc_in[first + gl];
            else r.cin = 0u;
        }
        const uint32_t loff = (real ? gl * (uint32_t)stride : g * kK1Bytes) + li * kK1LaneBytes + 4u * kK1Piece * (uint32_t)q;
#pragma unroll
        for (int k = 0; k < 4; ++k) r.d[k] = ld16_nt(wb + loff + k * kK1Piece);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto half0 = [&](K1Half &m) {
        if (li == 0) m.d[0].x ^= ~m.cin;
        return apply_op<4>(kAuxSpanFold, k1_half_value(m, c));
    };
    auto part0 = [&](uint32_t u0, K1Half &m1) { return reduce_level<0>(u0 ^ k1_half_value(m1, c), (lane & 1u) == 0u); };
    K1Half h[NH];
    const uint64_t nsteps = gend - grp;
    // half t (of the range) is step grp0 + t / 2, half t % 2, in slot t % NH
#pragma unroll
    for (int t = 0; t < NH - 1; ++t) ldh(h[t], grp + t / 2, t & 1);
    // One step s of the body (halves 2s, 2s + 1), each half preceded by the
    // issue of the half NH - 1 further on
    auto step = [&](int s, uint64_t base_grp) {
        const int ta = 2 * s, tb = 2 * s + 1;
        ldh(h[(ta + NH - 1) % NH], base_grp + (ta + NH - 1) / 2, (ta + NH - 1) & 1);
        const uint32_t u0 = half0(h[ta % NH]);
        ldh(h[(tb + NH - 1) % NH], base_grp + (tb + NH - 1) / 2, (tb + NH - 1) & 1);
        return part0(u0, h[tb % NH]);
    };
    uint64_t k = 0;
    for (; k + 4 <= nsteps; k += 4) {
        const uint32_t va = step(0, grp);
        const uint32_t vb = step(1, grp);
        const uint32_t vab = group_pair_level1(va, vb, lane);
        const uint32_t vc = step(2, grp);
        const uint32_t vd = step(3, grp);
        const uint32_t raw = group_reduce32_quad_span(vab, group_pair_level1(vc, vd, lane), lane);
        const uint64_t item = item_of(grp + (li & 3u));
        if (li < 4 && item < nitems) out[item] = ~raw;
        grp += 4;
    }
    // the last 0..3 steps: their halves (at most 6) are issued already when
    // NH = 8; with NH = 4 each step issues as in the body
    const uint64_t r = nsteps - k;
    if (r >= 2) {
        const uint32_t va = step(0, grp);
        const uint32_t vb = step(1, grp);
        const uint32_t raw = group_reduce32_pair_span(va, vb, lane);
        const uint64_t item = item_of(li == 0 ? grp : grp + 1);
        if (li < 2 && item < nitems) out[item] = ~raw;
    }
    if (r & 1) {
        uint32_t v = r >= 2 ? step(2, grp) : step(0, grp);
        const uint64_t gi = r >= 2 ? grp + 2 : grp;
        v = reduce_level<1>(v, (lane & 3u) == 0u);
        v = reduce_level<2>(v, (lane & 7u) == 0u);
        v = reduce_level<3>(v, (lane & 15u) == 0u);
        const uint32_t raw = reduce_level4_span(v, (lane & 31u) == 0u);
        const uint64_t item = item_of(gi);
        if (li == 0 && item < nitems) out[item] = ~raw;
    }
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
    uint32_t *out, *cin;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&out, kItems * 4));
    CHECK(hipMalloc(&cin, kItems * 4));
    fill<<<4096, 256>>>((uint32_t *)d, bytes / 4);
    fill<<<1024, 256>>>(cin, kItems);
    std::vector<uint32_t> img(mcrc::kImageK1Dwords);
    mcrc::build_lds_image_span(img.data(), 16);
    uint4 *dimg;
    CHECK(hipMalloc(&dimg, img.size() * 4));
    CHECK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    const void *ks[] = {(const void *)k_fixed<false, true>, (const void *)k_fixed<true, true>,
                        (const void *)k1_ring<false, 8, 512>, (const void *)k1_ring<true, 8, 512>,
                        (const void *)k1_ring<false, 4, 1024>, (const void *)k1_ring<false, 4, 512>};
    for (const void *k : ks) CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsImageK1Bytes));
    auto prod = [&](int threads, bool ci) {
        if (ci)
            hipLaunchKernelGGL((k_fixed<true, true>), dim3(cus), dim3(threads), kLdsImageK1Bytes, 0, d, kItemBytes, kItems,
                               dimg, cin, out);
        else
            hipLaunchKernelGGL((k_fixed<false, true>), dim3(cus), dim3(threads), kLdsImageK1Bytes, 0, d, kItemBytes, kItems,
                               dimg, nullptr, out);
    };
    {
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(300)) {
            for (int i = 0; i < 20; ++i) prod(1024, false);
            CHECK(hipDeviceSynchronize());
        }
    }
    std::vector<uint32_t> want(kItems), want_ci(kItems), h(kItems);
    prod(1024, false);
    CHECK(hipMemcpy(want.data(), out, kItems * 4, hipMemcpyDeviceToHost));
    prod(1024, true);
    CHECK(hipMemcpy(want_ci.data(), out, kItems * 4, hipMemcpyDeviceToHost));
    auto line = [&](const char *name, float ms, const std::vector<uint32_t> &w) {
        CHECK(hipMemcpy(h.data(), out, kItems * 4, hipMemcpyDeviceToHost));
        printf("%-28s %.4f ms  %7.1f GB/s  %5.1f %% of 8 TB/s  %s\n", name, ms, bytes / (ms * 1e-3) / 1e9,
               bytes / (ms * 1e-3) / 8e12 * 100, memcmp(h.data(), w.data(), kItems * 4) == 0 ? "crc ok" : "CRC MISMATCH");
        fflush(stdout);
    };
    // odd item counts: every tail of the ring kernels against the product
    for (uint64_t n : {1ull, 2ull, 3ull, 5ull, 4097ull, 65535ull, 1000003ull}) {
        CHECK(hipMemset(out, 0, kItems * 4));
        hipLaunchKernelGGL((k1_ring<true, 8, 512>), dim3(cus), dim3(512), kLdsImageK1Bytes, 0, d, kItemBytes, n, dimg, cin,
                           out);
        CHECK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
        printf("k1_ring<8> W8 crc_in, %llu items: %s\n", (unsigned long long)n,
               memcmp(h.data(), want_ci.data(), n * 4) == 0 ? "crc ok" : "CRC MISMATCH");
    }
    for (int round = 0; round < 4; ++round) {
        printf("-- round %d\n", round);
        CHECK(hipMemset(out, 0, kItems * 4));
        line("k_fixed W16 (product)", time_median([&] { prod(1024, false); }, reps), want);
        CHECK(hipMemset(out, 0, kItems * 4));
        line("k_fixed W8", time_median([&] { prod(512, false); }, reps), want);
        CHECK(hipMemset(out, 0, kItems * 4));
        line("k1_ring NH8 W8", time_median([&] {
                 hipLaunchKernelGGL((k1_ring<false, 8, 512>), dim3(cus), dim3(512), kLdsImageK1Bytes, 0, d, kItemBytes,
                                    kItems, dimg, nullptr, out);
             }, reps), want);
        CHECK(hipMemset(out, 0, kItems * 4));
        line("k1_ring NH4 W16", time_median([&] {
                 hipLaunchKernelGGL((k1_ring<false, 4, 1024>), dim3(cus), dim3(1024), kLdsImageK1Bytes, 0, d, kItemBytes,
                                    kItems, dimg, nullptr, out);
             }, reps), want);
        CHECK(hipMemset(out, 0, kItems * 4));
        line("k1_ring NH4 W8", time_median([&] {
                 hipLaunchKernelGGL((k1_ring<false, 4, 512>), dim3(cus), dim3(512), kLdsImageK1Bytes, 0, d, kItemBytes,
                                    kItems, dimg, nullptr, out);
             }, reps), want);
    }
    CHECK(hipFree(d));
    CHECK(hipFree(out));
    CHECK(hipFree(cin));
    return 0;
}
