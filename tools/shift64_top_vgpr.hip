// shift64_top_vgpr.hip -- names the cause of the 24-VGPR header miscompute
// (DESIGN.md §3.7).  Not part of the library; self-contained (the library's
// parse_hdr no longer has the 64-bit form under test).
//
// Hypothesis: a VALU 64-bit shift (v_lshlrev_b64 / v_lshrrev_b64 /
// v_ashrrev_i64) whose shift-amount operand is the LAST VGPR of the wave's
// allocation computes wrongly when another wave is co-resident on the SIMD.
// LLVM carries a workaround for a bug of this shape ("Shift64HighRegBug":
// amount in v7, v15, v23 ... moved to a free register) but enables it for
// gfx90a only.  The round-5 reproducer's failing parse (24 VGPRs) took the
// amount of both its left shifts from v23, the top of its allocation; the
// same instruction stream at 32 VGPRs (v23 no longer the top) was exact.
//
// The experiment holds the parse fixed (the round-5 64-bit funnel of image
// bytes 28..43) and moves only the register the left shifts read their
// amount from, pinned with an inline-asm register constraint:
//   C24      the compiler's choice (this build: v21), allocation 24
//   A24/v4   amount pinned to v4,  allocation 24  -> not the top
//   A24/v23  amount pinned to v23, allocation 24  -> the top
//   A32/v23  amount pinned to v23, allocation 32  -> 7 mod 8, not the top
//   A32/v31  amount pinned to v31, allocation 32  -> the top
//   A40/v31  amount pinned to v31, allocation 40  -> 7 mod 8, not the top
// Each kernel parses 1000 headers per 4 MiB wbuf at one alignment (16 runs,
// one per sh = (p + 28) & 15) over 300 x 64 MiB pages, as PS24 did, and
// counts headers whose nbytes / nkey are not the filled values.  The
// allocations are checked on the CPU from the assembly before any run
// (tools/shift64_top_vgpr.sh).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/shift64_top_vgpr.hip -o /tmp/shift64_top_vgpr
//   /tmp/shift64_top_vgpr PAGES
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

constexpr uint32_t kWaves = 4;  // waves (wbufs) per workgroup, as the walk
constexpr uint32_t kPer = 1000, kStride = 4176;

// x << n with n read from VGPR PIN (-1: wherever the compiler puts it)
template <int PIN>
__device__ __forceinline__ uint64_t shl64(uint64_t x, uint32_t n) {
    if constexpr (PIN < 0) {
        return x << n;
    } else {
        uint64_t r;
        if constexpr (PIN == 4) asm volatile("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "{v4}"(n), "v"(x));
        else if constexpr (PIN == 23) asm volatile("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "{v23}"(n), "v"(x));
        else asm volatile("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "{v31}"(n), "v"(x));
        return r;
    }
}

struct Hdr {
    uint32_t nbytes, nkey;
};

// the round-5 parse: bytes 28..43 of the image funnelled out of two aligned
// 16-B pieces with 64-bit shifts
template <int PIN>
__device__ __forceinline__ Hdr parse64(const uint8_t *it) {
    const uint32_t sh = (uint32_t)((uintptr_t)(it + 28) & 15u);
    const uint8_t *q = it + 28 - sh;
    const bool two = sh + 13 >= 16;
    const uint4 u0 = *reinterpret_cast<const uint4 *>(q), u1 = *reinterpret_cast<const uint4 *>(q + (two ? 16 : 0));
    const uint64_t w0 = u0.x | ((uint64_t)u0.y << 32), w1 = u0.z | ((uint64_t)u0.w << 32);
    const uint64_t w2 = two ? (u1.x | ((uint64_t)u1.y << 32)) : 0, w3 = two ? (u1.z | ((uint64_t)u1.w << 32)) : 0;
    const uint64_t a0 = sh < 8 ? w0 : w1, a1 = sh < 8 ? w1 : w2, a2 = sh < 8 ? w2 : w3;
    const uint32_t k = 8 * (sh & 7u);
    const uint64_t f0 = k ? (a0 >> k) | shl64<PIN>(a1, 64 - k) : a0;  // image bytes 28..35
    const uint64_t f1 = k ? (a1 >> k) | shl64<PIN>(a2, 64 - k) : a1;  // 36..43
    return {(uint32_t)(f0 >> 32), (uint32_t)(f1 >> 40) & 0xffu};
}

// TOP: the allocation is raised to TOP VGPRs by a clobber of v(TOP - 1)
template <int TOP, int PIN>
__global__ __launch_bounds__(64 * kWaves) void k_parse(const uint8_t *base, uint64_t region, uint64_t nw,
                                                       uint32_t *cnt) {
    if constexpr (TOP == 32) asm volatile("" ::: "v31");
    if constexpr (TOP == 40) asm volatile("" ::: "v39");
    const uint32_t j = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t bad = 0;
    for (uint64_t w = (uint64_t)blockIdx.x * kWaves + wave; w < nw; w += (uint64_t)gridDim.x * kWaves) {
        const uint8_t *wb = base + w * region;
#pragma unroll 1
        for (uint32_t r = 0; r < 16; ++r) {
            const uint32_t i = r * 64u + j;
            if (i >= kPer) break;
            const Hdr h = parse64<PIN>(wb + (uint64_t)i * kStride);
            // every image has nbytes < 2^20 and nkey 10 or 0 (k_fill)
            bad += (h.nbytes >> 20 != 0u) | (h.nkey != 10u && h.nkey != 0u);
        }
    }
    if (bad) atomicAdd(cnt, bad);
}

// item i of wbuf w at w * wbuf + phase + i * kStride; nbytes 4098 with at most
// one of bits 0..19 flipped, nkey 10 (a few 0)
__global__ void k_fill(uint8_t *base, uint64_t nwb, uint64_t wbuf, uint32_t seed, uint32_t phase) {
    const uint64_t n = nwb * kPer;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t *it = base + (i / kPer) * wbuf + phase + (i % kPer) * kStride;
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15;
        x *= 0x2c1b3c6du;
        x ^= x >> 12;
        uint32_t nbytes = 4098;
        uint8_t nkey = 10;
        if (x % 3000 == 7) nbytes ^= 1u << (x >> 20) % 20;
        if (x % 7000 == 11) nkey = 0;
        memcpy(it + 32, &nbytes, 4);
        it[36] = 1;
        it[37] = 0;
        it[38] = 2;
        it[39] = 0;
        it[40] = 17;
        it[41] = nkey;
    }
}

int main(int argc, char **argv) {
    const uint64_t pages = argc > 1 ? strtoull(argv[1], nullptr, 10) : 300;
    const uint64_t wbuf = 4ull << 20, nwb = pages * 16, bytes = nwb * wbuf;
    uint8_t *d = nullptr;
    uint32_t *cnt = nullptr;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&cnt, 4));
    const int gw = (int)std::min<uint64_t>((nwb + kWaves - 1) / kWaves, 65535);
    printf("pages %llu wbufs %llu headers per alignment %llu\n", (unsigned long long)pages, (unsigned long long)nwb,
           (unsigned long long)(nwb * kPer));
    const char *names[] = {"C24 (compiler's choice: v21, alloc 24)", "A24/v4  (alloc 24, not the top)",
                           "A24/v23 (alloc 24, the top)",             "A32/v23 (alloc 32, not the top)",
                           "A32/v31 (alloc 32, the top)",             "A40/v31 (alloc 40, not the top)"};
    for (int v = 0; v < 6; ++v) {
        printf("%s: wrong parses by sh:", names[v]);
        uint64_t total = 0;
        for (uint32_t phase = 0; phase < 16; ++phase) {
            CHECK(hipMemset(d, 0x5a, bytes));
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, d, nwb, wbuf, 777u + phase, phase);
            CHECK(hipMemset(cnt, 0, 4));
            const uint8_t *b = d + phase;
            const dim3 g(gw), blk(64 * kWaves);
            if (v == 0) hipLaunchKernelGGL((k_parse<0, -1>), g, blk, 0, 0, b, wbuf, nwb, cnt);
            if (v == 1) hipLaunchKernelGGL((k_parse<0, 4>), g, blk, 0, 0, b, wbuf, nwb, cnt);
            if (v == 2) hipLaunchKernelGGL((k_parse<0, 23>), g, blk, 0, 0, b, wbuf, nwb, cnt);
            if (v == 3) hipLaunchKernelGGL((k_parse<32, 23>), g, blk, 0, 0, b, wbuf, nwb, cnt);
            if (v == 4) hipLaunchKernelGGL((k_parse<32, 31>), g, blk, 0, 0, b, wbuf, nwb, cnt);
            if (v == 5) hipLaunchKernelGGL((k_parse<40, 31>), g, blk, 0, 0, b, wbuf, nwb, cnt);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            uint32_t nbad = 0;
            CHECK(hipMemcpy(&nbad, cnt, 4, hipMemcpyDeviceToHost));
            printf(" %u:%u", (phase + 28) & 15, nbad);
            total += nbad;
            fflush(stdout);
        }
        printf("  total %llu\n", (unsigned long long)total);
    }
    CHECK(hipFree(cnt));
    CHECK(hipFree(d));
    return 0;
}
