// k1_waves.hip -- dev experiment (not part of the library), round 6 review
// item 4: is the LDS-DMA streams' lead over K1 (84-86 % against 80.7 %,
// profiles/r05_k1_ceiling.txt) the LDS-DMA mechanism or the stream count?
// The r05 LDS-DMA streams ran 8 waves per CU, the register streams and K1 16.
// Over the headline batch (1 Mi x 4096 B), median of REPS event-timed
// launches after a 300 ms clock settle, one workgroup per CU:
//   k_fixed W16 / W8   the product K1 (included) with 1024 / 512 threads
//   reg W D            K1's load shape (each wave-instruction one contiguous
//                      KiB, nt) into a register ring of D item pairs (8 KiB
//                      each), XOR instead of the chains, W waves per CU
//   glds W8 S4096 B2   r05's best LDS-DMA stream (reference point)
// Every load-only mode writes each item's XOR of its dwords (checked equal).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/k1_waves.hip -o tools/k1_waves
//   tools/k1_waves [REPS]
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

struct Range {
    uint64_t g0, g1;
};
__device__ __forceinline__ Range k1_range(uint64_t ngroups) {  // K1's wave -> item-pair range
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t gstep = gridDim.x * waves;
    uint64_t grp = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6));
    if (gstep % 65521u) grp = (grp * 65521u) % gstep;
    const uint64_t cg = (ngroups + gstep - 1) / gstep;
    return Range{grp * cg, min((grp + 1) * cg, ngroups)};
}
__device__ __forceinline__ uint32_t wave_xor32(uint32_t v) {
    v ^= __shfl_xor(v, 1);
    v ^= __shfl_xor(v, 2);
    v ^= __shfl_xor(v, 4);
    v ^= __shfl_xor(v, 8);
    v ^= __shfl_xor(v, 16);
    return v;
}

struct Pair {
    uint4 v[8];
};
template <int D, int W>
__global__ __launch_bounds__(64 * W) void reg_ring(const uint8_t *__restrict__ base, uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t ngroups = kItems / 2;
    const Range rg = k1_range(ngroups);
    if (rg.g0 >= ngroups) return;
    Pair r[D];
    auto ld = [&](Pair &p, uint64_t gi) {
        const uint64_t gu = gi < rg.g1 ? gi : rg.g1 - 1;
        const uint8_t *wb = base + gu * 2 * kItemBytes;
#pragma unroll
        for (int j = 0; j < 8; ++j) p.v[j] = ld16_nt(wb + j * 1024 + lane * 16);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto fold = [&](const Pair &p, uint64_t gi) {
        uint32_t x = 0, y = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) x ^= p.v[j].x ^ p.v[j].y ^ p.v[j].z ^ p.v[j].w;
#pragma unroll
        for (int j = 4; j < 8; ++j) y ^= p.v[j].x ^ p.v[j].y ^ p.v[j].z ^ p.v[j].w;
        x = wave_xor32(x);
        y = wave_xor32(y);
        x ^= __shfl_xor(x, 32);
        y ^= __shfl_xor(y, 32);
        if (lane == 0) out[gi * 2] = x, out[gi * 2 + 1] = y;
    };
    uint64_t grp = rg.g0;
#pragma unroll
    for (int j = 0; j < D - 1; ++j) ld(r[j], grp + j);
    for (; grp + D <= rg.g1; grp += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            ld(r[(j + D - 1) % D], grp + j + D - 1);
            fold(r[j], grp + j);
        }
    }
#pragma unroll
    for (int j = 0; j < D - 1; ++j)
        if (grp + j < rg.g1) fold(r[j], grp + j);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}
template <int S, int B>
__global__ void glds(const uint8_t *__restrict__ base, uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int J = S / 1024;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
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
            __builtin_amdgcn_global_load_lds((const void *)(src + j * 1024),
                                             (__attribute__((address_space(3))) void *)(dst + j * 1024), 16, 0, 2);
    };
#pragma unroll
    for (int s = 0; s < B - 1; ++s) issue(s);
    uint32_t acc = 0;
    for (uint64_t s = 0; s < nsteps; ++s) {
        issue(s + B - 1);
        wait_vm<J * (B - 1)>();
        const __attribute__((address_space(3))) char *src = ring + (s % B) * S;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const u32x4 v = *(const __attribute__((address_space(3))) u32x4 *)(src + j * 1024 + lane * 16);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
            const uint64_t kib = s * J + j;
            if ((kib & 3) == 3) {
                uint32_t x = wave_xor32(acc);
                x ^= __shfl_xor(x, 32);
                if (lane == 0) out[rg.g0 * 2 + kib / 4] = x;
                acc = 0;
            }
        }
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
    uint32_t *out;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&out, kItems * 4));
    fill<<<4096, 256>>>((uint32_t *)d, bytes / 4);
    std::vector<uint32_t> img(mcrc::kImageK1Dwords);
    mcrc::build_lds_image_span(img.data(), 16);
    uint4 *dimg;
    CHECK(hipMalloc(&dimg, img.size() * 4));
    CHECK(hipMemcpy(dimg, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipFuncSetAttribute((const void *)k_fixed<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kLdsImageK1Bytes));
    auto run_k1 = [&](int threads) {
        hipLaunchKernelGGL((k_fixed<false, true>), dim3(cus), dim3(threads), kLdsImageK1Bytes, 0, d, kItemBytes, kItems,
                           dimg, nullptr, out);
    };
    if (reps > 1) {
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(300)) {
            for (int i = 0; i < 20; ++i) run_k1(1024);
            CHECK(hipDeviceSynchronize());
        }
    }
    std::vector<uint32_t> h_ref(kItems), h(kItems), h_crc(kItems), h_crc2(kItems);
    auto line = [&](const char *name, float ms, const char *note) {
        printf("%-24s %.4f ms  %7.1f GB/s  %5.1f %% of 8 TB/s  %s\n", name, ms, bytes / (ms * 1e-3) / 1e9,
               bytes / (ms * 1e-3) / 8e12 * 100, note);
        fflush(stdout);
    };
    // (the load-only kernels take 160 KiB of dynamic LDS: one workgroup per CU, as K1)
#define REG(W, D)                                                                                                 \
    {                                                                                                             \
        CHECK(hipFuncSetAttribute((const void *)reg_ring<D, W>, hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                  kLdsImageK1Bytes));                                                            \
        CHECK(hipMemset(out, 0, kItems * 4));                                                                    \
        const float t = time_median(                                                                             \
            [&] { hipLaunchKernelGGL((reg_ring<D, W>), dim3(cus), dim3(64 * (W)), kLdsImageK1Bytes, 0, d, out); }, reps); \
        CHECK(hipMemcpy(h.data(), out, kItems * 4, hipMemcpyDeviceToHost));                                      \
        if (!have_ref) h_ref = h, have_ref = true;                                                               \
        line("reg W" #W " D" #D, t, memcmp(h.data(), h_ref.data(), kItems * 4) == 0 ? "xor ok" : "XOR MISMATCH"); \
    }
    for (int round = 0; round < 3; ++round) {
        printf("-- round %d\n", round);
        bool have_ref = round > 0;
        CHECK(hipMemset(out, 0, kItems * 4));
        const float t16 = time_median([&] { run_k1(1024); }, reps);
        CHECK(hipMemcpy(h_crc.data(), out, kItems * 4, hipMemcpyDeviceToHost));
        line("k_fixed W16 (product)", t16, "");
        CHECK(hipMemset(out, 0, kItems * 4));
        const float t8 = time_median([&] { run_k1(512); }, reps);
        CHECK(hipMemcpy(h_crc2.data(), out, kItems * 4, hipMemcpyDeviceToHost));
        line("k_fixed W8", t8, memcmp(h_crc.data(), h_crc2.data(), kItems * 4) == 0 ? "crc = W16" : "CRC MISMATCH");
        REG(16, 2)
        REG(16, 3)
        REG(8, 2)
        REG(8, 3)
        REG(8, 4)
        REG(8, 6)
        REG(4, 4)
        REG(4, 8)
        {
            CHECK(hipFuncSetAttribute((const void *)glds<4096, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      8 * 4096 * 2));
            CHECK(hipMemset(out, 0, kItems * 4));
            const float t = time_median(
                [&] { hipLaunchKernelGGL((glds<4096, 2>), dim3(cus), dim3(512), 8 * 4096 * 2, 0, d, out); }, reps);
            CHECK(hipMemcpy(h.data(), out, kItems * 4, hipMemcpyDeviceToHost));
            line("glds W8 S4096 B2 nt", t, memcmp(h.data(), h_ref.data(), kItems * 4) == 0 ? "xor ok" : "XOR MISMATCH");
        }
    }
    CHECK(hipFree(d));
    CHECK(hipFree(out));
    return 0;
}
