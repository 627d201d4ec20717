// ubench.hip -- standalone microbenchmark for the fixed-length CRC kernel
// variants (no torch).  Dev tool: measures read bandwidth of each load pattern
// (LOAD_ONLY) and full CRC throughput, and checks every item against the
// shim's host CRC.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../memcached_amd/csrc/crc32c_gf2.h"
#include "../memcached_amd/csrc/crc32c_host.h"
#include "../memcached_amd/csrc/crc32c_kernels.hip"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                         \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9e3779b97f4a7c15ull;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        p[i] = z ^ (z >> 31);
    }
}

__global__ __launch_bounds__(1024) void k_read(const uint4 *__restrict__ p, uint64_t n16,
                                                uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^
               d.z ^ d.w;
    }
    for (; i < n16; i += stride) acc ^= p[i].x ^ p[i].y ^ p[i].z ^ p[i].w;
    if (acc == 0x12345678u) sink[0] = acc;
}

struct Variant {
    const char *name;
    int slice, lpi, ch;
    bool load_only;
    void (*kern)(const uint8_t *, uint64_t, uint64_t, const uint4 *, uint32_t, uint32_t,
                 const uint32_t *, uint32_t *);
    bool needs_cin = false;  // kernel reads crc_in[] unconditionally (CRCIN instances)
    uint32_t extra_lds = 0;
    bool k1img = false;  // MODE 13: the 160 KiB K1 image (shifted last-step tables)
};
#define V(S, L, C, R, M) \
    {#S "_l" #L "_c" #C "_r" #R "_m" #M, S, L, C, (M == 1 || M >= 9), mcrc_dev::k_fixed<S, L, C, R, M>}
#define VS(S, L, C, R, M, ST) \
    {#S "_l" #L "_c" #C "_r" #R "_m" #M "_st" #ST, S, L, C, (M == 1 || M >= 9), mcrc_dev::k_fixed<S, L, C, R, M, 2, ST>}
#define V3(S, L, C, R, M) \
    {#S "_l" #L "_c" #C "_r" #R "_m" #M "_d3", S, L, C, (M == 1 || M >= 9), mcrc_dev::k_fixed<S, L, C, R, M, 3>}
#define V11(F, CI) \
    {"4_l32_c32_r4_m11_f" #F "_ci" #CI, 4, 32, 32, false, mcrc_dev::k_fixed<4, 32, 32, 4, 11, 2, 0, 0, F, CI>, CI}
#define V12(F, CI) \
    {"4_l32_c32_r4_m12_f" #F "_ci" #CI, 4, 32, 32, false, mcrc_dev::k_fixed<4, 32, 32, 4, 12, 2, 0, 0, F, CI>, CI}
#define V13(F, CI) \
    {"4_l32_c32_r4_m13_f" #F "_ci" #CI, 4, 32, 32, false, mcrc_dev::k_fixed<4, 32, 32, 4, 13, 2, 0, 0, F, CI>, CI, 0, true}
#define V14(F, CI) \
    {"4_l32_c32_r4_m14_f" #F "_ci" #CI, 4, 32, 32, false, mcrc_dev::k_fixed<4, 32, 32, 4, 14, 2, 0, 0, F, CI>, CI, 0, true}
#define VP(S, L, C, R, M, D, P) \
    {#S "_l" #L "_c" #C "_r" #R "_m" #M "_d" #D "_p" #P, S, L, C, (M == 1 || M >= 9), mcrc_dev::k_fixed<S, L, C, R, M, D, 0, P>}

int main(int argc, char **argv) {
    const uint64_t nitems = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 20);
    const uint32_t len = 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const char *only = argc > 3 ? argv[3] : nullptr;  // substring filter on variant names
    const int only_bs = argc > 4 ? atoi(argv[4]) : 0;
    const int reps = argc > 5 ? atoi(argv[5]) : 1;  // interleaved repetitions of the variant list
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    printf("device %s CUs %d\n", prop.name, prop.multiProcessorCount);
    const uint64_t bytes = nitems * len;
    uint8_t *d_buf;
    uint32_t *d_out, *d_sink;
    CK(hipMalloc(&d_buf, bytes));
    CK(hipMalloc(&d_out, nitems * 4));
    CK(hipMalloc(&d_sink, 64));
    k_fill<<<4096, 256>>>((uint64_t *)d_buf, bytes / 8, 42);
    CK(hipDeviceSynchronize());

    std::vector<uint8_t> h_buf(bytes);
    CK(hipMemcpy(h_buf.data(), d_buf, bytes, hipMemcpyDeviceToHost));
    std::vector<uint32_t> want(nitems);
    auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = 0; i < nitems; ++i) want[i] = mcrc::crc32c_host_hw(0, &h_buf[i * len], len);
    auto t1 = std::chrono::steady_clock::now();
    printf("host crc (1 core): %.2f GiB/s\n",
           bytes / std::chrono::duration<double>(t1 - t0).count() / (1 << 30));

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (!only) {
        const int grid = prop.multiProcessorCount * 2;
        for (int w = 0; w < 2; ++w) k_read<<<grid, 1024>>>((const uint4 *)d_buf, bytes / 16, d_sink);
        CK(hipEventRecord(e0));
        for (int it = 0; it < iters; ++it)
            k_read<<<grid, 1024>>>((const uint4 *)d_buf, bytes / 16, d_sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        printf("%-28s %8.3f ms  %8.1f GB/s\n", "read_dwordx4_coalesced", ms, bytes / ms / 1e6);
    }

    Variant vars[] = {
        V11(true, false), V13(true, false), V14(true, false), V11(true, true), V13(true, true), V14(true, true),
        V(4, 32, 32, 4, 7),
        V(4, 32, 32, 4, 1),
    };
#ifdef MCRC_UBENCH_CLOCK
    const int max_grid = prop.multiProcessorCount * 2;
    uint64_t *d_stamps;
    CK(hipMalloc(&d_stamps, max_grid * 4 * sizeof(uint64_t)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(mcrc_dev::g_clock_stamps), &d_stamps, sizeof(d_stamps)));
    int wall_khz = 0;
    CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    std::vector<uint64_t> stamps(max_grid * 4);
#endif
    std::vector<uint32_t> img(mcrc::kImageK1Dwords);
    uint4 *d_img;
    CK(hipMalloc(&d_img, mcrc::kImageK1Dwords * 4));
    const uint32_t kfinal = ~mcrc::Gf2Op::zeros(len).apply(0xffffffffu);
    const uint32_t kspan = mcrc::xpow8n(len);
    std::vector<uint32_t> got(nitems);
    for (int rep = 0; rep < reps; ++rep)
    for (const Variant &v : vars) {
        if (only && only[0] && !strstr(v.name, only)) continue;
        uint32_t lds_bytes;
        if (v.slice == 1) {
            mcrc::build_lds_image1(img.data(), v.ch);
            lds_bytes = mcrc_dev::kLdsImage1Bytes;
        } else if (v.k1img) {
            mcrc::build_lds_image_k1(img.data(), v.ch);
            lds_bytes = mcrc_dev::kLdsImageK1Bytes;
        } else {
            mcrc::build_lds_image4(img.data(), v.ch);
            lds_bytes = mcrc_dev::kLdsImage4Bytes + v.extra_lds;
        }
        CK(hipMemcpy(d_img, img.data(), lds_bytes - v.extra_lds, hipMemcpyHostToDevice));
        CK(hipFuncSetAttribute((const void *)v.kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               lds_bytes));
        for (int pass = 0; pass < 3; ++pass) {
            const bool with_crc_in = pass == 1 || v.needs_cin;
            if (v.needs_cin && pass == 1) continue;
            const bool hot = pass == 2;  // stride 0: every item is item 0 (cache-resident)
            if (pass == 1 && (v.load_only || only_bs || reps > 1)) continue;
            if (hot && rep > 0) continue;
            const uint64_t istride = hot ? 0 : len;
            const int bs = 1024;
            const int grid = prop.multiProcessorCount * (v.slice == 1 ? 2 : 1);
            std::vector<uint32_t> cin(nitems);
            uint32_t *d_cin = nullptr;
            if (with_crc_in || v.needs_cin) {
                for (uint64_t i = 0; i < nitems; ++i) cin[i] = (uint32_t)(i * 2654435761u);
                CK(hipMalloc(&d_cin, nitems * 4));
                CK(hipMemcpy(d_cin, cin.data(), nitems * 4, hipMemcpyHostToDevice));
            }
            CK(hipMemset(d_out, 0, nitems * 4));
            v.kern<<<grid, bs, lds_bytes>>>(d_buf, istride, nitems, d_img, kfinal, kspan, d_cin, d_out);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int it = 0; it < iters; ++it)
                v.kern<<<grid, bs, lds_bytes>>>(d_buf, istride, nitems, d_img, kfinal, kspan, d_cin,
                                                d_out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= iters;
            uint64_t bad = 0;
            if (!v.load_only) {
                CK(hipMemcpy(got.data(), d_out, nitems * 4, hipMemcpyDeviceToHost));
                for (uint64_t i = 0; i < nitems; ++i) {
                    const uint32_t w = with_crc_in ? mcrc::crc32c_host_hw(cin[i], &h_buf[hot ? 0 : i * len], len)
                                       : hot         ? want[0]
                                                     : want[i];
                    bad += got[i] != w;
                }
            }
            double mhz = 0;
#ifdef MCRC_UBENCH_CLOCK
            {
                CK(hipMemcpy(stamps.data(), d_stamps, grid * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
                std::vector<double> f;
                for (int b = 0; b < grid; ++b) {
                    const double dw = (double)(stamps[4 * b + 3] - stamps[4 * b + 2]);
                    if (dw > 0) f.push_back((double)(stamps[4 * b + 1] - stamps[4 * b + 0]) / (dw / (wall_khz * 1e3)) / 1e6);
                }
                std::sort(f.begin(), f.end());
                if (!f.empty()) mhz = f[f.size() / 2];
            }
#endif
            printf("%-22s %s %8.3f ms  %8.1f GB/s  %5.1f%% of 8TB/s  bad=%llu  sclk~%.0f MHz\n", v.name,
                   hot ? "hot   " : with_crc_in ? "crc_in" : "      ", ms, bytes / ms / 1e6,
                   bytes / ms / 1e6 / 8000 * 100, (unsigned long long)bad, mhz);
            if (d_cin) CK(hipFree(d_cin));
        }
    }
    return 0;
}
