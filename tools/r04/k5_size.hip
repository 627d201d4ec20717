// k5_size.hip -- dev experiment (not part of the library): does K5 (k_items,
// MODE 0: equal 4133-B spans at stride 4165) have a fixed cost per launch?
// Times k_items<0, false> alone (events, medians of REPS) at 1, 2 and 4 Mi
// spans, alternating, next to K1 at the same sizes; T(n) = a + b n.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/k5_size.hip -o tools/k5_size
//   ./tools/k5_size [REPS]
#include <stdio.h>
#include <stdlib.h>

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

__global__ void k_fill(uint32_t *p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull;
        z = (z ^ (z >> 31)) * 0xbf58476d1ce4e5b9ull;
        p[i] = (uint32_t)(z ^ (z >> 29));
    }
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t maxn = 4ull << 20, stride = 4165, len = 4133;
    const uint64_t bytes = maxn * stride + 64;
    uint8_t *base;
    uint32_t *out;
    uint2 *rt;
    uint4 *img, *img_k1, *zero;
    CHECK(hipMalloc(&base, bytes));
    CHECK(hipMalloc(&out, maxn * 4));
    CHECK(hipMalloc(&rt, maxn * 8));
    CHECK(hipMalloc(&img, kLdsImageK1Bytes));
    CHECK(hipMalloc(&img_k1, kLdsImageK1Bytes));
    CHECK(hipMalloc(&zero, kZeroBytes));
    CHECK(hipMemset(zero, 0, kZeroBytes));
    std::vector<uint32_t> h(kLdsImageK1Bytes / 4);
    mcrc::build_lds_image_span(h.data(), kSpanCH);
    CHECK(hipMemcpy(img, h.data(), kLdsImageK1Bytes, hipMemcpyHostToDevice));
    mcrc::build_lds_image_k1(h.data(), kK1CH);
    CHECK(hipMemcpy(img_k1, h.data(), kLdsImageK1Bytes, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)base, bytes / 4);
    CHECK(hipFuncSetAttribute((const void *)k_items<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kLdsImageK1Bytes));
    CHECK(hipFuncSetAttribute((const void *)k_fixed<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kLdsImageK1Bytes));
    CHECK(hipDeviceSynchronize());
    auto k5 = [&](uint64_t n) {
        SpanArgs a{};
        a.base = base + 32;
        a.base_bytes = bytes - 32;
        a.stride = stride;
        a.len = (uint32_t)len;
        a.n = n;
        a.zero = zero;
        ItemsOut io{};
        io.rt = rt;
        hipLaunchKernelGGL((k_items<0, false>), dim3(std::min<uint64_t>(cus, (n + 31) / 32)), dim3(1024),
                           kLdsImageK1Bytes, 0, a, img, io);
    };
    auto k1 = [&](uint64_t n) {
        hipLaunchKernelGGL(k_fixed<false>, dim3(cus), dim3(1024), kLdsImageK1Bytes, 0, base, 4096ull, n, img_k1,
                           (const uint32_t *)nullptr, out);
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 300; ++i) k1(1ull << 20);
    CHECK(hipDeviceSynchronize());
    for (int round = 0; round < 3; ++round)
        for (int which = 0; which < 2; ++which) {
            double t[3];
            int j = 0;
            for (uint64_t n : {1ull << 20, 2ull << 20, 4ull << 20}) {
                std::vector<double> ms;
                for (int r = 0; r < reps; ++r) {
                    CHECK(hipEventRecord(e0));
                    if (which) k1(n); else k5(n);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float x;
                    CHECK(hipEventElapsedTime(&x, e0, e1));
                    ms.push_back(x);
                }
                t[j++] = med(ms);
            }
            const double b = (t[2] - t[0]) / 3.0, a0 = t[0] - b;
            const double per = which ? 4096.0 : (double)len;
            printf("round %d %s: 1/2/4 Mi %.4f %.4f %.4f ms; fit a = %.1f us, b = %.4f ms per Mi (%.1f %% of 8 TB/s)\n",
                   round, which ? "K1 k_fixed      " : "K5 k_items<0>   ", t[0], t[1], t[2], a0 * 1e3, b,
                   100.0 * per * (1 << 20) / (b * 1e-3) / 8e12);
            fflush(stdout);
        }
    return 0;
}
