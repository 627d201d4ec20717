// fetch_calib.hip -- dev experiment (not part of the library): what does
// rocprofv3's FETCH_SIZE count for k_count's access pattern?
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE for wide coalesced streaming
// reads only (it reports half their bytes).  k_count reads, per item, a few
// 16-B pieces scattered one or two per 128-B line.  Three kernels over a
// 2 GiB buffer (far past the 256 MiB Infinity Cache), each touching a known
// set of distinct lines once:
//   K0 stream    every lane reads 16 contiguous bytes: all lines, whole
//   K1 one16     one 16-B piece in each of N random distinct lines
//   K2 two16     two 16-B pieces (bytes 0-15 and 64-79) of each of N lines
// Run each under rocprofv3 --pmc FETCH_SIZE and compare FETCH_SIZE * 1024
// with the lines touched * 128 B (tools/fetch_calib.sh).
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o /tmp/fetch_calib
//   /tmp/fetch_calib MODE
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

__global__ void k_stream(const uint4 *buf, uint64_t n16, unsigned *sink) {
    uint32_t x = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) atomicAdd(sink, 1u);
}

template <int PIECES>
__global__ void k_scatter(const uint8_t *buf, const uint32_t *lines, uint64_t n, unsigned *sink) {
    uint32_t x = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *l = buf + (uint64_t)lines[i] * 128;
        const uint4 a = *reinterpret_cast<const uint4 *>(l);
        x ^= a.x ^ a.w;
        if (PIECES == 2) {
            const uint4 b = *reinterpret_cast<const uint4 *>(l + 64);
            x ^= b.y ^ b.z;
        }
    }
    if (x == 0x9e3779b9u) atomicAdd(sink, 1u);
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const uint64_t bytes = 2ull << 30, nlines_all = bytes / 128;
    const uint64_t n = 4u << 20;  // lines touched by the scatter kernels (512 MiB of lines)
    uint8_t *buf = nullptr;
    uint32_t *lines = nullptr;
    unsigned *sink = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0x5a, bytes));
    CHECK(hipMalloc(&sink, 4));
    // N distinct lines in random order: a multiplicative permutation of the
    // line indices (odd multiplier modulo a power of two is a bijection)
    std::vector<uint32_t> h(n);
    for (uint64_t i = 0; i < n; ++i) h[i] = (uint32_t)((i * 2654435761ull + 12345) & (nlines_all - 1));
    CHECK(hipMalloc(&lines, n * 4));
    CHECK(hipMemcpy(lines, h.data(), n * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0)
            hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const uint4 *)buf, bytes / 16, sink);
        else if (mode == 1)
            hipLaunchKernelGGL(k_scatter<1>, dim3(4096), dim3(256), 0, 0, buf, lines, n, sink);
        else
            hipLaunchKernelGGL(k_scatter<2>, dim3(4096), dim3(256), 0, 0, buf, lines, n, sink);
        CHECK(hipDeviceSynchronize());
    }
    const uint64_t line_bytes = mode == 0 ? bytes : n * 128;
    printf("mode %d: lines touched %llu (%llu bytes of whole lines), requested %llu bytes per dispatch\n", mode,
           (unsigned long long)(line_bytes / 128), (unsigned long long)line_bytes,
           (unsigned long long)(mode == 0 ? bytes : n * 16 * (mode == 2 ? 2 : 1)));
    CHECK(hipFree(buf));
    CHECK(hipFree(lines));
    CHECK(hipFree(sink));
    return 0;
}
