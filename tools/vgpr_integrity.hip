// vgpr_integrity.hip -- does a wave's register file hold what it wrote when
// the wave is allocated 24 VGPRs and shares its SIMD with waves of other
// workgroups?  (The walk miscompute of DESIGN.md §3.7 / tools/walk_vgpr_repro:
// exact at a 32-VGPR allocation and at one workgroup per CU, wrong at 24 with
// co-resident workgroups, the header bytes a lane parsed not the bytes in
// memory.)  Not part of the library.
//
// Each iteration of each lane, in one asm statement (so the registers are the
// ones named):
//   * v16..v19 <- lane- and wave-unique patterns;
//   * a 16-B global load of a known element into v20..v23, a wait for it, a
//     short sleep;
//   * v16..v19 compared with the patterns, v20..v23 with the element.
// Every other register is the compiler's (v0..v15).  Variants:
//   A24   the allocation is 24 VGPRs (v16..v23 the top granule);
//   A32   the same with v31 clobbered: a 32-VGPR allocation, same code;
//   A24/1 A24 with 100 KiB of unused dynamic LDS (one workgroup per CU);
//   S24, S32, S24/1  the same for k_shift (the parse's 64-bit funnel shift).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/vgpr_integrity.hip -o /tmp/vgpr_integrity
//   /tmp/vgpr_integrity ITERS REPS
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint4 elem(uint32_t k) { return make_uint4(k, k ^ 0x5a5a5a5au, k * 3u, ~k); }

__global__ void k_fill(uint4 *src, uint64_t n) {
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x)
        src[k] = elem((uint32_t)k);
}

// bad[0]: lanes whose v16..v19 changed; bad[1]: loads whose v20..v23 were not the element
template <int TOP>
__global__ __launch_bounds__(256) void k_regs(const uint4 *src, uint64_t n, uint32_t iters, unsigned long long *bad) {
    if (TOP == 32) asm volatile("" ::: "v31");
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t gw = blockIdx.x * 4ull + (threadIdx.x >> 6);
    const uint32_t pa = (uint32_t)(gw << 6 | lane), pb = ~pa * 0x9e3779b1u;
    uint32_t nidle = 0, nload = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const uint32_t k = ((uint32_t)(gw * 64 + lane) * 7919u + i * 1000003u) & (uint32_t)(n - 1);
        const uint4 *p = src + k;
        uint32_t d, x, y, z, w;
        asm volatile(
            "v_mov_b32 v16, %5\n\t"
            "v_mov_b32 v17, %6\n\t"
            "v_mov_b32 v18, %6\n\t"
            "v_mov_b32 v19, %5\n\t"
            "global_load_dwordx4 v[20:23], %7, off\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            "s_sleep 1\n\t"
            "v_xor_b32 %0, v16, %5\n\t"
            "v_xor_b32 %1, v17, %6\n\t"
            "v_or_b32 %0, %0, %1\n\t"
            "v_xor_b32 %1, v18, %6\n\t"
            "v_or_b32 %0, %0, %1\n\t"
            "v_xor_b32 %1, v19, %5\n\t"
            "v_or_b32 %0, %0, %1\n\t"
            "v_mov_b32 %1, v20\n\t"
            "v_mov_b32 %2, v21\n\t"
            "v_mov_b32 %3, v22\n\t"
            "v_mov_b32 %4, v23"
            : "=&v"(d), "=&v"(x), "=&v"(y), "=&v"(z), "=&v"(w)
            : "v"(pa), "v"(pb), "v"(p)
            : "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "memory");
        const uint4 e = elem(k);
        nidle += d != 0u;
        nload += (x != e.x) | (y != e.y) | (z != e.z) | (w != e.w);
    }
    if (nidle) atomicAdd(&bad[0], (unsigned long long)nidle);
    if (nload) atomicAdd(&bad[1], (unsigned long long)nload);
}

// The walk's parse failed only where it funnel-shifts (64-bit v_lshrrev_b64 /
// v_lshlrev_b64 by k and 64 - k, k != 0; tools/walk_vgpr_repro PS24).  The
// same two shifts in the top granule: the element loaded into v[20:23], then
// v[16:17] = v[20:21] >> k | v[22:23] << (64 - k), compared with the host's
// arithmetic; bad[1] counts the wrong results.
template <int TOP>
__global__ __launch_bounds__(256) void k_shift(const uint4 *src, uint64_t n, uint32_t iters, unsigned long long *bad) {
    if (TOP == 32) asm volatile("" ::: "v31");
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t gw = blockIdx.x * 4ull + (threadIdx.x >> 6);
    const uint32_t k = 8u * (1u + (lane % 7u)), kc = 64u - k;  // 8 .. 56
    uint32_t nwrong = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const uint32_t e = ((uint32_t)(gw * 64 + lane) * 7919u + i * 1000003u) & (uint32_t)(n - 1);
        const uint4 *p = src + e;
        uint32_t lo, hi;
        asm volatile(
            "global_load_dwordx4 v[20:23], %2, off\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            "v_lshrrev_b64 v[16:17], %3, v[20:21]\n\t"
            "v_lshlrev_b64 v[18:19], %4, v[22:23]\n\t"
            "v_or_b32 %0, v16, v18\n\t"
            "v_or_b32 %1, v17, v19"
            : "=&v"(lo), "=&v"(hi)
            : "v"(p), "v"(k), "v"(kc)
            : "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "memory");
        const uint4 x = elem(e);
        const uint64_t a0 = (uint64_t)x.y << 32 | x.x, a1 = (uint64_t)x.w << 32 | x.z;
        const uint64_t want = (a0 >> k) | (a1 << kc);
        nwrong += (lo != (uint32_t)want) | (hi != (uint32_t)(want >> 32));
    }
    if (nwrong) atomicAdd(&bad[1], (unsigned long long)nwrong);
}

int main(int argc, char **argv) {
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const int reps = argc > 2 ? atoi(argv[2]) : 2;
    const uint64_t n = 64ull << 20;  // 1 GiB of 16-B elements (a power of two: k_regs masks)
    uint4 *src = nullptr;
    unsigned long long *bad = nullptr;
    CHECK(hipMalloc(&src, n * 16));
    CHECK(hipMalloc(&bad, 16));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, src, n);
    CHECK(hipDeviceSynchronize());
    CHECK(hipFuncSetAttribute((const void *)k_regs<24>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10));
    CHECK(hipFuncSetAttribute((const void *)k_shift<24>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10));
    const uint32_t nblk = 2048;  // 8 workgroups (32 waves) per CU when they fit
    for (int r = 0; r < reps; ++r) {
        for (int v = 0; v < 6; ++v) {
            CHECK(hipMemset(bad, 0, 16));
            if (v == 0) hipLaunchKernelGGL(k_regs<24>, dim3(nblk), dim3(256), 0, 0, src, n, iters, bad);
            if (v == 1) hipLaunchKernelGGL(k_regs<32>, dim3(nblk), dim3(256), 0, 0, src, n, iters, bad);
            if (v == 2) hipLaunchKernelGGL(k_regs<24>, dim3(nblk), dim3(256), 100 << 10, 0, src, n, iters, bad);
            if (v == 3) hipLaunchKernelGGL(k_shift<24>, dim3(nblk), dim3(256), 0, 0, src, n, iters, bad);
            if (v == 4) hipLaunchKernelGGL(k_shift<32>, dim3(nblk), dim3(256), 0, 0, src, n, iters, bad);
            if (v == 5) hipLaunchKernelGGL(k_shift<24>, dim3(nblk), dim3(256), 100 << 10, 0, src, n, iters, bad);
            CHECK(hipDeviceSynchronize());
            unsigned long long hb[2];
            CHECK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
            static const char *names[] = {"A24", "A32", "A24/1 (one workgroup per CU)", "S24", "S32",
                                          "S24/1 (one workgroup per CU)"};
            if (v < 3)
                printf("%s: lane-iterations %llu, v16..v19 changed %llu, v20..v23 not the loaded element %llu\n",
                       names[v], (unsigned long long)nblk * 256 * iters, hb[0], hb[1]);
            else
                printf("%s: lane-iterations %llu, funnel shifts wrong %llu\n", names[v],
                       (unsigned long long)nblk * 256 * iters, hb[1]);
            fflush(stdout);
        }
    }
    CHECK(hipFree(src));
    CHECK(hipFree(bad));
    return 0;
}
