// crc32c_device.h -- CDNA4 (gfx950) device primitives for batched CRC-32C.
//
// Work model.  A 32-lane group owns one item span (a wavefront holds two).
// The span is cut into 4 KiB blocks; lane i of the group holds the 16-B
// pieces at 512 k + 16 i of a block (k = 0..7: each load instruction reads
// 512 contiguous bytes per group) and runs one table-driven chain per piece.
// The chains of each 2 KiB half fold through shifted last-step tables, the
// first half moves up by M_2048, and the lane values of a group merge in a
// 5-level reduction whose level k applies the fixed zeros operator
// M_{16 * 2^k}.  This is the algebra the reference uses to merge its three
// crc32q streams (crc32c.c:184-220, zeros operators crc32c.c:85-137), widened
// from 3 streams to 256 per 4 KiB.
//
// Tables live in LDS.  The slice-by-4 tables are replicated once per bank of a
// 32-lane bank group so every data lookup is conflict-free (lane l always
// reads bank l % 32); the 160 KiB image (crc32c_gf2.h build_lds_image_span at
// chunk 16, one image for every kernel since round 5):
//   [0, 28 KiB)          aux tables, plain: table t entry e at t*1024 + e*4
//   [28 KiB, +64 KiB)    row e: T3[e] x 32 | T2[e] x 32
//   [92 KiB, +64 KiB)    row e: T1[e] x 32 | T0[e] x 32
//   [156 KiB, 160 KiB)   four more aux tables (the M_1536 shifted last step)
// where Tk[b] = register after byte b then k zero bytes (crc32c.c:366-389).
//
// Aux tables hold the byte slices of zeros operators (crc32c.c:121-137 form);
// operator o occupies aux tables 4o..4o+3:
//   o = 0..3 : M_{16 * 2^o}  (lane-group reduction level o; level 4 = level 3 twice)
//   o = 4    : M_2048, the half-block fold (kAuxSpanFold)
//   o = 5, 6 : the shifted last steps M_512, M_1024 (tables 156..159: M_1536)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcrc_dev {

constexpr uint32_t kAuxTree = 0;
constexpr uint32_t kAux4Bytes = 28 * 1024;  // 28 KiB of plain aux tables

constexpr uint32_t kPoly = 0x82f63b78u;

// The kernels declare no static LDS, so dynamic LDS starts at address 0 and a
// byte offset is an LDS address (saves the base add hipcc emits for
// `smem + off`).
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;

__device__ __forceinline__ uint32_t lds_ld(uint32_t byte_addr) {
    return *reinterpret_cast<lds_cu32 *>(static_cast<uintptr_t>(byte_addr));
}

// VGPR allocation floor.  The walk experiment (tools/walk_hazard.hip,
// DESIGN.md section 3) found a kernel whose identical instruction stream walks
// wrongly when allocated 24 VGPRs with several workgroups per CU and exactly
// at 32, 40 and 48 (and at 24 with one workgroup per CU).  Every kernel that
// runs several workgroups per CU therefore allocates at least 32 VGPRs; on
// gfx950 that costs no occupancy (8 waves per SIMD up to 64 VGPRs).
// tests/test_kernel_resources.py checks the built code object.
#define MCRC_VGPR_FLOOR() asm volatile("" ::: "v31")

// Per-lane constants for table addressing.
struct LaneCtx {
    uint32_t lane4;    // (lane & 31) << 2
    uint32_t lane4hi;  // lane4 | 0x10000 (selects the second 64 KiB table set)
};

template <int SLICE>
struct Step;

// Slice-by-4 aux tables (plain, not replicated).
template <>
struct Step<4> {
    __device__ __forceinline__ static uint32_t aux(uint32_t t, uint32_t e) {
        return lds_ld((t << 10) | (e << 2));
    }
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Slice-by-4 step fused with the next data dword: returns
//   T3[x0] ^ T2[x1] ^ T1[x2] ^ T0[x3] ^ w_next
// with two v_bitop3 (3-input XOR) instead of four v_xor.
__device__ __forceinline__ uint32_t step4_next(uint32_t x, uint32_t w_next, const LaneCtx &c) {
    const uint32_t a3 = lds_ld(__builtin_amdgcn_perm(x, c.lane4, 0x0c0c0400u) + kAux4Bytes);
    const uint32_t a2 = lds_ld(__builtin_amdgcn_perm(x, c.lane4, 0x0c0c0500u) + kAux4Bytes + 128u);
    const uint32_t a1 = lds_ld(__builtin_amdgcn_perm(x, c.lane4hi, 0x0c020600u) + kAux4Bytes);
    const uint32_t a0 = lds_ld(__builtin_amdgcn_perm(x, c.lane4hi, 0x0c020700u) + kAux4Bytes + 128u);
    return xor3(xor3(a3, a2, a1), a0, w_next);
}

// Shifted last-step tables (crc32c_gf2.h build_lds_image_k1 at chunk 16):
// pieces 0, 1, 2 of each half with their fold M_{(3-k)*512} applied (4 plain
// tables each).
constexpr uint32_t kAuxShift0 = 156, kAuxShift1 = 24, kAuxShift2 = 20;
constexpr uint32_t kLdsImageK1Bytes = 160 * 1024;

// Last slice-by-4 step of a row chain through the shifted tables t0..t0+3:
// returns M_shift(T3[x0] ^ T2[x1] ^ T1[x2] ^ T0[x3]).
__device__ __forceinline__ uint32_t step4_last_shifted(uint32_t x, uint32_t t0) {
    return xor3(Step<4>::aux(t0, x & 0xffu), Step<4>::aux(t0 + 1, (x >> 8) & 0xffu),
                Step<4>::aux(t0 + 2, (x >> 16) & 0xffu)) ^
           Step<4>::aux(t0 + 3, x >> 24);
}

// Apply the zeros operator stored in aux tables t0..t0+3.
template <int SLICE>
__device__ __forceinline__ uint32_t apply_op(uint32_t t0, uint32_t v) {
    return Step<SLICE>::aux(t0, v & 0xffu) ^ Step<SLICE>::aux(t0 + 1, (v >> 8) & 0xffu) ^
           Step<SLICE>::aux(t0 + 2, (v >> 16) & 0xffu) ^ Step<SLICE>::aux(t0 + 3, v >> 24);
}

// Value of lane (l + 2^k) for lanes whose partner stays inside a 32-lane
// group: DPP row shifts for k <= 3, v_permlane16_swap for k = 4.  No LDS.
template <int K>
__device__ __forceinline__ uint32_t lane_down(uint32_t v) {
    if constexpr (K < 4) {
        return __builtin_amdgcn_update_dpp(0u, v, 0x100 | (1 << K), 0xf, 0xf, false);  // row_shl:2^K
    } else {
        static_assert(K == 4, "groups are 32 lanes");
        return __builtin_amdgcn_permlane16_swap(v, v, false, false)[1];  // row r gets row r^1
    }
}

// One level of the LPI = 32 reduction on the lanes selected by `on`.
template <int K>
__device__ __forceinline__ uint32_t reduce_level(uint32_t v, bool on) {
    const uint32_t x = lane_down<K>(v);
    if (on) v = xor3(Step<4>::aux(kAuxTree + 4 * K, v & 0xffu) ^ x, Step<4>::aux(kAuxTree + 4 * K + 1, (v >> 8) & 0xffu),
                     Step<4>::aux(kAuxTree + 4 * K + 2, (v >> 16) & 0xffu)) ^
                Step<4>::aux(kAuxTree + 4 * K + 3, v >> 24);
    return v;
}

// Level 1 of two items' reductions (A on lanes 0 mod 4, B on lanes 1 mod 4
// afterwards), for group_reduce32_quad.
__device__ __forceinline__ uint32_t group_pair_level1(uint32_t a, uint32_t b, uint32_t lane) {
    const uint32_t bs = __builtin_amdgcn_update_dpp(0u, b, 0x111, 0xf, 0xf, false);  // row_shr:1
    return reduce_level<1>((lane & 1u) ? bs : a, (lane & 3u) < 2u);
}

// Aux tables 16..19 hold the half-block fold M_2048 (build_lds_image_span at
// chunk 16: M_{128 chunk}) instead of tree level 4.
constexpr uint32_t kAuxSpanFold = 16;

// The full five-level reduction of a group's lane values into lane 0: level
// 4 (M_256) is level 3 (M_128) applied twice.
__device__ __forceinline__ uint32_t group_reduce32_span(uint32_t v, uint32_t lane) {
    v = reduce_level<0>(v, (lane & 1u) == 0u);
    v = reduce_level<1>(v, (lane & 3u) == 0u);
    v = reduce_level<2>(v, (lane & 7u) == 0u);
    v = reduce_level<3>(v, (lane & 15u) == 0u);
    const uint32_t x = lane_down<4>(v);
    if ((lane & 31u) == 0u) v = apply_op<4>(kAuxTree + 12, apply_op<4>(kAuxTree + 12, v)) ^ x;
    return v;
}

// Level 4 as level 3 twice (tables 16..19 hold the half-block fold), and the
// pair / quad reductions of two or four items per group.
__device__ __forceinline__ uint32_t reduce_level4_span(uint32_t v, bool on) {
    const uint32_t x = lane_down<4>(v);
    if (on) v = apply_op<4>(kAuxTree + 12, apply_op<4>(kAuxTree + 12, v)) ^ x;
    return v;
}

__device__ __forceinline__ uint32_t group_reduce32_pair_span(uint32_t a, uint32_t b, uint32_t lane) {
    const uint32_t bs = __builtin_amdgcn_update_dpp(0u, b, 0x111, 0xf, 0xf, false);  // row_shr:1
    uint32_t v = (lane & 1u) ? bs : a;
    v = reduce_level<1>(v, (lane & 3u) < 2u);
    v = reduce_level<2>(v, (lane & 7u) < 2u);
    v = reduce_level<3>(v, (lane & 15u) < 2u);
    return reduce_level4_span(v, (lane & 31u) < 2u);
}

__device__ __forceinline__ uint32_t group_reduce32_quad_span(uint32_t ab, uint32_t cd, uint32_t lane) {
    const uint32_t cs = __builtin_amdgcn_update_dpp(0u, cd, 0x112, 0xf, 0xf, false);  // row_shr:2
    uint32_t v = (lane & 2u) ? cs : ab;
    v = reduce_level<2>(v, (lane & 7u) < 4u);
    v = reduce_level<3>(v, (lane & 15u) < 4u);
    return reduce_level4_span(v, (lane & 31u) < 4u);
}

// Copy a table image from global memory into this workgroup's LDS.
// (A thread's loads are all issued before its LDS stores: one load, wait and
// store per iteration made the 160 KiB copy ten dependent L2 round trips per
// workgroup.)
__device__ __forceinline__ void load_tables(char *lds, const uint4 *__restrict__ img, uint32_t bytes) {
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    const uint32_t n = bytes / 16;
    constexpr uint32_t U = 10;  // 160 KiB / (1024 threads x 16 B)
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += U * blockDim.x) {
        uint4 v[U];
        // (indices clamped, not predicated: under a branch each load would be
        // sunk to its store and waited for at once; a clamped thread rewrites
        // the last entry with its own value)
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = img[min(i0 + u * blockDim.x, n - 1)];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) dst[min(i0 + u * blockDim.x, n - 1)] = v[u];
    }
    __syncthreads();
}

// Reflected polynomial product mod P (device twin of mcrc::mulmodp).
__device__ __forceinline__ uint32_t mulmodp_dev(uint32_t a, uint32_t b) {
    uint32_t prod = 0;
#pragma unroll 4
    for (int i = 31; i >= 0; --i) {
        prod ^= ((a >> i) & 1u) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
    }
    return prod;
}

}  // namespace mcrc_dev
