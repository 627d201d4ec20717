// walk_hazard.hip -- dev experiment (not part of the library): why did the
// SGPR/readlane form of the device page walk (round 2, commit 30e3f9d) count
// large page sets wrongly and differently on each run?
//
// Count-pass variants of k_walk over the bench's config-5 page layout (4 MiB
// wbufs of 1007 packed 4165-B images, zero tail, a few corrupt headers), each
// run REPS times; every run's per-wbuf counts are compared with a host walk of
// the same headers.
//   V0  the shipped form: walk state in VGPRs, lane m broadcast by ds_bpermute
//   V1  the round-2 failing form: lane m's flag and size read with v_readlane
//       into SGPRs (wave-uniform scalar walk state)
//   V2  V1 with 5 wait states (s_nop 4) between the ballot's VCC write and its
//       SALU reads (s_ff1)
//   V3  V1 with 5 wait states after each v_readlane before the SGPR is read
//   V4  V1 with 5 wait states before each v_readlane (after the SALU write of
//       its lane-select SGPR)
//   V5  V1 with each v_readlane and 5 wait states after it in one asm
//       statement (no SALU or VALU read of its SGPR within 5 states)
//   V6  V5 with 5 more wait states before each v_readlane
//   V7  V1 recording, per wbuf, its first four round trips (off, s, m, k,
//       lane 0's header fields) for the post-mortem of a wrong wbuf
//   V9, V10, V11  V1 with its VGPR allocation raised from 24 to 32, 40 and 48
//       (an asm clobber of v31 / v39 / v47; the code is V1's)
//   V8  V1 with the lane's header offset in 32-bit arithmetic (off + j * s
//       < 4 GiB in a wbuf): no v_mad_u64_u32, whose carry-out SGPR pair the
//       compiler reuses 5 instructions later for an s_cselect in V1-V7
//
//   V1 at 1 and 2 workgroups per CU (dynamic LDS of 100 and 64 KiB, nothing
//   else changed): whether the failures need waves of several workgroups
//   sharing a SIMD
//
// k_rl: the walk's shape with nothing else -- a loop-carried wave-uniform
// value (acc) that picks the next load address, takes lane m's loaded word
// by v_readlane (SGPR, MODE 0) or by a ds_bpermute broadcast (VGPR, MODE 1),
// and is updated by scalar (MODE 0) or vector (MODE 1) arithmetic; every wave
// computes the same chain, checked against the host
//
// and a register-level test of that pattern (k_waw): v_mad_u64_u32 with its
// carry-out in an SGPR pair, three VALU instructions, then an SALU write
// (s_cselect_b64 -1) of the same pair, which must read back -1; P = the
// number of s_nop 7 between them (0: the sequence of V1-V7)
//
//   bash tools/walk_hazard.sh OUT  (or: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_hazard.hip -o /tmp/walk_hazard)
//   /tmp/walk_hazard PAGES REPS
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "crc32c_kernels.hip"

using namespace mcrc_dev;

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

__device__ uint32_t *g_trace;  // V7: [wbuf][round 0..3][8 dwords]

template <int V>
__global__ __launch_bounds__(64 * kWalkWaves) void k_count_v(SpanArgs a, uint64_t nw, uint32_t *cnt) {
    // V9-V11: V1 with its VGPR allocation raised from 24 to 32 / 40 / 48
    // (a clobber of the top register; nothing else changes)
    if (V == 9) asm volatile("" ::: "v31");
    if (V == 10) asm volatile("" ::: "v39");
    if (V == 11) asm volatile("" ::: "v47");
    const uint32_t j = threadIdx.x & 63u;
    const uint64_t wbuf = a.region;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t w = (uint64_t)blockIdx.x * kWalkWaves + wave; w < nw; w += (uint64_t)gridDim.x * kWalkWaves) {
        const uint64_t start = w * wbuf, size = a.base_bytes - start < wbuf ? a.base_bytes - start : wbuf;
        const uint8_t *wb = a.base + start;
        uint64_t off = 0, s = 0;
        uint32_t c = 0, round = 0;
        while (off + 48 <= size) {
            const uint64_t o = off + j * s;
            const bool in = (j == 0 || s != 0) && o + 48 <= size;
            ItemHdr h{0u, 0u, 0u, 0u};
            if (in) h = parse_hdr(wb + o);
            const uint64_t nt = h.ntotal(4);
            const bool item = in && h.nkey != 0;
            uint64_t brk = __ballot(!(item && nt == s));
            if (V == 2) asm volatile("s_nop 4" : "+s"(brk));
            const uint32_t m = brk ? (uint32_t)__ffsll((unsigned long long)brk) - 1u : 64u;
            bool last_item = false;
            uint64_t nt_m = 0;
            if (V == 0) {
                const int src = m < 64u ? (int)m : 0;
                last_item = m < 64u && __shfl((int)item, src, 64) != 0;
                nt_m = (uint64_t)(uint32_t)__shfl((int)(uint32_t)nt, src, 64) |
                       ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(nt >> 32), src, 64) << 32);
            } else if (V >= 5 && V <= 7 && m < 64u) {
                int li, lo, hi;
                const int iv = (int)item, lov = (int)(uint32_t)nt, hiv = (int)(uint32_t)(nt >> 32);
                if (V == 5) {
                    asm volatile("v_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(li) : "v"(iv), "s"(m));
                    asm volatile("v_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(lo) : "v"(lov), "s"(m));
                    asm volatile("v_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(hi) : "v"(hiv), "s"(m));
                } else {
                    asm volatile("s_nop 4\n\tv_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(li) : "v"(iv), "s"(m));
                    asm volatile("s_nop 4\n\tv_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(lo) : "v"(lov), "s"(m));
                    asm volatile("s_nop 4\n\tv_readlane_b32 %0, %1, %2\n\ts_nop 4" : "=s"(hi) : "v"(hiv), "s"(m));
                }
                last_item = li != 0;
                nt_m = (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
            } else if (m < 64u) {
                int mm = (int)m;
                if (V == 4) asm volatile("s_nop 4" : "+s"(mm));
                int li = __builtin_amdgcn_readlane((int)item, mm);
                int lo = __builtin_amdgcn_readlane((int)(uint32_t)nt, mm);
                int hi = __builtin_amdgcn_readlane((int)(uint32_t)(nt >> 32), mm);
                if (V == 3) asm volatile("s_nop 4" : "+s"(li), "+s"(lo), "+s"(hi));
                last_item = li != 0;
                nt_m = (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
            }
            const uint32_t k = m < 64u ? m + (last_item ? 1u : 0u) : 64u;
            if (V == 7 && round < 4) {
                uint32_t *t = g_trace + (w * 4 + round) * 8;
                const uint32_t l0nb = __shfl(h.nbytes, 0, 64), l0nk = __shfl(h.nkey, 0, 64);
                const uint32_t l0nt = (uint32_t)__shfl((int)(uint32_t)nt, 0, 64);
                if (j == 0) {
                    t[0] = (uint32_t)off;
                    t[1] = (uint32_t)s;
                    t[2] = m | (last_item ? 0x100u : 0u) | (k << 16);
                    t[3] = (uint32_t)nt_m;
                    t[4] = (uint32_t)brk;
                    t[5] = (uint32_t)(brk >> 32);
                    t[6] = l0nb | (l0nk << 24);
                    t[7] = l0nt;
                }
            }
            ++round;
            c += k;
            if (m == 64u) {
                off += 64u * s;
            } else if (!last_item) {
                break;
            } else {
                off += m * s + nt_m;
                s = nt_m;
            }
        }
        if (j == 0) cnt[w] = c;
    }
}

// config-5 layout: item i of wbuf w at w * wbuf + i * 4165; header fields as
// bench.py workload_config5; `bad` items get a flipped bit in nbytes / nkey.
__global__ void k_fill(uint8_t *base, uint64_t nwb, uint64_t wbuf, uint32_t seed) {
    const uint64_t n = nwb * 1007;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t *it = base + (i / 1007) * wbuf + (i % 1007) * 4165;
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15;
        x *= 0x2c1b3c6du;
        x ^= x >> 12;
        uint32_t nbytes = 4098;
        uint8_t nkey = 10;
        if (x % 3000 == 7) nbytes ^= 1u << (x >> 20) % 20;  // a corrupt length
        if (x % 7000 == 11) nkey = 0;                       // a zeroed key length
        memcpy(it + 32, &nbytes, 4);
        it[36] = 1;
        it[37] = 0;
        it[38] = 2;  // ITEM_CAS
        it[39] = 0;
        it[40] = 17;
        it[41] = nkey;
    }
}

template <int P>
__global__ __launch_bounds__(256) void k_waw(unsigned long long *bad, uint32_t iters, uint32_t s_lo, uint32_t s_hi,
                                             uint64_t sv) {
    const uint32_t j = threadIdx.x & 63u;
    uint64_t acc = (uint64_t)blockIdx.x << 20;
    uint32_t nb = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        uint64_t flag;
        uint32_t t0, t1;
        if (P == 0)
            asm volatile(
                "v_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
                "v_mul_lo_u32 %2, %4, 0\n\t"
                "v_mul_lo_u32 %3, %6, %5\n\t"
                "v_add_u32 %3, %3, %2\n\t"
                "s_cmp_lg_u64 %7, 0\n\t"
                "s_cselect_b64 %1, -1, 0"
                : "+v"(acc), "=&s"(flag), "=&v"(t0), "=&v"(t1)
                : "s"(s_lo), "v"(j), "s"(s_hi), "s"(sv)
                : "scc");
        else
            asm volatile(
                "v_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
                "v_mul_lo_u32 %2, %4, 0\n\t"
                "v_mul_lo_u32 %3, %6, %5\n\t"
                "v_add_u32 %3, %3, %2\n\t"
                "s_nop 7\n\ts_nop 7\n\t"
                "s_cmp_lg_u64 %7, 0\n\t"
                "s_cselect_b64 %1, -1, 0"
                : "+v"(acc), "=&s"(flag), "=&v"(t0), "=&v"(t1)
                : "s"(s_lo), "v"(j), "s"(s_hi), "s"(sv)
                : "scc");
        nb += flag != ~0ull;
        acc += t1 & 1u;
    }
    if (j == 0 && nb) atomicAdd(bad, (unsigned long long)nb);
    if (acc == 0x123456789ull) atomicAdd(bad, 1ull << 40);  // (keeps acc live)
}

template <int MODE, int CLOB = 0>
__global__ __launch_bounds__(256) void k_rl(const uint32_t *tab, uint32_t iters, uint32_t *out) {
    // CLOB: the VGPR allocation raised to 16 / 24 / 32 (a clobber of the top register)
    if (CLOB == 16) asm volatile("" ::: "v15");
    if (CLOB == 24) asm volatile("" ::: "v23");
    if (CLOB == 32) asm volatile("" ::: "v31");
    const uint32_t j = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const uint32_t x = tab[(acc + j) & 4095u];
        const uint32_t m = (acc >> 7) & 63u;
        uint32_t r;
        if (MODE == 0)
            r = __builtin_amdgcn_readlane(x, __builtin_amdgcn_readfirstlane(m));
        else
            r = (uint32_t)__shfl((int)x, (int)m, 64);
        acc = acc * 2654435761u + r + i;
    }
    if (j == 0) out[wave] = acc;
}

static uint32_t host_rl(const std::vector<uint32_t> &tab, uint32_t iters) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const uint32_t m = (acc >> 7) & 63u;
        const uint32_t r = tab[(acc + m) & 4095u];
        acc = acc * 2654435761u + r + i;
    }
    return acc;
}

static uint32_t host_walk(const uint8_t *h, uint64_t size) {
    uint64_t off = 0;
    uint32_t c = 0;
    while (off + 48 <= size) {
        const uint8_t *it = h + off;
        if (it[41] == 0) break;
        uint32_t nbytes;
        uint16_t flags;
        memcpy(&nbytes, it + 32, 4);
        memcpy(&flags, it + 38, 2);
        const uint64_t nt = 48ull + it[41] + 1 + nbytes + ((flags & 256) ? 4 : 0) + ((flags & 2) ? 8 : 0);
        ++c;
        off += nt;
    }
    return c;
}

int main(int argc, char **argv) {
    const uint64_t pages = argc > 1 ? strtoull(argv[1], nullptr, 10) : 300;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const uint64_t wbuf = 4ull << 20, nwb = pages * 16, bytes = nwb * wbuf;
    uint8_t *d = nullptr;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(d, 0x5a, bytes));
    for (uint64_t w = 0; w < nwb; ++w) CHECK(hipMemset(d + w * wbuf + 1007 * 4165, 0, wbuf - 1007 * 4165));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, d, nwb, wbuf, 12345u);
    CHECK(hipDeviceSynchronize());
    // host walk of every wbuf (headers only matter; copy wbuf by wbuf)
    std::vector<uint32_t> want(nwb);
    std::vector<uint8_t> hb(wbuf);
    uint64_t total = 0;
    for (uint64_t w = 0; w < nwb; ++w) {
        CHECK(hipMemcpy(hb.data(), d + w * wbuf, wbuf, hipMemcpyDeviceToHost));
        want[w] = host_walk(hb.data(), wbuf);
        total += want[w];
    }
    printf("pages %llu wbufs %llu items (host walk) %llu\n", (unsigned long long)pages, (unsigned long long)nwb,
           (unsigned long long)total);
    uint32_t *cnt = nullptr, *trace = nullptr;
    CHECK(hipMalloc(&cnt, nwb * 4));
    CHECK(hipMalloc(&trace, nwb * 32 * 4));
    CHECK(hipMemset(trace, 0xee, nwb * 32 * 4));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &trace, sizeof trace));
    std::vector<uint32_t> got(nwb);
    SpanArgs a{};
    a.base = d;
    a.base_bytes = bytes;
    a.region = wbuf;
    a.cfl = 4;
    const int gw = (int)std::min<uint64_t>((nwb + kWalkWaves - 1) / kWalkWaves, 65535);
    CHECK(hipFuncSetAttribute((const void *)k_count_v<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10));
    auto run = [&](int v, int lds_kib = 0) {
        CHECK(hipMemset(cnt, 0xff, nwb * 4));
        switch (v) {
            case 0: hipLaunchKernelGGL(k_count_v<0>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 1:
                hipLaunchKernelGGL(k_count_v<1>, dim3(gw), dim3(64 * kWalkWaves), lds_kib << 10, 0, a, nwb, cnt);
                break;
            case 2: hipLaunchKernelGGL(k_count_v<2>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 3: hipLaunchKernelGGL(k_count_v<3>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 4: hipLaunchKernelGGL(k_count_v<4>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 5: hipLaunchKernelGGL(k_count_v<5>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 6: hipLaunchKernelGGL(k_count_v<6>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 7: hipLaunchKernelGGL(k_count_v<7>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 8: hipLaunchKernelGGL(k_count_v<8>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 9: hipLaunchKernelGGL(k_count_v<9>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            case 10: hipLaunchKernelGGL(k_count_v<10>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
            default: hipLaunchKernelGGL(k_count_v<11>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt); break;
        }
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(got.data(), cnt, nwb * 4, hipMemcpyDeviceToHost));
        uint64_t bad = 0, sum = 0;
        int64_t first = -1;
        for (uint64_t w = 0; w < nwb; ++w) {
            sum += got[w];
            if (got[w] != want[w]) {
                ++bad;
                if (first < 0) first = (int64_t)w;
            }
        }
        printf("V%d%s: items %llu, wbufs wrong %llu", v,
               lds_kib == 100 ? " (1 workgroup per CU)" : lds_kib == 64 ? " (2 workgroups per CU)" : "",
               (unsigned long long)sum, (unsigned long long)bad);
        if (first >= 0) {
            printf(" (first: wbuf %lld got %u want %u; next %u/%u)", (long long)first, got[first], want[first],
                   first + 1 < (int64_t)nwb ? got[first + 1] : 0u, first + 1 < (int64_t)nwb ? want[first + 1] : 0u);
        }
        printf("\n");
        if (v == 7 && bad) {  // the first three wrong wbufs' round trips
            std::vector<uint32_t> tr(nwb * 32);
            CHECK(hipMemcpy(tr.data(), trace, nwb * 32 * 4, hipMemcpyDeviceToHost));
            int shown = 0;
            for (uint64_t w = 0; w < nwb && shown < 3; ++w) {
                if (got[w] == want[w]) continue;
                ++shown;
                printf("  wbuf %llu got %u want %u\n", (unsigned long long)w, got[w], want[w]);
                for (int r = 0; r < 4; ++r) {
                    const uint32_t *t = &tr[(w * 4 + r) * 8];
                    printf("    round %d: off %u s %u m %u last %u k %u nt_m %u brk %08x%08x lane0 nbytes %u nkey %u nt %u\n",
                           r, t[0], t[1], t[2] & 0xff, (t[2] >> 8) & 1, t[2] >> 16, t[3], t[5], t[4], t[6] & 0xffffff,
                           t[6] >> 24, t[7]);
                }
            }
        }
        fflush(stdout);
    };
    if (argc > 3 && !strcmp(argv[3], "vgpr")) {  // only the VGPR-allocation variants
        for (int r = 0; r < reps; ++r)
            for (int v : {0, 1, 9, 10, 11}) run(v);
        run(1, 100);
        // k_rl (readlane/SGPR chain) at 8 (its own count), 16, 24 and 32 VGPRs
        std::vector<uint32_t> tab(4096);
        for (uint32_t i = 0; i < 4096; ++i) tab[i] = i * 2246822519u ^ (i >> 3) * 3266489917u;
        uint32_t *dtab = nullptr, *dout = nullptr;
        const uint32_t nblk = 2048, nwave = nblk * 4, iters = 20000;
        CHECK(hipMalloc(&dtab, 4096 * 4));
        CHECK(hipMalloc(&dout, nwave * 4));
        CHECK(hipMemcpy(dtab, tab.data(), 4096 * 4, hipMemcpyHostToDevice));
        const uint32_t want = host_rl(tab, iters);
        std::vector<uint32_t> gotw(nwave);
        for (int r = 0; r < reps; ++r)
            for (int cl : {0, 16, 24, 32}) {
                CHECK(hipMemset(dout, 0, nwave * 4));
                if (cl == 0) hipLaunchKernelGGL((k_rl<0, 0>), dim3(nblk), dim3(256), 0, 0, dtab, iters, dout);
                if (cl == 16) hipLaunchKernelGGL((k_rl<0, 16>), dim3(nblk), dim3(256), 0, 0, dtab, iters, dout);
                if (cl == 24) hipLaunchKernelGGL((k_rl<0, 24>), dim3(nblk), dim3(256), 0, 0, dtab, iters, dout);
                if (cl == 32) hipLaunchKernelGGL((k_rl<0, 32>), dim3(nblk), dim3(256), 0, 0, dtab, iters, dout);
                CHECK(hipDeviceSynchronize());
                CHECK(hipMemcpy(gotw.data(), dout, nwave * 4, hipMemcpyDeviceToHost));
                uint32_t bad = 0;
                for (uint32_t w = 0; w < nwave; ++w) bad += gotw[w] != want;
                printf("k_rl readlane/SGPR chain, VGPRs %s: waves %u, wrong %u\n",
                       cl == 0 ? "8 (own)" : cl == 16 ? "16" : cl == 24 ? "24" : "32", nwave, bad);
                fflush(stdout);
            }
        return 0;
    }
    // the register-level test: 2048 blocks of 4 waves (8 per CU), 20000
    // sequences per wave, with and without the pad
    unsigned long long *dbad = nullptr;
    CHECK(hipMalloc(&dbad, 8));
    for (int r = 0; r < reps; ++r) {
        for (int pad = 0; pad <= 1; ++pad) {
            CHECK(hipMemset(dbad, 0, 8));
            if (pad)
                hipLaunchKernelGGL(k_waw<1>, dim3(2048), dim3(256), 0, 0, dbad, 20000u, 4165u, 0u, 4165ull);
            else
                hipLaunchKernelGGL(k_waw<0>, dim3(2048), dim3(256), 0, 0, dbad, 20000u, 4165u, 0u, 4165ull);
            CHECK(hipDeviceSynchronize());
            unsigned long long hb = 0;
            CHECK(hipMemcpy(&hb, dbad, 8, hipMemcpyDeviceToHost));
            printf("k_waw pad %d: sequences %llu, SGPR pair not -1 after the s_cselect: %llu\n", pad,
                   2048ull * 4 * 20000, hb);
            fflush(stdout);
        }
    }
    CHECK(hipFree(dbad));
    {
        std::vector<uint32_t> tab(4096);
        for (uint32_t i = 0; i < 4096; ++i) tab[i] = i * 2246822519u ^ (i >> 3) * 3266489917u;
        uint32_t *dtab = nullptr, *dout = nullptr;
        const uint32_t nblk = 2048, nwave = nblk * 4, iters = 20000;
        CHECK(hipMalloc(&dtab, 4096 * 4));
        CHECK(hipMalloc(&dout, nwave * 4));
        CHECK(hipMemcpy(dtab, tab.data(), 4096 * 4, hipMemcpyHostToDevice));
        CHECK(hipFuncSetAttribute((const void *)k_rl<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10));
        const uint32_t want = host_rl(tab, iters);
        std::vector<uint32_t> got(nwave);
        for (int r = 0; r < reps; ++r) {
            for (int mode = 0; mode <= 2; ++mode) {  // 2: MODE 0 at one workgroup per CU
                CHECK(hipMemset(dout, 0, nwave * 4));
                if (mode == 1)
                    hipLaunchKernelGGL(k_rl<1>, dim3(nblk), dim3(256), 0, 0, dtab, iters, dout);
                else
                    hipLaunchKernelGGL(k_rl<0>, dim3(nblk), dim3(256), mode == 2 ? 100 << 10 : 0, 0, dtab, iters, dout);
                CHECK(hipDeviceSynchronize());
                CHECK(hipMemcpy(got.data(), dout, nwave * 4, hipMemcpyDeviceToHost));
                uint32_t bad = 0, first = ~0u;
                for (uint32_t w = 0; w < nwave; ++w)
                    if (got[w] != want) {
                        ++bad;
                        if (first == ~0u) first = w;
                    }
                printf("k_rl %s: waves %u, wrong %u (first wave %d)\n",
                       mode == 0 ? "readlane/SGPR chain" : mode == 1 ? "bpermute/VGPR chain" : "readlane/SGPR chain, 1 workgroup per CU",
                       nwave, bad, (int)first);
                fflush(stdout);
            }
        }
        CHECK(hipFree(dtab));
        CHECK(hipFree(dout));
    }
    for (int r = 0; r < reps; ++r) {
        for (int v = 0; v <= 11; ++v) run(v);
        run(1, 100);
        run(1, 64);
    }
    CHECK(hipFree(cnt));
    CHECK(hipFree(d));
    return 0;
}
