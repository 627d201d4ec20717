// walk_vgpr_repro.hip -- reduced reproducer of the 24-VGPR walk miscompute
// (the full experiment is tools/walk_hazard.hip).  Not part of
// the library.
//
// The count pass of the round-2 page walk (lane m's break flag and size read
// with v_readlane into SGPRs, the walk state wave-uniform) over the bench's
// config-5 pages, against a host walk of the same headers:
//   W24     the walk as the compiler allocates it: 24 VGPRs;
//   W32     the same instruction stream at 32 VGPRs (an asm clobber of v31);
//   W24/1   W24 with 100 KiB of unused dynamic LDS (one workgroup per CU);
//   T24     W24 recording, for each wbuf's first four round trips, the walk
//           state and lane m's parsed header fields (read back from that lane
//           with v_readlane; still 24 VGPRs -- recording lane m's pointer as
//           well takes 25-28, and at 32 the failure is gone);
//   T32     T24 at 32 VGPRs;
//   R24     W24 with the wbufs dealt to the waves from the end (workgroup b
//           walks wbufs nw - 1 - 4b ..): the first workgroups on each CU
//           then walk the wbufs past 4 GiB, the co-resident ones those below
//           -- the two conditions under which W24 fails, always together in
//           the original order, separated;
//   R32     R24 at 32 VGPRs;
//   P24     the parse alone (k_parse: every lane parses its images' headers
//           against the values the fill gives, no walk state), 24 VGPRs;
//   P32     P24 at 32 VGPRs;
//   PS24    P24 over pages whose images all sit at one alignment (16 page
//           sets, one per sh = (p + 28) & 15): which alignments go wrong;
//   PS32    PS24 at 32 VGPRs;
//   PSA     PS24 with the header taken by v_alignbyte_b32 instead of 64-bit
//           shifts (parse_hdr_alignbyte: 19 VGPRs, allocated 24);
//   PSAP    PSA with 5 loaded values held live across the loop, so that the
//           allocation's top registers are in use (24 VGPRs).
// For the wrong wbufs of T24 the host replays the same lane-parallel walk and
// prints the first round trip that differs: the kernel's state and lane m's
// parsed fields against the header bytes at the pointer that state implies.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_vgpr_repro.hip -o /tmp/walk_vgpr_repro
//   /tmp/walk_vgpr_repro PAGES REPS
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

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

constexpr int kRounds = 4, kTr = 8;  // traced round trips per wbuf, dwords per round trip
constexpr int kAbVgprs = 19;         // k_parse<0, true, true>'s count in this build (allocated: 24)
constexpr int kAbPad = 5, kAbPadVgprs = 24;  // PSAP: pad values, k_parse<0, true, true, kAbPad>'s count

template <int CLOB, bool TRACE, bool REV = false>
__global__ __launch_bounds__(64 * kWalkWaves) void k_walk(SpanArgs a, uint64_t nw, uint32_t *cnt, uint32_t *trace) {
    if (CLOB == 32) asm volatile("" ::: "v31");
    const uint32_t j = threadIdx.x & 63u;
    const uint64_t wbuf = a.region;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t wv = (uint64_t)blockIdx.x * kWalkWaves + wave; wv < nw; wv += (uint64_t)gridDim.x * kWalkWaves) {
        const uint64_t w = REV ? nw - 1 - wv : wv;
        const uint64_t start = w * wbuf, size = a.base_bytes - start < wbuf ? a.base_bytes - start : wbuf;
        const uint8_t *wb = a.base + start;
        uint64_t off = 0, s = 0;
        uint32_t c = 0, round = 0;
        while (off + 48 <= size) {
            const uint64_t o = off + j * s;
            const bool in = (j == 0 || s != 0) && o + 48 <= size;
            const uint8_t *p = wb + o;
            ItemHdr h{0u, 0u, 0u, 0u};
            if (in) h = parse_hdr(p);
            const uint64_t nt = h.ntotal(4);
            const bool item = in && h.nkey != 0;
            const uint64_t brk = __ballot(!(item && nt == s));
            const uint32_t m = brk ? (uint32_t)__ffsll((unsigned long long)brk) - 1u : 64u;
            bool last_item = false;
            uint64_t nt_m = 0;
            if (m < 64u) {
                const int li = __builtin_amdgcn_readlane((int)item, (int)m);
                const int lo = __builtin_amdgcn_readlane((int)(uint32_t)nt, (int)m);
                const int hi = __builtin_amdgcn_readlane((int)(uint32_t)(nt >> 32), (int)m);
                last_item = li != 0;
                nt_m = (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
            }
            const uint32_t k = m < 64u ? m + (last_item ? 1u : 0u) : 64u;
            if (TRACE && round < (uint32_t)kRounds) {
                const int src = m < 64u ? (int)m : 0;
                const uint32_t nb = __builtin_amdgcn_readlane((int)h.nbytes, src);
                const uint32_t nk = __builtin_amdgcn_readlane((int)h.nkey, src);
                if (j == 0) {
                    uint32_t *t = trace + (w * kRounds + round) * kTr;
                    t[0] = (uint32_t)off;
                    t[1] = (uint32_t)s;
                    t[2] = m | (last_item ? 0x100u : 0u) | (k << 16);
                    t[3] = (uint32_t)nt_m;
                    t[4] = 0u;
                    t[5] = 0u;
                    t[6] = nb;
                    t[7] = nk;
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

// parse_hdr without 64-bit shifts: the 16 header bytes from the two pieces'
// dwords with v_alignbyte_b32 (byte funnel of two dwords)
__device__ __forceinline__ ItemHdr parse_hdr_alignbyte(const uint8_t *it) {
    const uint32_t sh = (uint32_t)((uintptr_t)(it + 28) & 15u);
    const uint8_t *q = it + 28 - sh;
    const bool two = sh + 13 >= 16;
    const Piece v0 = ld_piece(q), v1 = ld_piece(q + (two ? 16 : 0));
    const uint32_t d[8] = {(uint32_t)v0.lo, (uint32_t)(v0.lo >> 32), (uint32_t)v0.hi, (uint32_t)(v0.hi >> 32),
                           two ? (uint32_t)v1.lo : 0u, two ? (uint32_t)(v1.lo >> 32) : 0u,
                           two ? (uint32_t)v1.hi : 0u, two ? (uint32_t)(v1.hi >> 32) : 0u};
    const uint32_t qi = sh >> 2, b = sh & 3u;
    uint32_t w[5];
#pragma unroll
    for (uint32_t m = 0; m < 5; ++m)
        w[m] = qi == 0 ? d[m] : qi == 1 ? d[m + 1] : qi == 2 ? d[m + 2] : d[m + 3];
    // out[m] = image bytes 28 + 4m .. 31 + 4m
    const uint32_t o1 = __builtin_amdgcn_alignbyte(w[2], w[1], b), o2 = __builtin_amdgcn_alignbyte(w[3], w[2], b),
                   o3 = __builtin_amdgcn_alignbyte(w[4], w[3], b);
    (void)w[0];
    return {__builtin_amdgcn_alignbyte(w[1], w[0], b), o1, (o2 >> 16) & 0xffffu, (o3 >> 8) & 0xffu};
}

// The parse alone (no walk state, no readlane): every lane parses the header
// of image r * 64 + j of its wave's wbuf, as the walk's lanes do, and checks
// nbytes / nkey against the values the fill gives (LAYOUT: the one-alignment
// pages; AB: parse_hdr_alignbyte; PAD: values held live across the loop).
template <int CLOB, bool LAYOUT = false, bool AB = false, int PAD = 0>
__global__ __launch_bounds__(64 * kWalkWaves) void k_parse(SpanArgs a, uint64_t nw, uint32_t *cnt) {
    if (CLOB == 32) asm volatile("" ::: "v31");
    const uint32_t j = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t bad = 0;
    // PAD values loaded before and used after the loop: live across every
    // parse, they fill the allocation up to its top registers
    uint32_t pad[PAD > 0 ? PAD : 1];
#pragma unroll
    for (int m = 0; m < PAD; ++m) {
        pad[m] = reinterpret_cast<const uint32_t *>(a.base)[m * 64 + j];
        asm volatile("" : "+v"(pad[m]));
    }
    for (uint64_t w = (uint64_t)blockIdx.x * kWalkWaves + wave; w < nw; w += (uint64_t)gridDim.x * kWalkWaves) {
        const uint8_t *wb = a.base + w * a.region;
#pragma unroll 1
        for (uint32_t r = 0; r < 16; ++r) {
            const uint32_t i = r * 64u + j;
            if (i >= (LAYOUT ? 1000u : 1007u)) break;
            const uint8_t *p = wb + (uint64_t)i * (LAYOUT ? 4176u : 4165u);
            const ItemHdr h = AB ? parse_hdr_alignbyte(p) : parse_hdr(p);
            // every image here has nbytes < 2^20 (4098, at most one bit of 0..19
            // flipped) and nkey 10 or 0; the walk's wrong parses gave
            // nbytes 0x0a111002 or nkey 105 (checking against byte loads of
            // the image instead takes the kernel to 26-27 VGPRs)
            bad += (h.nbytes >> 20 != 0u) | (h.nkey != 10u && h.nkey != 0u);
        }
    }
#pragma unroll
    for (int m = 0; m < PAD; ++m) {
        asm volatile("" : "+v"(pad[m]));
        bad += pad[m] == 0x13572468u;  // (never: the pages hold no such word)
    }
    if (bad) atomicAdd(cnt, bad);
}

// config-5 layout (bench.py workload_config5): item i of wbuf w at
// w * wbuf + i * 4165, a few headers with a flipped nbytes bit or nkey 0
__global__ void k_fill(uint8_t *base, uint64_t nwb, uint64_t wbuf, uint32_t seed, uint32_t per = 1007,
                       uint32_t stride = 4165, uint32_t phase = 0) {
    const uint64_t n = nwb * per;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t *it = base + (i / per) * wbuf + phase + (i % per) * stride;
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
        it[38] = 2;  // ITEM_CAS
        it[39] = 0;
        it[40] = 17;
        it[41] = nkey;
    }
}

struct Hdr {
    uint32_t nbytes, nkey, flags;
    uint64_t nt;
};
static Hdr host_hdr(const uint8_t *it) {
    Hdr h;
    memcpy(&h.nbytes, it + 32, 4);
    uint16_t fl;
    memcpy(&fl, it + 38, 2);
    h.flags = fl;
    h.nkey = it[41];
    h.nt = 48ull + h.nkey + 1 + h.nbytes + ((fl & 256) ? 4 : 0) + ((fl & 2) ? 8 : 0);
    return h;
}

static uint32_t host_walk(const uint8_t *b, uint64_t size) {
    uint64_t off = 0;
    uint32_t c = 0;
    while (off + 48 <= size) {
        const Hdr h = host_hdr(b + off);
        if (h.nkey == 0) break;
        ++c;
        off += h.nt;
    }
    return c;
}

// the kernel's lane-parallel walk replayed on the host: round trip r's trace
struct Rt {
    uint64_t off, s, nt_m, lane_off;
    uint32_t m, last, k;
    Hdr hm;
};
static std::vector<Rt> host_rounds(const uint8_t *b, uint64_t size, int nr) {
    std::vector<Rt> out;
    uint64_t off = 0, s = 0;
    while (off + 48 <= size && (int)out.size() < nr) {
        uint32_t m = 64;
        bool last = false;
        Hdr hm{0, 0, 0, 49};
        for (uint32_t j = 0; j < 64; ++j) {
            const uint64_t o = off + j * s;
            const bool in = (j == 0 || s != 0) && o + 48 <= size;
            const Hdr h = in ? host_hdr(b + o) : Hdr{0, 0, 0, 49};
            const bool item = in && h.nkey != 0;
            if (!(item && h.nt == s)) {
                m = j;
                last = item;
                hm = h;
                break;
            }
            if (j == 0) hm = h;
        }
        Rt r{off, s, m < 64 ? hm.nt : 0, off + (m < 64 ? m : 0) * s, m, last, m < 64 ? m + (last ? 1u : 0u) : 64u,
             hm};
        out.push_back(r);
        if (m == 64) off += 64 * s;
        else if (!last) break;
        else {
            off += m * s + hm.nt;
            s = hm.nt;
        }
    }
    return out;
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
    std::vector<uint32_t> want(nwb);
    std::vector<uint8_t> hb(wbuf);
    uint64_t total = 0;
    for (uint64_t w = 0; w < nwb; ++w) {
        CHECK(hipMemcpy(hb.data(), d + w * wbuf, wbuf, hipMemcpyDeviceToHost));
        want[w] = host_walk(hb.data(), wbuf);
        total += want[w];
    }
    printf("pages %llu wbufs %llu items (host walk) %llu, device base %p\n", (unsigned long long)pages,
           (unsigned long long)nwb, (unsigned long long)total, (void *)d);
    uint32_t *cnt = nullptr, *trace = nullptr;
    CHECK(hipMalloc(&cnt, nwb * 4));
    CHECK(hipMalloc(&trace, nwb * kRounds * kTr * 4));
    std::vector<uint32_t> got(nwb), tr(nwb * kRounds * kTr);
    SpanArgs a{};
    a.base = d;
    a.base_bytes = bytes;
    a.region = wbuf;
    a.cfl = 4;
    const int gw = (int)std::min<uint64_t>((nwb + kWalkWaves - 1) / kWalkWaves, 65535);
    CHECK(hipFuncSetAttribute((const void *)k_walk<24, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10));
    auto run = [&](const char *name, int v, int lds_kib) {
        CHECK(hipMemset(cnt, 0xff, nwb * 4));
        CHECK(hipMemset(trace, 0xee, nwb * kRounds * kTr * 4));
        const dim3 g(gw), b(64 * kWalkWaves);
        if (v == 0) hipLaunchKernelGGL((k_walk<24, false>), g, b, lds_kib << 10, 0, a, nwb, cnt, trace);
        if (v == 1) hipLaunchKernelGGL((k_walk<32, false>), g, b, 0, 0, a, nwb, cnt, trace);
        if (v == 2) hipLaunchKernelGGL((k_walk<24, true>), g, b, 0, 0, a, nwb, cnt, trace);
        if (v == 3) hipLaunchKernelGGL((k_walk<32, true>), g, b, 0, 0, a, nwb, cnt, trace);
        if (v == 4) hipLaunchKernelGGL((k_walk<24, false, true>), g, b, 0, 0, a, nwb, cnt, trace);
        if (v == 5) hipLaunchKernelGGL((k_walk<32, false, true>), g, b, 0, 0, a, nwb, cnt, trace);
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
        // wrong wbufs below / past 4 GiB, and by whether their workgroup is
        // one of the first 256 (one per CU) or a co-resident one
        uint64_t lo4 = 0, hi4 = 0, firstwg = 0, laterwg = 0, lastw = 0;
        for (uint64_t w = 0; w < nwb; ++w) {
            if (got[w] == want[w]) continue;
            (w * wbuf < (4ull << 30) ? lo4 : hi4) += 1;
            const uint64_t wv = v >= 4 ? nwb - 1 - w : w;
            (wv / kWalkWaves < 256 ? firstwg : laterwg) += 1;
            lastw = w;
        }
        printf("%s: items %llu, wbufs wrong %llu", name, (unsigned long long)sum, (unsigned long long)bad);
        if (first >= 0)
            printf(" (wbufs %lld..%llu; below 4 GiB %llu, past %llu; in workgroups 0-255 %llu, 256+ %llu)",
                   (long long)first, (unsigned long long)lastw, (unsigned long long)lo4, (unsigned long long)hi4,
                   (unsigned long long)firstwg, (unsigned long long)laterwg);
        printf("\n");
        if ((v == 2 || v == 3) && bad) {
            CHECK(hipMemcpy(tr.data(), trace, tr.size() * 4, hipMemcpyDeviceToHost));
            int shown = 0;
            uint64_t diverged = 0, state_ok_fields_bad = 0, fields_ok = 0;
            for (uint64_t w = 0; w < nwb; ++w) {
                if (got[w] == want[w]) continue;
                CHECK(hipMemcpy(hb.data(), d + w * wbuf, wbuf, hipMemcpyDeviceToHost));
                const std::vector<Rt> hr = host_rounds(hb.data(), wbuf, kRounds);
                for (size_t r = 0; r < hr.size(); ++r) {
                    const uint32_t *t = &tr[(w * kRounds + r) * kTr];
                    const uint32_t m = t[2] & 0xff, last = (t[2] >> 8) & 1;
                    const bool state = t[0] == (uint32_t)hr[r].off && t[1] == (uint32_t)hr[r].s;
                    if (state && m == hr[r].m && last == hr[r].last && t[3] == (uint32_t)hr[r].nt_m) continue;
                    ++diverged;
                    // the header at the pointer the kernel's own state implies for lane m
                    const uint64_t lane = m < 64 ? m : 0, o = (uint64_t)t[0] + lane * (uint64_t)t[1];
                    const bool inside = o + 48 <= wbuf;
                    const Hdr at = inside ? host_hdr(hb.data() + o) : Hdr{0, 0, 0, 0};
                    const bool same_fields = inside && at.nbytes == t[6] && at.nkey == t[7];
                    fields_ok += same_fields;
                    state_ok_fields_bad += state && !same_fields;
                    if (shown < 6) {
                        ++shown;
                        printf("  wbuf %llu (got %u want %u), first differing round trip %zu:\n", (unsigned long long)w,
                               got[w], want[w], r);
                        printf("    kernel: off %u s %u m %u last %u nt_m %u; lane %llu parsed nbytes %u nkey %u\n", t[0],
                               t[1], m, last, t[3], (unsigned long long)lane, t[6], t[7]);
                        printf("    bytes at wbuf offset %llu (what that state implies): nbytes %u nkey %u (%s)\n",
                               (unsigned long long)o, at.nbytes, at.nkey, same_fields ? "same" : "DIFFERENT");
                        printf("    host replay: off %llu s %llu m %u last %u nt_m %llu (lane %u header nbytes %u nkey %u)\n",
                               (unsigned long long)hr[r].off, (unsigned long long)hr[r].s, hr[r].m, hr[r].last,
                               (unsigned long long)hr[r].nt_m, hr[r].m, hr[r].hm.nbytes, hr[r].hm.nkey);
                    }
                    break;
                }
            }
            printf("  wrong wbufs diverging within %d round trips: %llu; state (off, s) still right but lane m's parsed "
                   "header not the bytes there: %llu; parsed header right (the wrong value arose after the parse): %llu\n",
                   kRounds, (unsigned long long)diverged, (unsigned long long)state_ok_fields_bad,
                   (unsigned long long)fields_ok);
        }
        fflush(stdout);
    };
    for (int r = 0; r < reps; ++r) {
        run("W24", 0, 0);
        run("W32", 1, 0);
        run("W24/1 (one workgroup per CU)", 0, 100);
        run("T24", 2, 0);
        run("T32", 3, 0);
        run("R24", 4, 0);
        run("R32", 5, 0);
        for (int pv = 0; pv < 2; ++pv) {
            CHECK(hipMemset(cnt, 0, 4));
            if (pv == 0) hipLaunchKernelGGL(k_parse<24>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt);
            else hipLaunchKernelGGL(k_parse<32>, dim3(gw), dim3(64 * kWalkWaves), 0, 0, a, nwb, cnt);
            CHECK(hipDeviceSynchronize());
            uint32_t nbad = 0;
            CHECK(hipMemcpy(&nbad, cnt, 4, hipMemcpyDeviceToHost));
            printf("%s: headers parsed %llu, not as their bytes %u\n", pv ? "P32" : "P24",
                   (unsigned long long)nwb * 1007, nbad);
            fflush(stdout);
        }
    }
    // PS24 / PS32: the parse over pages whose 1000 images per wbuf all sit at
    // one alignment: image i at phase + 4176 i, so sh = (phase + 28) & 15
    // for all of them (k_parse<LAYOUT>: the same code with 4176 / 1000 for
    // 4165 / 1007, the phase in the base pointer)
    {
        const uint32_t per = 1000, stride = 4176;
        SpanArgs b = a;
        for (int cl = 24; cl <= 48; cl += 8) {  // (40: PSA, the v_alignbyte parse at its own allocation; 48: PSAP)
            if (cl == 48) printf("PSAP (PSA with %d values live across the loop: %d VGPRs): wrong parses of %llu by sh:", kAbPad,
                                 kAbPadVgprs, (unsigned long long)nwb * per);
            else if (cl == 40) printf("PSA (parse_hdr_alignbyte, %d VGPRs): wrong parses of %llu by sh = (p + 28) & 15:", kAbVgprs,
                                 (unsigned long long)nwb * per);
            else printf("PS%d: wrong parses of %llu by sh = (p + 28) & 15:", cl, (unsigned long long)nwb * per);
            for (uint32_t phase = 0; phase < 16; ++phase) {
                CHECK(hipMemset(d, 0x5a, bytes));
                hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, d, nwb, wbuf, 777u + phase, per, stride, phase);
                b.base = d + phase;  // (the last wbuf's images end 4176 B short of the pages' end)
                CHECK(hipMemset(cnt, 0, 4));
                if (cl == 24) hipLaunchKernelGGL((k_parse<24, true>), dim3(gw), dim3(64 * kWalkWaves), 0, 0, b, nwb, cnt);
                else if (cl == 32) hipLaunchKernelGGL((k_parse<32, true>), dim3(gw), dim3(64 * kWalkWaves), 0, 0, b, nwb, cnt);
                else if (cl == 40) hipLaunchKernelGGL((k_parse<0, true, true>), dim3(gw), dim3(64 * kWalkWaves), 0, 0, b, nwb, cnt);
                else hipLaunchKernelGGL((k_parse<0, true, true, kAbPad>), dim3(gw), dim3(64 * kWalkWaves), 0, 0, b, nwb, cnt);
                CHECK(hipDeviceSynchronize());
                uint32_t nbad = 0;
                CHECK(hipMemcpy(&nbad, cnt, 4, hipMemcpyDeviceToHost));
                printf(" %u:%u", (phase + 28) & 15, nbad);
                fflush(stdout);
            }
            printf("\n");
        }
    }
    CHECK(hipFree(cnt));
    CHECK(hipFree(trace));
    CHECK(hipFree(d));
    return 0;
}
