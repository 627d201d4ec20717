// crc32c_kernels.hip -- hand-written gfx950 kernels for batched CRC-32C.
//
// K1  k_fixed<SLICE, LPI, CH, R>: equal-length, 16-B aligned items at a fixed
//     stride, len = R*LPI*CH (extstore spill batches of one slab class;
//     BASELINE configs 2 and 4).  Replaces N calls of crc32c(0, item, len),
//     crc32c_hw (crc32c.c:161-246) reached from storage.c:567.
// K2  k_spans<UNALIGNED, MODE=0>: any offsets, lengths and alignment; one
//     32-lane group per span (configs 3 and 5, storage.c:172 read-back spans).
// K3  k_spans<true, MODE=1>: verify packed item images in extstore pages: the
//     span [off+32, off+ITEM_ntotal) is checked against the CRC stored in the
//     item's exptime field (storage.c:160-178 over the page walk of
//     storage.c:950-960).
//
// See crc32c_device.h for the lane-group work model and LDS table layouts.
#include "crc32c_device.h"

namespace mcrc_dev {

// ===========================================================================
// K1: fixed-length aligned items
// ===========================================================================

__device__ __forceinline__ uint32_t dw4(const uint4 &v, int k) {
    return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}

// One lane's share of one item: R rows x CH bytes, 16-B loads.
template <int LPI, int CH, int R>
struct ItemRegs {
    static constexpr int Q = CH / 16;
    uint4 d[R][Q];

    __device__ __forceinline__ void load(const uint8_t *__restrict__ p, uint32_t li) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < Q; ++q)
                d[r][q] = *reinterpret_cast<const uint4 *>(p + (size_t)r * LPI * CH + li * CH + 16 * q);
    }
    __device__ __forceinline__ uint32_t checksum() const {
        uint32_t a = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < Q; ++q) a ^= d[r][q].x ^ d[r][q].y ^ d[r][q].z ^ d[r][q].w;
        return a;
    }
};

// Lane partial: R independent chains (interleaved dword by dword for ILP),
// folded with M_{LPI*CH} into the raw CRC of the lane's R chunks as placed in
// the item.  FOLD=false is a profiling ablation.
template <int SLICE, int LPI, int CH, int R, bool FOLD = true>
__device__ __forceinline__ uint32_t lane_partial(const ItemRegs<LPI, CH, R> &it, const LaneCtx &c) {
    constexpr int Q = CH / 16;
    constexpr uint32_t kFold = 4 * (LPI == 64 ? 6 : LPI == 32 ? 5 : 4);  // M_{LPI*CH}
    uint32_t s[R];
#pragma unroll
    for (int r = 0; r < R; ++r) s[r] = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint4 &v = it.d[r][q];
                const uint32_t w = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
                s[r] = Step<SLICE>::dword(s[r] ^ w, c);
            }
        }
    }
    uint32_t a = s[0];
#pragma unroll
    for (int r = 1; r < R; ++r) a = (FOLD ? apply_op<SLICE>(kFold, a) : a) ^ s[r];
    return a;
}

// Lane partial for SLICE 4, LPI 32: chains fused with bitop3 XORs.
template <int CH, int R>
__device__ __forceinline__ uint32_t lane_partial_x3(const ItemRegs<32, CH, R> &it, const LaneCtx &c) {
    constexpr int Q = CH / 16;
    constexpr int N = 4 * Q;  // dwords per chain
    uint32_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = it.d[r][0].x;
#pragma unroll
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t wn = i + 1 < N ? dw4(it.d[r][(i + 1) >> 2], (i + 1) & 3) : 0u;
            x[r] = step4_next(x[r], wn, c);
        }
    }
    uint32_t a = x[0];
#pragma unroll
    for (int r = 1; r < R; ++r) a = apply_op<4>(kAuxOp5, a) ^ x[r];
    return a;
}

// Same as lane_partial_x3, but the loads of the NEXT step (into `nxt`) are
// issued one at a time between dword steps of this chain, so the vector
// memory queue is fed steadily instead of in one burst per step.
template <int CH, int R>
__device__ __forceinline__ uint32_t lane_partial_x3_feed(const ItemRegs<32, CH, R> &it, const LaneCtx &c,
                                                         ItemRegs<32, CH, R> &nxt, const uint8_t *np,
                                                         uint32_t li) {
    constexpr int Q = CH / 16;
    constexpr int N = 4 * Q;       // dwords per chain
    constexpr int NL = R * Q;      // loads per step
    constexpr int EVERY = N / NL > 0 ? N / NL : 1;
    uint32_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = it.d[r][0].x;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (i % EVERY == 0 && i / EVERY < NL) {
            constexpr int dummy = 0;
            (void)dummy;
            const int l = i / EVERY, r = l / Q, q = l % Q;
            nxt.d[r][q] = *reinterpret_cast<const uint4 *>(np + (size_t)r * 32 * CH + li * CH + 16 * q);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t wn = i + 1 < N ? dw4(it.d[r][(i + 1) >> 2], (i + 1) & 3) : 0u;
            x[r] = step4_next(x[r], wn, c);
        }
    }
#pragma unroll
    for (int l = (N + EVERY - 1) / EVERY; l < NL; ++l) {
        const int r = l / Q, q = l % Q;
        nxt.d[r][q] = *reinterpret_cast<const uint4 *>(np + (size_t)r * 32 * CH + li * CH + 16 * q);
    }
    uint32_t a = x[0];
#pragma unroll
    for (int r = 1; r < R; ++r) a = apply_op<4>(kAuxOp5, a) ^ x[r];
    return a;
}

// Persistent grid-stride loop; each wave handles 64/LPI items per step and
// loads the next step's items before reducing the current ones (register
// ping-pong, no copies).
//   out[i] = crc32c(crc_in ? crc_in[i] : 0, base + i*stride, len),  len = R*LPI*CH
//   kfinal = ~M_len(0xffffffff), kspan = x^(8*len) mod P.
// MODE 0: full CRC.  Ablations for profiling (wrong results by design):
// MODE 1: loads only; MODE 2: no lane-group reduction; MODE 3: data chains only.
// MODE 4/5: full CRC, optimised variants (SLICE 4, LPI 32 only).
// MODE 6: MODE 5 with the next step's loads spread over the chains.
template <int SLICE, int LPI, int CH, int R, int MODE, int DEPTH = 2, int STAGGER = 0>
__global__ __launch_bounds__(1024) void k_fixed(const uint8_t *__restrict__ base, uint64_t stride,
                                                uint64_t nitems, const uint4 *__restrict__ img,
                                                uint32_t kfinal, uint32_t kspan,
                                                const uint32_t *__restrict__ crc_in,
                                                uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, LdsImage<SLICE>::bytes);
    constexpr uint32_t IPW = 64 / LPI;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t li = lane % LPI;
    const uint32_t g = lane / LPI;
    LaneCtx c;
    c.lane4 = (lane & 31u) << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t gstep = gridDim.x * waves;
    const uint64_t ngroups = (nitems + IPW - 1) / IPW;
    uint64_t grp = blockIdx.x * waves + (threadIdx.x >> 6);
    if (grp >= ngroups) return;
    if constexpr (STAGGER > 0) {
        // desynchronise the workgroup's waves: odd waves start STAGGER x 8K cycles late
        if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 1u)
            for (int i = 0; i < STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
    }

    auto item_of = [&](uint64_t gi) { return gi * IPW + g; };
    auto clamp = [&](uint64_t it) { return it < nitems ? it : nitems - 1; };
    auto finish = [&](const ItemRegs<LPI, CH, R> &regs, uint64_t gi) {
        const uint64_t item = item_of(gi);
        if (MODE == 1) {
            const uint32_t a = regs.checksum();
            if (a == 0x9e3779b9u && item < nitems) out[item] = a;
            return;
        }
        uint32_t raw;
        if (MODE == 5)  // optimised: bitop3 chains + DPP reduction (SLICE 4, LPI 32)
            raw = group_reduce32_dpp(lane_partial_x3<CH, R>(regs, c), lane);
        else if (MODE == 4)  // bitop3 chains, LDS-shuffle reduction
            raw = group_reduce<SLICE, LPI>(lane_partial_x3<CH, R>(regs, c), lane);
        else if (MODE == 3)
            raw = lane_partial<SLICE, LPI, CH, R, false>(regs, c);
        else if (MODE == 2)
            raw = lane_partial<SLICE, LPI, CH, R>(regs, c);
        else
            raw = group_reduce<SLICE, LPI>(lane_partial<SLICE, LPI, CH, R>(regs, c), lane);
        if (li == 0 && item < nitems) {
            out[item] = crc_in ? ~(mulmodp_dev(~crc_in[item], kspan) ^ raw) : raw ^ kfinal;
        }
    };

    auto addr = [&](uint64_t gi) { return base + clamp(item_of(gi < ngroups ? gi : ngroups - 1)) * stride; };
    ItemRegs<LPI, CH, R> ra, rb;
    if constexpr (MODE == 6) {
        // loads of the next step interleaved with this step's chains
        auto fin6 = [&](const ItemRegs<LPI, CH, R> &cur, ItemRegs<LPI, CH, R> &nxt, uint64_t gi) {
            const uint64_t item = item_of(gi);
            const uint32_t raw =
                group_reduce32_dpp(lane_partial_x3_feed<CH, R>(cur, c, nxt, addr(gi + gstep), li), lane);
            if (li == 0 && item < nitems)
                out[item] = crc_in ? ~(mulmodp_dev(~crc_in[item], kspan) ^ raw) : raw ^ kfinal;
        };
        ra.load(addr(grp), li);
        for (;;) {
            fin6(ra, rb, grp);
            grp += gstep;
            if (grp >= ngroups) break;
            fin6(rb, ra, grp);
            grp += gstep;
            if (grp >= ngroups) break;
        }
    } else if (DEPTH == 2) {
        ra.load(addr(grp), li);
        for (;;) {
            rb.load(addr(grp + gstep), li);
            finish(ra, grp);
            grp += gstep;
            if (grp >= ngroups) break;
            ra.load(addr(grp + gstep), li);
            finish(rb, grp);
            grp += gstep;
            if (grp >= ngroups) break;
        }
    } else {
        // three register buffers: two steps in flight while one is reduced
        ItemRegs<LPI, CH, R> rc;
        ra.load(addr(grp), li);
        rb.load(addr(grp + gstep), li);
        for (;;) {
            rc.load(addr(grp + 2 * gstep), li);
            finish(ra, grp);
            grp += gstep;
            if (grp >= ngroups) break;
            ra.load(addr(grp + 2 * gstep), li);
            finish(rb, grp);
            grp += gstep;
            if (grp >= ngroups) break;
            rb.load(addr(grp + 2 * gstep), li);
            finish(rc, grp);
            grp += gstep;
            if (grp >= ngroups) break;
        }
    }
}

// ===========================================================================
// K2/K3: arbitrary spans, one 32-lane group per work unit
// ===========================================================================
//
// Work units.  A span longer than kSegBytes is cut into segments of kSegBytes
// anchored at its END (segment 0, the head, holds the remainder); every
// segment is one work unit, so no group owns more than 64 KiB and a batch of
// Zipf-sized items balances over the grid.  Units come from k_count ->
// exclusive scan -> k_expand; a batch whose spans are all <= kSegBytes uses
// unit u = span u directly.  k_combine folds the segment CRCs of long spans:
//   raw(span) = sum_s M_{64 KiB * (nseg-1-s)}(raw(segment s))   (Horner)
//
// Unit geometry (CH = 64, LPI = 32): a unit [p, E) is covered by npairs row
// pairs anchored at E: pair k covers [G + 4096k, G + 4096(k+1)) with
// G = E - 4096 * npairs, row A = first 2048 bytes, row B = second.  Lane li
// owns bytes [64 li, 64 li + 64) of each row.  Bytes before p are zero, which
// leaves a zero-initialised register unchanged, so the grid needs no tail
// handling and every lane chain ends on a row boundary.  Per pair a lane folds
//   acc = M_4096(acc) ^ M_2048(raw A chunk) ^ raw B chunk,
// and the 32 lane accumulators are merged by the lane-group reduction.
//
// Loads are always 16-B aligned pieces that overlap [p, E) (so they never leave
// the pages holding the span); a piece wholly outside is read from a zeroed
// device buffer instead, so no load is predicated.  When E is not 16-B aligned
// every lane reads five pieces and realigns them with v_alignbyte.

constexpr uint32_t kSpanCH = 64;
constexpr uint32_t kRowBytes = 32 * kSpanCH;  // 2048
constexpr uint32_t kPairBytes = 2 * kRowBytes;
constexpr uint32_t kSegBytes = 64 * 1024;
constexpr uint32_t kWhole = 0xffffffffu;      // unit segment index: the whole span

struct SpanArgs {
    const uint8_t *base;       // all spans live in [base, base + base_bytes)
    uint64_t base_bytes;
    const uint64_t *offsets;   // span i starts at base + offsets[i] (MODE 0)
                               // or item image i at base + offsets[i] (MODE 1)
    uint64_t stride;           // when offsets == nullptr: base + i * stride
    const uint32_t *lens;      // per-span lengths, or nullptr: every span is `len`
    uint32_t len;
    uint32_t kspan;            // x^(8*len) when lens == nullptr
    const uint32_t *crc_in;    // MODE 0: per-span initial CRC or nullptr (0)
    uint32_t *out;             // MODE 0: CRC per span
    uint8_t *ok;               // MODE 1: 1 if the stored CRC matches
    unsigned long long *nbad;  // MODE 1: count of mismatches (atomic)
    uint64_t n;                // spans (items)
    const uint32_t *xpow;      // 3 x 1024 table: x^(8*j), x^(8*1024*j), x^(8*2^20*j)
    const uint4 *zero;         // 16 zero bytes in device memory
    // work units (nullptr: unit u = span u, one segment)
    const uint2 *units;        // (span index, segment index or kWhole)
    const uint32_t *nunits;    // device-side unit count
    uint32_t *seg_raw;         // raw CRC of each unit of a multi-segment span
};

struct ItemDesc {
    const uint8_t *p;
    uint32_t len;
    uint32_t aux;  // MODE 0: initial CRC; MODE 1: stored CRC
    bool sane;     // MODE 1: header parsed to an in-bounds span
};

__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p) { return *p; }
__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t *p) {
    return ld_u8(p) | (ld_u8(p + 1) << 8) | (ld_u8(p + 2) << 16) | (ld_u8(p + 3) << 24);
}

__device__ __forceinline__ uint32_t nseg_of(uint32_t len) {
    return len <= kSegBytes ? 1u : (len + kSegBytes - 1) / kSegBytes;
}

template <int MODE>
__device__ __forceinline__ ItemDesc fetch_item(const SpanArgs &a, uint64_t i) {
    ItemDesc d;
    const uint64_t off = a.offsets ? a.offsets[i] : i * a.stride;
    if (MODE == 0) {
        d.p = a.base + off;
        d.len = a.lens ? a.lens[i] : a.len;
        d.aux = a.crc_in ? a.crc_in[i] : 0u;
        d.sane = true;
    } else {
        // item header fields (memcached.h:613-636), ITEM_ntotal (:149-152)
        const uint8_t *it = a.base + off;
        const bool hdr_ok = off + 48 <= a.base_bytes;
        const uint32_t nbytes = hdr_ok ? ld_u32_unaligned(it + 32) : 0u;
        const uint32_t flags = hdr_ok ? (ld_u8(it + 38) | (ld_u8(it + 39) << 8)) : 0u;
        const uint32_t nkey = hdr_ok ? ld_u8(it + 41) : 0u;
        const uint64_t ntotal = 48ull + nkey + 1 + nbytes + ((flags & 256u) ? 4 : 0) + ((flags & 2u) ? 8 : 0);
        d.aux = hdr_ok ? ld_u32_unaligned(it + 28) : 0u;
        d.sane = hdr_ok && nkey != 0 && nbytes < 0x80000000u && off + ntotal <= a.base_bytes;
        d.p = it + 32;
        d.len = d.sane ? (uint32_t)(ntotal - 32) : 0u;
    }
    return d;
}

struct UnitDesc {
    const uint8_t *p;  // first byte of this unit
    uint32_t len;      // bytes of this unit
    uint32_t npairs;
    uint32_t aux;      // of the span
    uint32_t span_len;
    uint64_t item;     // span index
    uint64_t unit;
    bool valid;
    bool single;       // the unit is the whole span: finalise directly
    bool sane;
};

template <int MODE>
__device__ __forceinline__ UnitDesc fetch_unit(const SpanArgs &a, uint64_t u, uint64_t nunits) {
    UnitDesc d;
    d.valid = u < nunits;
    d.p = a.base;
    d.len = 0;
    d.aux = 0;
    d.span_len = 0;
    d.item = 0;
    d.unit = u;
    d.single = true;
    d.sane = true;
    if (d.valid) {
        uint32_t seg = kWhole;  // without a unit list every span is one unit
        d.item = u;
        if (a.units) {
            const uint2 e = a.units[u];
            d.item = e.x;
            seg = e.y;
        }
        const ItemDesc it = fetch_item<MODE>(a, d.item);
        d.aux = it.aux;
        d.span_len = it.len;
        d.sane = it.sane;
        const uint32_t nseg = seg == kWhole ? 1u : nseg_of(it.len);
        d.single = nseg == 1;
        if (d.single) {
            d.p = it.p;
            d.len = it.len;
        } else {
            const uint8_t *seg_end = it.p + it.len - (size_t)(nseg - 1 - seg) * kSegBytes;
            d.p = seg == 0 ? it.p : seg_end - kSegBytes;
            d.len = (uint32_t)(seg_end - d.p);
        }
    }
    d.npairs = (d.len + kPairBytes - 1) / kPairBytes;
    return d;
}

template <bool UNALIGNED>
struct RowWin {
    static constexpr int NP = UNALIGNED ? 5 : 4;
    uint4 v[NP];
};

template <bool UNALIGNED>
struct PairWin {
    RowWin<UNALIGNED> a, b;
};

// Issue the loads of row pair k of unit d for lane li.
template <bool UNALIGNED>
__device__ __forceinline__ void load_pair(PairWin<UNALIGNED> &w, const UnitDesc &d, uint32_t k, uint32_t li,
                                          const uint4 *zero) {
    const uint8_t *E = d.p + d.len;
    const uint8_t *G = E - (size_t)kPairBytes * d.npairs + (size_t)kPairBytes * k;
    const uint8_t *sa = G + kSpanCH * li;
    const uint32_t u = UNALIGNED ? (uint32_t)((uintptr_t)E & 15u) : 0u;
    const uint8_t *wa = sa - u;
    const uint8_t *wb = wa + kRowBytes;
#pragma unroll
    for (int j = 0; j < RowWin<UNALIGNED>::NP; ++j) {
        const uint8_t *pa = wa + 16 * j, *pb = wb + 16 * j;
        const bool oka = d.valid && pa + 16 > d.p && pa < E;
        const bool okb = d.valid && pb + 16 > d.p && pb < E;
        w.a.v[j] = *(oka ? reinterpret_cast<const uint4 *>(pa) : zero);
        w.b.v[j] = *(okb ? reinterpret_cast<const uint4 *>(pb) : zero);
    }
}

// Realign a five-piece window to the 16 chunk dwords starting at byte u.
__device__ __forceinline__ void realign(const RowWin<true> &w, uint32_t u, uint32_t out[16]) {
    uint32_t t[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) t[i] = dw4(w.v[i >> 2], i & 3);
    const bool q2 = u & 8u, q1 = u & 4u;
#pragma unroll
    for (int i = 0; i < 18; ++i) t[i] = q2 ? t[i + 2] : t[i];
#pragma unroll
    for (int i = 0; i < 17; ++i) t[i] = q1 ? t[i + 1] : t[i];
    const uint32_t b = u & 3u;
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = __builtin_amdgcn_alignbyte(t[i + 1], t[i], b);
}

__device__ __forceinline__ void straight(const RowWin<false> &w, uint32_t out[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = dw4(w.v[i >> 2], i & 3);
}

// Zero the chunk bytes that precede the unit start p (lo = p - chunk start).
__device__ __forceinline__ void mask_head(uint32_t v[16], int64_t lo) {
    const int32_t l = lo < 0 ? 0 : lo > 64 ? 64 : (int32_t)lo;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int32_t k = l - 4 * i;
        k = k < 0 ? 0 : k > 4 ? 4 : k;
        v[i] &= (uint32_t)(0xffffffffull << (8 * k));
    }
}

// Two independent chains (rows A and B) from zero registers, interleaved,
// with bitop3-fused XORs.
__device__ __forceinline__ void chain16x2(const uint32_t a[16], const uint32_t b[16], const LaneCtx &c,
                                          uint32_t &sa, uint32_t &sb) {
    uint32_t x = a[0], y = b[0];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        x = step4_next(x, i + 1 < 16 ? a[i + 1] : 0u, c);
        y = step4_next(y, i + 1 < 16 ? b[i + 1] : 0u, c);
    }
    sa = x;
    sb = y;
}

// x^(8*len) mod P from the three-level table (len < 2^30).
__device__ __forceinline__ uint32_t xpow8_dev(const uint32_t *xp, uint32_t len) {
    uint32_t r = xp[len & 1023u];
    if (len >> 10) r = mulmodp_dev(r, xp[1024 + ((len >> 10) & 1023u)]);
    if (len >> 20) r = mulmodp_dev(r, xp[2048 + ((len >> 20) & 1023u)]);
    return r;
}

// crc32c(c, D) = ~(M_len(~c) ^ raw(D)), then store (MODE 0) or compare (MODE 1).
template <int MODE>
__device__ __forceinline__ void finalize(const SpanArgs &a, uint64_t item, uint32_t raw, uint32_t aux,
                                         uint32_t span_len, bool sane) {
    uint32_t init;
    if (MODE == 0 && a.lens == nullptr)
        init = mulmodp_dev(~aux, a.kspan);
    else
        init = mulmodp_dev(MODE == 0 ? ~aux : 0xffffffffu, xpow8_dev(a.xpow, span_len));
    const uint32_t crc = ~(init ^ raw);
    if (MODE == 0) {
        a.out[item] = crc;
    } else {
        const bool good = sane && crc == aux;
        a.ok[item] = good;
        if (!good) atomicAdd(a.nbad, 1ull);
    }
}

template <bool UNALIGNED, int MODE>
__global__ __launch_bounds__(1024) void k_spans(SpanArgs a, const uint4 *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImage4Bytes);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t li = lane & 31u;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t nunits = a.units ? (uint64_t)*a.nunits : a.n;
    const uint64_t ngroups_total = (uint64_t)gridDim.x * (blockDim.x >> 5);
    uint64_t u = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 2 + (lane >> 5);

    UnitDesc cur = fetch_unit<MODE>(a, u, nunits);
    UnitDesc nxt = fetch_unit<MODE>(a, u + ngroups_total, nunits);
    uint32_t k = 0;    // pair index inside cur
    uint32_t acc = 0;  // lane accumulator over the pairs of cur
    PairWin<UNALIGNED> w0, w1;
    load_pair<UNALIGNED>(w0, cur, 0, li, a.zero);

    // Process the pair held in `w` (pair k of cur) after issuing the loads of
    // the group's next pair into `wn`.  Returns false once this group is done.
    auto step = [&](PairWin<UNALIGNED> &w, PairWin<UNALIGNED> &wn) -> bool {
        const bool last = k + 1 >= cur.npairs;
        if (!last)
            load_pair<UNALIGNED>(wn, cur, k + 1, li, a.zero);
        else
            load_pair<UNALIGNED>(wn, nxt, 0, li, a.zero);

        if (cur.npairs) {
            uint32_t va[16], vb[16];
            const uint8_t *E = cur.p + cur.len;
            const uint8_t *sa = E - (size_t)kPairBytes * cur.npairs + (size_t)kPairBytes * k + kSpanCH * li;
            if constexpr (UNALIGNED) {
                const uint32_t uo = (uint32_t)((uintptr_t)E & 15u);
                realign(w.a, uo, va);
                realign(w.b, uo, vb);
            } else {
                straight(w.a, va);
                straight(w.b, vb);
            }
            // Bytes before p inside a loaded piece belong to something else.
            const int64_t lo = (int64_t)(cur.p - sa);
            if (__any(lo > 0 && ((uintptr_t)cur.p & 15u))) {
                mask_head(va, lo);
                mask_head(vb, lo - (int64_t)kRowBytes);
            }
            uint32_t s_a, s_b;
            chain16x2(va, vb, c, s_a, s_b);
            acc = xor3(apply_op<4>(kAuxOp6, acc), apply_op<4>(kAuxOp5, s_a), s_b);
        }
        if (last) {
            if (cur.valid) {
                const uint32_t raw = group_reduce32_dpp(acc, lane);
                if (li == 0) {
                    if (cur.single)
                        finalize<MODE>(a, cur.item, raw, cur.aux, cur.span_len, cur.sane);
                    else
                        a.seg_raw[cur.unit] = raw;
                }
            }
            acc = 0;
            k = 0;
            u += ngroups_total;
            cur = nxt;
            nxt = fetch_unit<MODE>(a, u + ngroups_total, nunits);
        } else {
            ++k;
        }
        return cur.valid;
    };

    for (;;) {
        if (!step(w0, w1)) break;
        if (!step(w1, w0)) break;
    }
}

// Segments per span (for the exclusive scan that places the work units).
template <int MODE>
__global__ void k_count(SpanArgs a, uint32_t *nseg) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.n;
         i += (uint64_t)gridDim.x * blockDim.x)
        nseg[i] = nseg_of(fetch_item<MODE>(a, i).len);
}

// Write unit descriptors at prefix[i].  Spans whose units would pass `cap`
// (possible only when spans overlap) are listed in `whole` and processed as
// one unit each by a second pass; *nvalid = units written before the first
// such span.
__global__ void k_expand(const uint32_t *nseg, const uint32_t *prefix, uint64_t n, uint2 *units, uint64_t cap,
                         uint32_t *nvalid, uint2 *whole, uint32_t *nwhole) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p0 = prefix[i], ns = nseg[i];
        if (p0 + ns <= cap) {
            for (uint32_t s = 0; s < ns; ++s) units[p0 + s] = make_uint2((uint32_t)i, s);
            if (i + 1 == n) *nvalid = (uint32_t)(p0 + ns);
        } else {
            if (p0 <= cap) atomicMin(nvalid, (uint32_t)p0);
            whole[atomicAdd(nwhole, 1u)] = make_uint2((uint32_t)i, kWhole);
        }
    }
}

// Fold the segment CRCs of every multi-segment span (one thread per span).
template <int MODE>
__global__ void k_combine(SpanArgs a, const uint32_t *nseg, const uint32_t *prefix, const uint32_t *nvalid,
                          uint32_t kseg) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t ns = nseg[i];
        const uint64_t p0 = prefix[i];
        if (ns <= 1 || p0 + ns > *nvalid) continue;  // single, or processed whole
        uint32_t acc = 0;
        for (uint32_t s = 0; s < ns; ++s) acc = mulmodp_dev(acc, kseg) ^ a.seg_raw[p0 + s];
        const ItemDesc it = fetch_item<MODE>(a, i);
        finalize<MODE>(a, i, acc, it.aux, it.len, it.sane);
    }
}

}  // namespace mcrc_dev
