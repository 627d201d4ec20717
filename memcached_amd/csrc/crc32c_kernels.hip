// crc32c_kernels.hip -- hand-written gfx950 kernels for batched CRC-32C.
//
// K1  k_fixed<CRCIN, NT>: equal 4 KiB, 16-B aligned items at a fixed stride
//     (extstore spill batches of one slab class; BASELINE configs 2 and 4).
//     Replaces N calls of crc32c(0, item, len), crc32c_hw (crc32c.c:161-246)
//     reached from storage.c:567.
// K2  k_spans<UNITS>: any offsets, lengths and alignment; one 32-lane group
//     per work unit of <= 128 KiB (configs 3 and 5, storage.c:172 read-back
//     spans), then k_final<MODE 0> per span.
// K3  the same kernels over the spans of packed item images in extstore
//     pages, [off+32, off+ITEM_ntotal) (k_count<MODE 1/2> parses the
//     headers): k_final<MODE 1> checks the CRC stored in the item's exptime
//     field (storage.c:160-178 over the page walk of storage.c:950-960);
//     k_final<MODE 2> stamps it (the spill CRC of storage.c:567, batched per
//     wbuf).  k_walk walks the pages on the device.
// K4  k_blocks: spans whose unit is one 4 KiB block (K1's loop, gathered).
// K5  k_lines<MODE>: spans or item images whose span is one 4 KiB window of
//     whole lines after a short head (every 4165-B image of config 5 and the
//     config-2 variant), each image's header, head and tail done once by one
//     lane of a run of consecutive images; k_fix stamps (MODE 2).
//     k_small: batches of up to 8192 spans in one launch (IO batches, wbufs,
//     the coalescing queue).
//
// See crc32c_device.h for the lane-group work model and LDS table layouts.
#include "crc32c_device.h"

namespace mcrc_dev {

// ===========================================================================
// K1: fixed-length aligned items
// ===========================================================================

// 16-B load of item bytes.  (The streaming reads of K1, K5 and the span
// kernels use ld16_nt below, since round 5 on whole lines; non-temporal
// loads of 16-B anchored blocks were 5-11 % worse in round 1.)
__device__ __forceinline__ uint4 ld16(const void *p) { return *reinterpret_cast<const uint4 *>(p); }
// Global-memory byte and piece pointers.  k_lines keeps its addresses in
// these: derived from the kernel arguments through generic pointers, they
// lost their address space to an optimizer freeze, and the flat loads that
// result also count in lgkmcnt (every LDS wait of the chains then waits for
// the block prefetch too).
typedef const __attribute__((address_space(1))) uint8_t gbyte;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16(gbyte *p) {
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Non-temporal 16-B load (the `nt` policy bit: the line is streamed, not kept
// in L2 / the Infinity Cache).
__device__ __forceinline__ uint4 ld16_nt(const uint8_t *p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld16_nt(gbyte *p) {
    const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t dw4(const uint4 &v, int k) {
    return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}

// K1 geometry: a 32-lane group owns one 4096-B item, a wave two items per
// step.
constexpr uint32_t kK1Bytes = 4096;

// K1's lane layout (round 5).  A 32-lane group owns one 4096-B item, and lane
// i holds the 16-B pieces at 512 k + 16 i, k = 0..7: each load instruction
// reads 512 contiguous bytes per group (two items, 1 KiB per wave), so every
// 128-B line is read whole by one instruction.  With non-temporal loads that
// reads 4 GiB at 82-83 % of the HBM peak, against 73-76 % for the 32-B-per-
// lane rows of rounds 1-4 (lane i at 32 i + 16 q of each KiB, two
// instructions per line) and 69-71 % for either shape with the default
// policy (profiles/r05_k1_ceiling.txt).  Algebra: the piece at 512 k + 16 i
// stands M_{512 (7-k) + 16 (31-i)} from the item's end.  Lane i runs one
// four-dword chain per piece; the chains of each half item fold through the
// shifted last steps M_1536, M_1024, M_512 (and the plain step), the first
// half moves up by M_2048, and the lane tree merges 16-B granules (levels
// M_16 .. M_128; level 4 = level 3 twice).  Table image: build_lds_image_span
// at chunk 16 (crc32c_gf2.h): tree at tables 0..15, M_2048 at 16..19, the
// shifted steps at kAuxShift2 / kAuxShift1 / kAuxShift0.
constexpr uint32_t kK1Pieces = 8, kK1Piece = 512;  // pieces per lane and item, their spacing
constexpr uint32_t kK1LaneBytes = 16;              // (the image's chunk)
static_assert(kK1Pieces * kK1Piece == 4096 && 32 * kK1LaneBytes == kK1Piece, "K1 covers a 4 KiB item");

struct K1Regs {
    uint4 d[kK1Pieces];  // piece k: item bytes [512 k + 16 i, +16) for lane i
    uint32_t cin;        // the item's initial CRC
    // wb: wave-uniform base (SGPR), loff: this lane's offset from it
    // NT: the non-temporal policy, for whole-line (128-B aligned) items; a
    // 16-B anchored block shares its end lines with its neighbours, which a
    // non-temporal load fetches twice
    template <bool NT>
    __device__ __forceinline__ void load_at(const uint8_t *__restrict__ wb, uint32_t loff) {
#pragma unroll
        for (int k = 0; k < (int)kK1Pieces; ++k)
            d[k] = NT ? ld16_nt(wb + loff + k * kK1Piece) : ld16(wb + loff + k * kK1Piece);
    }
};

// The lane value M_{2048}(u_A) ^ u_B: u_A / u_B the first / second half's
// four chains, each ended by its shifted last step.
__device__ __forceinline__ uint32_t k1_lane_value(const K1Regs &r, const LaneCtx &c) {
    constexpr uint32_t kShift[3] = {kAuxShift0, kAuxShift1, kAuxShift2};  // M_1536, M_1024, M_512
    uint32_t x[kK1Pieces];
#pragma unroll
    for (int k = 0; k < (int)kK1Pieces; ++k) x[k] = r.d[k].x;
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < (int)kK1Pieces; ++k) x[k] = step4_next(x[k], dw4(r.d[k], i), c);
#pragma unroll
    for (int k = 0; k < (int)kK1Pieces; ++k)
        x[k] = (k & 3) < 3 ? step4_last_shifted(x[k], kShift[k & 3]) : step4_next(x[k], 0u, c);
    const uint32_t ua = xor3(x[0], x[1], x[2]) ^ x[3], ub = xor3(x[4], x[5], x[6]) ^ x[7];
    return apply_op<4>(kAuxSpanFold, ua) ^ ub;
}

// Half an item's pieces for one lane (pieces 4 q .. 4 q + 3 of half q).
struct K1Half {
    uint4 d[4];
    uint32_t cin;  // (half 0) the item's initial CRC
};
// The value of half Q: its four chains, each ended by its shifted last step
// (M_1536, M_1024, M_512, plain: the half's pieces stand 512 (3 - k) from its
// end); the item's lane value is M_2048(u_0) ^ u_1 (k1_lane_value).
__device__ __forceinline__ uint32_t k1_half_value(const K1Half &r, const LaneCtx &c) {
    constexpr uint32_t kShift[3] = {kAuxShift0, kAuxShift1, kAuxShift2};
    uint32_t x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = r.d[k].x;
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = step4_next(x[k], dw4(r.d[k], i), c);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = k < 3 ? step4_last_shifted(x[k], kShift[k]) : step4_next(x[k], 0u, c);
    return xor3(x[0], x[1], x[2]) ^ x[3];
}

// NT: non-temporal loads, for a 128-B aligned base and stride (every line
// whole in one item); otherwise the default policy, so that a line two
// neighbouring items share is not fetched twice (K1Regs::load_at).
template <bool CRCIN, bool NT>
__global__ __launch_bounds__(1024) void k_fixed(const uint8_t *__restrict__ base, uint64_t stride,
                                                uint64_t nitems, const uint4 *__restrict__ img,
                                                const uint32_t *__restrict__ crc_in,
                                                uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
    constexpr uint32_t IPW = 2;  // items per wave and step
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t li = lane & 31u;
    const uint32_t g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t gstep = gridDim.x * waves;
    const uint64_t ngroups = (nitems + IPW - 1) / IPW;
    // wave-uniform (SGPR) group index: the loop exits are then scalar
    // branches, and the waitcnt pass sees one path into the loop header (a
    // divergent exit merged an un-waited path there and forced vmcnt(0),
    // which drained the prefetched step).
    uint64_t grp = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6));
    // the ranges dealt to the waves in a scrambled order: wave w takes range
    // (w * 65521) mod W (65521 is prime: a bijection unless it divides W), so
    // a CU's 16 waves stream ranges far apart rather than 16 neighbouring
    // MiB: -0.6 % at 1 and 4 Mi items in every round
    // (profiles/r04_ablations/k1_range_order_ab.txt)
    if (gstep % 65521u) grp = (grp * 65521u) % gstep;
    // wave w takes the contiguous groups [w cg, (w + 1) cg): 1.0-1.4 % faster
    // than the grid-stride order at 1 Mi items, 0.6-3.7 % at 4 Mi, on two
    // boxes (profiles/r04_ablations/k1_chunk_and_census_ab.txt,
    // k1_item_order_ab.txt); a range per workgroup with its waves interleaved
    // was 4.5 % slower
    const uint64_t cg = (ngroups + gstep - 1) / gstep;
    const uint64_t gend = min((grp + 1) * cg, ngroups);
    grp *= cg;
    if (grp >= ngroups) return;
    const uint64_t glast = gend - 1;
    auto item_of = [&](uint64_t gi) { return gi * IPW + g; };

    // The loads run three half-steps ahead: a ring of four half-buffers (the
    // registers of two whole steps), so while one half is checksummed the
    // next three (12 KiB per wave) are in flight.  Uniform step base +
    // per-lane offset: no 64-bit VGPR address math at the top of a step.  A
    // wave's last prefetches run past its last group; they read the table
    // image instead (in L2 since every workgroup copied it; their results are
    // not used): re-reading the wave's last group fetched it from HBM again
    // (non-temporal loads), 0.7 % of the launch's bytes, and clamping every
    // wave to the batch's last group made 4096 waves read the same 8 KiB at
    // the end of the launch.  The sched_barrier keeps the loads where they
    // are issued: left alone, the scheduler sinks them into the chains and
    // the next half waits on loads issued moments before.
    auto ldh = [&](K1Half &r, uint64_t gi, int q) {
        const bool real = gi < gend;  // (wave-uniform)
        const uint64_t gu = real ? gi : glast;
        const uint64_t first = gu * IPW;
        const uint8_t *wb = real ? base + first * stride : reinterpret_cast<const uint8_t *>(img);
        const uint32_t gl = first + g < nitems ? g : (uint32_t)(nitems - 1 - first);
        // crc_in first: it is consumed before the first chain step, and
        // vmcnt counts in issue order
        if (q == 0) {
            if constexpr (CRCIN) r.cin = crc_in[first + gl];
            else r.cin = 0u;
        }
        const uint32_t loff = (real ? gl * (uint32_t)stride : g * kK1Bytes) + li * kK1LaneBytes + 4u * kK1Piece * (uint32_t)q;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            r.d[k] = NT ? ld16_nt(wb + loff + k * kK1Piece) : ld16((gbyte *)(wb + loff + k * kK1Piece));
        __builtin_amdgcn_sched_barrier(0);
    };
    // lane 0 XORs ~crc_in into the item's first dword (a register seeded
    // with ~crc_in, crc32c.c:166)
    auto half0 = [&](K1Half &m) {
        if (li == 0) m.d[0].x ^= ~m.cin;
        return apply_op<4>(kAuxSpanFold, k1_half_value(m, c));
    };
    auto part0 = [&](uint32_t u0, K1Half &m1) {
        return reduce_level<0>(u0 ^ k1_half_value(m1, c), (lane & 1u) == 0u);
    };
    K1Half h0, h1, h2, h3;
    // Step k's halves live in h0/h1 (k even) or h2/h3 (k odd).  Before step k
    // is checksummed, its two halves and step k + 1's first are issued; each
    // half's checksum is preceded by the issue of the half three later.
    const uint64_t nsteps = gend - grp;
    ldh(h0, grp, 0);
    ldh(h1, grp, 1);
    ldh(h2, grp + 1, 0);
    // (even step k at grp: h0/h1 -> issue h3 (k+1, B), h0 (k+2, A))
    auto step_even = [&](uint64_t s) {
        ldh(h3, s + 1, 1);
        const uint32_t u0 = half0(h0);
        ldh(h0, s + 2, 0);
        return part0(u0, h1);
    };
    auto step_odd = [&](uint64_t s) {
        ldh(h1, s + 1, 1);
        const uint32_t u0 = half0(h2);
        ldh(h2, s + 2, 0);
        return part0(u0, h3);
    };
    // One exit, at the bottom of each loop: a break between the halves would
    // give the loop header a second (un-waited) predecessor, and the waitcnt
    // pass would then drain every prefetched load there.
    uint64_t k = 0;
    for (; k + 4 <= nsteps; k += 4) {
        const uint32_t va = step_even(grp);
        const uint32_t vb = step_odd(grp + 1);
        const uint32_t vab = group_pair_level1(va, vb, lane);
        const uint32_t vc = step_even(grp + 2);
        const uint32_t vd = step_odd(grp + 3);
        const uint32_t raw = group_reduce32_quad_span(vab, group_pair_level1(vc, vd, lane), lane);
        const uint64_t item = item_of(grp + (li & 3u));
        if (li < 4 && item < nitems) out[item] = ~raw;
        grp += 4;
    }
    for (; k + 2 <= nsteps; k += 2) {
        const uint32_t va = step_even(grp);
        const uint32_t vb = step_odd(grp + 1);
        const uint32_t raw = group_reduce32_pair_span(va, vb, lane);
        const uint64_t item = item_of(li == 0 ? grp : grp + 1);
        if (li < 2 && item < nitems) out[item] = ~raw;
        grp += 2;
    }
    if (nsteps & 1) {
        uint32_t v = step_even(grp);
        v = reduce_level<1>(v, (lane & 3u) == 0u);
        v = reduce_level<2>(v, (lane & 7u) == 0u);
        v = reduce_level<3>(v, (lane & 15u) == 0u);
        const uint32_t raw = reduce_level4_span(v, (lane & 31u) == 0u);
        const uint64_t item = item_of(grp);
        if (li == 0 && item < nitems) out[item] = ~raw;
    }
}

// ===========================================================================
// K2/K3: arbitrary spans, one 32-lane group per work unit
// ===========================================================================
//
// Pieces as they lie.  A span D = [p, E) is read as the 16-B aligned pieces
// [ph, Ea), ph = p rounded down to 16 and Ea = E rounded up to a 128-B line
// (grid_pad, round 5; 16 before), the head's foreign bytes F_h = [ph, p)
// included and the tail's F_t = [E, Ea) cleared in registers (the last line
// of the span's last block, mask_tail; round 5): the span kernel computes
// R = raw([ph, E) followed by t = |F_t| zeros) with no initial value.  The
// algebra of crc32c.c:58-137 gives
//   R = M_{|D|+t}(raw(F_h)) ^ M_t(raw(D)), so
//   crc32c(c, D) = ~M_{-t}(R ^ Z),   Z = M_{|D|+t}(~c ^ raw(F_h)).
// Z depends only on c and the at most 15 bytes of F_h, which share the head
// piece (and for item images the header's line), so one thread per span
// computes it (span_corr: k_count before the span kernel, or k_final after
// it), at a thirty-second of the cost of doing it in a 32-lane group; the
// span kernel's per-unit work is its lane reduction and one store.  (Until
// round 5 the thread also read F_t and XORed raw(F_t) into Z: a line per
// span that the span kernel reads again.)
//
// Work units.  A virtual span longer than kSegBytes is cut into segments of
// kSegBytes anchored at Ea (segment 0, the head, holds the remainder: 17 B to
// kSegBytes + 16 B); every segment is one work unit, so no group owns much
// more than 64 KiB and a batch of
// Zipf-sized items balances over the grid.  Units come from k_count ->
// exclusive scan -> k_expand; a batch whose spans all fit one unit uses unit
// u = span u directly.  Segment units shift their value into place and XOR it
// into the span's accumulator:
//   R(span) = sum_s M_{kSegBytes * (nseg-1-s)}(R(segment s)),
// then k_final turns R into the CRC (or the verdict) of every span.
//
// Unit geometry (the K1 geometry: CH = 32, LPI = 32): a unit [p, e), e
// 16-aligned, is covered by `niters` blocks of 4 KiB anchored at e; block k
// covers [G + 4096k, G + 4096(k+1)), G = e - 4096 * niters, as four 1 KiB rows.
// Lane li owns bytes [32 li, 32 li + 32) of every row (two 16-B pieces) and
// runs one chain per row; rows wholly before p (for every lane of the wave)
// are skipped.  Per block a lane folds
//   acc = M_4096(acc) ^ (((s0 M_1024 ^ s1) M_1024 ^ s2) M_1024 ^ s3),
// and the lane accumulators merge in the K1 lane-group reduction.
//
// Loads are 16-B aligned pieces that overlap [p, E) (so they never leave the
// pages holding the span); a piece wholly outside is read from a zeroed device
// buffer instead, so no load is predicated.

constexpr uint32_t kRowBytes = 1024;  // a row: two of K1's 512-B piece rows (the head-block skip)
constexpr uint32_t kBlockBytes = 4 * kRowBytes;  // 4096
// (round 5: 128 KiB; config 3 -1.1..-1.3 % against 64 KiB in two sessions, the
// mixed pages and config 5 within noise, 256 KiB like 128 --
// profiles/r05_ablations/segment_size_ab.txt; rounds 1-3 found 24-64 KiB alike)
constexpr uint32_t kSegBytes = 128 * 1024;
// Longest span (CRC32C_MAX_SPAN): a unit's grid offsets (eo, G - p, the block
// count times 4 KiB) are 32-bit and signed, and a span that overlaps others
// past the plan's capacity is one unit.  Twice the largest item memcached
// stores (ITEM_SIZE_MAX_UPPER_LIMIT = 1 GiB, memcached.h:115).  Longer spans
// are not read (out = 0, counted as out of range / malformed).
constexpr uint32_t kMaxSpan = 0x7fff0000u;
constexpr uint32_t kWhole = 0xffffffffu;      // unit segment index: the whole span
// Pieces outside a span are read from a zeroed buffer; workgroup b reads the
// 16 B at zero + 4 KiB * (b % 256), so the workgroups' zero reads spread over
// L2 channels instead of all landing on one line (cf. K1's last prefetch).
constexpr uint32_t kZeroSlots = 256;
constexpr uint64_t kZeroBytes = 4096ull * kZeroSlots;

// Rows of the shift table (SpanArgs::segpow) below its second-factor rows:
// units ending less than 16 MiB before their span's end take one multiply.
constexpr uint32_t kSegpowLo = 4096;

struct SpanArgs {
    const uint8_t *base;       // all spans live in [base, base + base_bytes)
    uint64_t base_bytes;
    const uint64_t *offsets;   // span i starts at base + offsets[i] (MODE 0)
                               // or item image i at base + offsets[i] (MODE 1)
    uint64_t stride;           // when offsets == nullptr: base + i * stride
    const uint32_t *lens;      // per-span lengths, or nullptr: every span is `len`
    uint32_t len;
    const uint32_t *crc_in;    // MODE 0: per-span initial CRC or nullptr (0)
    uint32_t *out;             // MODE 0: CRC per span
    uint8_t *ok;               // MODE 1: 1 if the stored CRC matches
    unsigned long long *nbad;  // MODE 1/2: count of mismatches / malformed images;
                               // MODE 0: spans outside [base, base + base_bytes) (atomic)
    uint64_t n;                // spans (items)
    const uint32_t *xpow;      // x^(8*j), x^(8*1024*j), x^(8*2^20*j) (3 x 1024), x^(-8t) (16),
                               // x^(8*2^30*j) (8): layout kXpow*
    const uint32_t *tab8;      // 16 x 256 byte tables (Tab8)
    const uint4 *zero;         // kZeroBytes of zeros in device memory
    // work units (nullptr: unit u = span u, one segment)
    const struct UnitRec *units;
    const uint32_t *nunits;    // device-side unit count
    uint32_t *span_acc;        // planned batches: R per span (segment units XOR their shifted values in)
    const uint32_t *segpow;    // rows k (x^i * x^(8 * 4096 * k), i < 32) for k < kSegpowLo, then k = kSegpowLo j
    const uint32_t *starts;    // balanced plan: share v's records are [starts[v], starts[v + 1])
                               // (0xffffffff: *nunits); nullptr: round robin over units
    uint32_t rounds;           // balanced plan: group g takes shares g, G + g, .. (rounds of them)
    uint64_t region;           // MODE 1: items never cross a multiple of `region` (0: no bound)
    uint32_t cfl;              // MODE 1/2: bytes of the ITEM_CFLAGS suffix, sizeof(client_flags_t):
                               // 4, or 8 in a LARGE_CLIENT_FLAGS build (memcached.h:96-100)
    // k_small only (nullptr: nbad is the caller's to zero and read): the last
    // workgroup moves *nbad to this pinned host word and zeroes *nbad and *done
    unsigned long long *host_nbad;
    uint32_t *done;            // finished workgroups
    // planned path over a list whose length is known only on the device (K5's
    // fallback list): n spans at most, *dn of them (nullptr: n)
    const uint32_t *dn;
};

__device__ __forceinline__ uint64_t span_count(const SpanArgs &a) { return a.dn ? (uint64_t)*a.dn : a.n; }

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

// t = Ea - E: a span's grid ends at Ea = E rounded up to 16.  (Rounding up to
// a 128-B line makes every block whole lines -- a 16-B anchored block fetches
// 33 lines per 4 KiB -- and the span kernel 1.6-2.4 % faster, but the span's
// thread then reads and folds up to 127 foreign bytes: k_count +40 %, k_final
// +57 %, a net loss on configs 2r and 5.)
constexpr uint32_t kTailAlign = 16;
__device__ __forceinline__ uint32_t tail_pad(const uint8_t *p, uint32_t len) {
    return (uint32_t)(-(uintptr_t)(p + len)) & (kTailAlign - 1);
}
// The planned path's grid (round 5): anchored at Ea = E rounded up to a
// 128-B line, so every block of a unit is whole lines and the span kernel's
// non-temporal loads never share a line between two instructions; the
// span's thread folds up to 127 foreign tail bytes instead of 15.
constexpr uint32_t kGridAlign = 128;
__device__ __forceinline__ uint32_t grid_pad(const uint8_t *p, uint32_t len) {
    return (uint32_t)(-(uintptr_t)(p + len)) & (kGridAlign - 1);
}

// Segments of a virtual span of vlen bytes, anchored at Ea; the head segment
// keeps the remainder (17 B up to kSegBytes + 16 B).
__device__ __forceinline__ uint32_t nseg_of(uint32_t vlen) {
    return vlen <= kSegBytes + 16 ? 1u : (vlen - 16 + kSegBytes - 1) / kSegBytes;
}

// Layout of the x^(8n) table (SpanArgs::xpow).
constexpr uint32_t kXpowInv = 3072;                // x^(-8t), t < kGridAlign
constexpr uint32_t kXpowL3 = kXpowInv + kGridAlign;  // x^(8 * 2^30 * j), j < 8
constexpr uint32_t kXpowDwords = kXpowL3 + 8;

// x^(8n) mod P (n < 2^33): one to four table entries multiplied.
__device__ __forceinline__ uint32_t xpow8_dev(const uint32_t *xp, uint64_t n) {
    uint32_t r = xp[n & 1023u];
    if (n >> 10) r = mulmodp_dev(r, xp[1024 + ((n >> 10) & 1023u)]);
    if (n >> 20) r = mulmodp_dev(r, xp[2048 + ((n >> 20) & 1023u)]);
    if (n >> 30) r = mulmodp_dev(r, xp[kXpowL3 + (uint32_t)(n >> 30)]);
    return r;
}

// A 16-B piece as two little-endian halves.
struct Piece {
    uint64_t lo, hi;
};
__device__ __forceinline__ Piece ld_piece(const uint8_t *p) {
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    return {v.x | ((uint64_t)v.y << 32), v.z | ((uint64_t)v.w << 32)};
}
__device__ __forceinline__ Piece ld_piece(gbyte *p) {
    const uint4 v = ld16(p);
    return {v.x | ((uint64_t)v.y << 32), v.z | ((uint64_t)v.w << 32)};
}
// Bytes moved s positions up (s <= 16), zeros shifted in.
__device__ __forceinline__ Piece shl_bytes(Piece v, uint32_t s) {
    if (s >= 16) return {0, 0};
    if (s >= 8) return {0, v.lo << (8 * (s - 8))};
    if (s == 0) return v;
    return {v.lo << (8 * s), (v.hi << (8 * s)) | (v.lo >> (64 - 8 * s))};
}
// Byte tables in LDS for the per-thread work of k_count / k_final: T_j[b] =
// the register after byte b followed by j zero bytes, j < 16 (T_0 is
// crc32c.c:399's byte-wise table crc32c_table_little[0]; crc32c.c:401-415 uses
// eight of them).  A whole 16-B piece is one step of 16 independent lookups:
// only the four that read the running register depend on the previous step,
// so a thread's chain is one LDS latency per 16 bytes.  (A dword per step
// took 0.21 ms of k_count on config 3, a copy of one table per bank with four
// dependent lookups per dword 0.45 ms: the per-thread chains are
// latency-bound, not conflict-bound.)
struct Tab8 {
    const uint32_t *s;  // T_j at s + 256 j
    __device__ __forceinline__ uint32_t T(uint32_t j, uint32_t b) const { return s[256 * j + b]; }
    // the register r advanced over the 16 bytes of v
    __device__ __forceinline__ uint32_t piece(uint32_t r, Piece v) const {
        const uint32_t x = r ^ (uint32_t)v.lo, d1 = (uint32_t)(v.lo >> 32), d2 = (uint32_t)v.hi,
                       d3 = (uint32_t)(v.hi >> 32);
        return (T(15, x & 255u) ^ T(14, (x >> 8) & 255u) ^ T(13, (x >> 16) & 255u) ^ T(12, x >> 24)) ^
               (T(11, d1 & 255u) ^ T(10, (d1 >> 8) & 255u) ^ T(9, (d1 >> 16) & 255u) ^ T(8, d1 >> 24)) ^
               (T(7, d2 & 255u) ^ T(6, (d2 >> 8) & 255u) ^ T(5, (d2 >> 16) & 255u) ^ T(4, d2 >> 24)) ^
               (T(3, d3 & 255u) ^ T(2, (d3 >> 8) & 255u) ^ T(1, (d3 >> 16) & 255u) ^ T(0, d3 >> 24));
    }
    // M_4096(r): operator tables 16..19 (slice k: M_4096 of byte b at bits 8k)
    __device__ __forceinline__ uint32_t block(uint32_t r) const {
        return (T(16, r & 255u) ^ T(17, (r >> 8) & 255u)) ^ (T(18, (r >> 16) & 255u) ^ T(19, r >> 24));
    }
    // M_n(r): the register r advanced over n zero bytes, 0 <= n <= 16
    __device__ __forceinline__ uint32_t zeros(uint32_t r, uint32_t n) const {
        if (n >= 4)
            return T(n - 1, r & 255u) ^ T(n - 2, (r >> 8) & 255u) ^ T(n - 3, (r >> 16) & 255u) ^ T(n - 4, r >> 24);
        uint32_t z = n == 0 ? r : r >> (8 * n);  // the bytes not yet shifted out
        for (uint32_t k = 0; k < n; ++k) z ^= T(n - 1 - k, (r >> (8 * k)) & 255u);
        return z;
    }
};
constexpr uint32_t kTab8Dwords = 20 * 256;  // 16 byte tables + the M_4096 operator, 20 KiB
// (every thread of the block calls it)
// (s: 16-B aligned; 16-B pieces, every load of a thread issued before its
// stores, as load_tables)
__device__ __forceinline__ Tab8 load_tab8(uint32_t *s, const uint32_t *tab8) {
    constexpr uint32_t n = kTab8Dwords / 4, U = 8;
    uint4 *dst = reinterpret_cast<uint4 *>(s);
    const uint4 *src = reinterpret_cast<const uint4 *>(tab8);
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += U * blockDim.x) {
        uint4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = src[min(i0 + u * blockDim.x, n - 1)];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) dst[min(i0 + u * blockDim.x, n - 1)] = v[u];
    }
    __syncthreads();
    return {s};
}

// Register after the 16 bytes of v from a zero register.
__device__ __forceinline__ uint32_t raw16(Piece v, const Tab8 &t) { return t.piece(0u, v); }

// Bytes [0, k) of v cleared.
__device__ __forceinline__ Piece clear_below(Piece v, uint32_t k) {
    const Piece m = shl_bytes({~0ull, ~0ull}, k);
    return {v.lo & m.lo, v.hi & m.hi};
}

// Register r advanced over the n bytes at p (one thread), one step per 16-B
// piece: a partial first or last piece is moved to the top of a zeroed piece
// (leading zeros leave a zero register unchanged), so
//   r' = M_m(r) ^ raw16(the m bytes at the top).
// Every load is an aligned piece holding a byte of [p, p + n).
constexpr int kAdvUnroll = 4;  // (8 and 16 measured slower: profiles/r04_ablations/k_count_unroll_ab.txt)
__device__ __forceinline__ uint32_t reg_advance(uint32_t r, const uint8_t *p, uint32_t n, const Tab8 &t) {
    if (n == 0) return r;
    const uint32_t kh = (uint32_t)((uintptr_t)p & 15u);
    const uint8_t *q = p - kh;
    if (kh + n <= 16u) {  // inside one piece: bytes [kh, kh + n)
        const Piece v = shl_bytes(ld_piece(q), 16u - kh - n);
        return t.zeros(r, n) ^ raw16(clear_below(v, 16u - n), t);
    }
    if (kh) {  // bytes [kh, 16) of the first piece
        r = t.zeros(r, 16u - kh) ^ raw16(clear_below(ld_piece(q), kh), t);
        n -= 16u - kh;
        q += 16;
    }
#pragma unroll kAdvUnroll
    for (; n >= 16; n -= 16, q += 16) r = t.piece(r, ld_piece(q));
    if (n) r = t.zeros(r, n) ^ raw16(shl_bytes(ld_piece(q), 16u - n), t);  // bytes [0, n) of the last piece
    return r;
}

// Head fragment.  The block grid of a span is anchored at Ea, 4 KiB apart
// (segments are whole numbers of blocks, so every unit of the span uses the
// same grid); G1 = the first grid point after ph.  The span kernel would
// spend a whole block step of its group on [p, G1), mostly on rows without a
// byte of the span; when G1 - p <= kFragMax the span's thread takes those
// bytes instead (reg_advance), the head unit starts at G1, and a span whose
// virtual length is at most kWholeMax is not given to the span kernel at all.
// (The limits are measured: a thread's chain is serial, one LDS round trip
// per 16 B, so long fragments cost more than the block step they save --
// DESIGN.md section 3.)
constexpr uint32_t kFragMax = 128;    // a head fragment [p, G1) of at most this
// (512 since round 5: 256-512 beat 1024 by 1.0-1.3 % on the mixed pages and
// matched it on config 3; 2048 / 3072 were 1-3 % slower --
// profiles/r05_ablations/whole_span_limit_ab.txt)
constexpr uint32_t kWholeMax = 512;   // a whole span of vlen at most this
static_assert(kWholeMax + kGridAlign <= kBlockBytes, "a whole span held by its thread is its own fragment (G1 = Ea)");
// Is the head fragment (G1 - p = g1o) the span thread's?  For vlen <= kWholeMax
// the fragment is the whole span (G1 = Ea).
__device__ __forceinline__ bool frag_drop(uint32_t len, uint64_t g1o, uint64_t vlen) {
    return len != 0 && (g1o <= kFragMax || vlen <= kWholeMax);
}
struct SpanHead {
    uint64_t g1o;  // G1 - p
    bool drop;     // [p, G1) is the thread's
};
__device__ __forceinline__ SpanHead span_head(const uint8_t *p, uint32_t len) {
    const uint64_t kh = (uintptr_t)p & 15u;
    const uint64_t x = (uint64_t)len + grid_pad(p, len) + kh;  // Ea - ph
    const uint64_t g1o = x - kBlockBytes * ((x - 1) / kBlockBytes) - kh;
    return {g1o, frag_drop(len, g1o, x - kh)};
}

// One-block geometry of span [p, p + len): true if its unit is one whole block
// (at G1 when its head fragment is the thread's, else at ph; *g1 = the block),
// or it has no unit at all (*none); false: neither.
__device__ __forceinline__ bool one_block(const uint8_t *p, uint32_t len, const uint8_t **g1, bool *none) {
    const uint64_t kh = (uintptr_t)p & 15u;
    const uint64_t vlen = (uint64_t)len + grid_pad(p, len);  // (64-bit: len may be close to 2^32)
    const uint64_t x = vlen + kh;  // Ea - ph
    const uint64_t g1o = x - kBlockBytes * ((x - 1) / kBlockBytes) - kh;
    const bool drop = frag_drop(len, g1o, vlen);
    *none = len == 0 || (drop && g1o == vlen);
    if (!drop && x == kBlockBytes) {  // the unit [ph, Ea) is itself one block
        *g1 = p - kh;
        return true;
    }
    *g1 = p + g1o;
    return *none || (drop && vlen - g1o == kBlockBytes);
}

// Z of span [p, p + len) with initial CRC c (see "Pieces as they lie"), for
// the R that the span kernel computes over the span's units (F_t cleared):
// - no bytes: the kernel reads nothing (R = 0), Z = M_t(~c);
// - head fragment taken (span_head): the kernel reads [G1, Ea), so
//   Z = M_{Ea-G1}(r) with r = the register from ~c over [p, G1),
//   or, when G1 = Ea, Z = M_t(register from ~c over D);
// - otherwise Z = M_{len+t}(~c ^ raw(F_h)): raw(F_h) = raw of the head
//   piece's first kh bytes moved to its top (leading zeros leave a zero
//   register unchanged).
// One thread.  (`pieces`: the third case whatever the head -- k_count's
// wave-cooperative whole spans, whole_chunks, whose R covers [ph, Ea).)
//
// Z as a register y to be moved up by N bytes: Z = M_N(y).  Every case of
// span_corr is of this form, so a wave whose spans take different cases
// (a head fragment taken or not) runs the multiply by x^(8N) once, not once
// per case (round 5: in k_count the divergent cases each ran theirs).
struct CorrArg {
    uint32_t y;
    uint64_t N;
};
__device__ __forceinline__ CorrArg span_corr_arg(const uint8_t *p, uint32_t len, uint32_t c, const Tab8 &t8,
                                                 bool pieces) {
    const uint32_t t = grid_pad(p, len);
    if (len == 0) return {~c, t};
    const uint64_t vlen = (uint64_t)len + t;
    const SpanHead h = span_head(p, len);
    if (pieces || !h.drop) {
        // the kernel's R covers the pieces [ph, Ea): y = ~c ^ raw(F_h), N = len + t
        const uint32_t kh = (uint32_t)((uintptr_t)p & 15u);
        uint32_t y = ~c;
        if (kh) y ^= raw16(shl_bytes(ld_piece(p - kh), 16 - kh), t8);  // raw(F_h)
        return {y, vlen};
    }
    // the head fragment [p, G1) is the thread's; G1 = Ea: the whole span,
    // whose register moves up by t
    const bool all = h.g1o == vlen;
    return {reg_advance(~c, p, all ? len : (uint32_t)h.g1o, t8), all ? (uint64_t)t : vlen - h.g1o};
}
__device__ __forceinline__ uint32_t corr_apply(const CorrArg &z, const Tab8 &t8, const uint32_t *xp) {
    // (one block, every one-block span: a table step)
    return z.N == kBlockBytes ? t8.block(z.y) : mulmodp_dev(z.y, xpow8_dev(xp, z.N));
}
__device__ __forceinline__ uint32_t span_corr(const uint8_t *p, uint32_t len, uint32_t c, const Tab8 &t8,
                                              const uint32_t *xp) {
    return corr_apply(span_corr_arg(p, len, c, t8, false), t8, xp);
}

// Item header fields (memcached.h:613-636) from bytes 28..43 of the image at
// it, read as the two aligned pieces holding them (every byte of those pieces
// shares its 16-B granule with a header byte, so no read leaves the image's
// pages).  ITEM_ntotal as memcached.h:149-152.
struct ItemHdr {
    uint32_t exptime;  // bytes 28..31: the spill CRC (storage.c:567)
    uint32_t nbytes;   // 32..35
    uint32_t flags;    // it_flags, 38..39
    uint32_t nkey;     // 41
    // cfl = sizeof(client_flags_t) (SpanArgs::cfl)
    __device__ __forceinline__ uint64_t ntotal(uint32_t cfl) const {
        return 48ull + nkey + 1 + nbytes + ((flags & 256u) ? cfl : 0) + ((flags & 2u) ? 8 : 0);
    }
};
//
// The fields are funnelled out of the pieces' dwords with v_alignbyte_b32, not
// with 64-bit shifts: a v_lshlrev_b64 whose shift amount sits in the last VGPR
// of the wave's allocation computes wrongly beside a co-resident wave on
// gfx950 (tools/shift64_top_vgpr.hip), and the 64-bit funnel
// this parse used through round 5 put its amount exactly there in a 24-VGPR
// kernel.  tests/test_kernel_resources.py checks that no kernel of the
// library, and no instruction of this parse, takes that form.
template <typename BytePtr>
__device__ __forceinline__ ItemHdr parse_hdr(BytePtr it) {
    // (pointer arithmetic, not an integer round trip: the loads stay global
    // loads instead of flat ones, which would also count in lgkmcnt)
    const uint32_t sh = (uint32_t)((uintptr_t)(it + 28) & 15u);  // 0..15
    const BytePtr q = it + 28 - sh;
    const bool two = sh + 13 >= 16;  // byte 41 lies in the next piece
    const Piece v0 = ld_piece(q), v1 = ld_piece(q + (two ? 16 : 0));
    const uint32_t d[8] = {(uint32_t)v0.lo, (uint32_t)(v0.lo >> 32), (uint32_t)v0.hi, (uint32_t)(v0.hi >> 32),
                           two ? (uint32_t)v1.lo : 0u, two ? (uint32_t)(v1.lo >> 32) : 0u,
                           two ? (uint32_t)v1.hi : 0u, two ? (uint32_t)(v1.hi >> 32) : 0u};
    // w[m] = the dword holding image byte 28 + 4m (and the next one's low bytes)
    const uint32_t qi = sh >> 2, b = sh & 3u;
    uint32_t w[5];
#pragma unroll
    for (uint32_t m = 0; m < 5; ++m) w[m] = qi == 0 ? d[m] : qi == 1 ? d[m + 1] : qi == 2 ? d[m + 2] : d[m + 3];
    // image bytes 28..31, 32..35, 36..39 (it_flags 38..39), 40..43 (nkey 41)
    const uint32_t o0 = __builtin_amdgcn_alignbyte(w[1], w[0], b), o1 = __builtin_amdgcn_alignbyte(w[2], w[1], b),
                   o2 = __builtin_amdgcn_alignbyte(w[3], w[2], b), o3 = __builtin_amdgcn_alignbyte(w[4], w[3], b);
    return {o0, o1, (o2 >> 16) & 0xffffu, (o3 >> 8) & 0xffu};
}

// The CRC span of the item image at base + off with header h (parsed when
// hdr_ok): [off + 32, off + ITEM_ntotal) (STORE_OFFSET, storage.h:43), the
// stored CRC in aux.
__device__ __forceinline__ ItemDesc item_desc(const SpanArgs &a, uint64_t off, const ItemHdr &h, bool hdr_ok) {
    ItemDesc d;
    const uint64_t ntotal = h.ntotal(a.cfl);
    d.aux = h.exptime;
    // an item never crosses its write buffer (extstore.c:627-636), so a
    // header claiming otherwise is corrupt
    const bool in_region = a.region == 0 || off / a.region == (off + ntotal - 1) / a.region;
    d.sane = hdr_ok && h.nkey != 0 && h.nbytes < 0x80000000u && ntotal - 32 <= kMaxSpan &&
             off + ntotal <= a.base_bytes && in_region;
    d.p = a.base + off + 32;
    d.len = d.sane ? (uint32_t)(ntotal - 32) : 0u;
    return d;
}

template <int MODE>
__device__ __forceinline__ ItemDesc fetch_item(const SpanArgs &a, uint64_t i) {
    const uint64_t off = a.offsets ? a.offsets[i] : i * a.stride;
    if (MODE == 0) {
        // a span outside [base, base + base_bytes) is not read (out = 0, counted)
        ItemDesc d;
        const uint32_t len = a.lens ? a.lens[i] : a.len;
        d.sane = off <= a.base_bytes && len <= a.base_bytes - off && len <= kMaxSpan;
        d.p = a.base + (d.sane ? off : 0);
        d.len = d.sane ? len : 0u;
        d.aux = a.crc_in ? a.crc_in[i] : 0u;
        return d;
    }
    const bool hdr_ok = off + 48 <= a.base_bytes;
    ItemHdr h{0u, 0u, 0u, 0u};
    if (hdr_ok) h = parse_hdr(a.base + off);
    return item_desc(a, off, h, hdr_ok);
}

// Work-unit record written by k_expand (32 B, one dwordx4 pair per unit):
//   a = {offset of the unit's first byte from base (lo, hi), e - p, E - p}
//   b = {z (the span's item record), span index, flags | niters << 8,
//        4 KiB blocks from e to the span's end: (kSegBytes / 4 KiB) (nseg - 1 - segment), more for a piece}
struct alignas(16) UnitRec {
    uint4 a, b;
};

// Item record written by k_count: {offset of the span (lo, hi | !sane << 31), len, z}:
// z = Z (span_corr; MODE 0 and 2) or, for a verify (MODE 1), W = Z ^ M_t(~stored CRC),
// so that the stored CRC matches iff R == W.
constexpr uint32_t kInsane = 0x80000000u;

// Decoded descriptor of one work unit (two are live per lane).
struct UnitDesc {
    const uint8_t *p;  // first byte of this unit
    uint32_t eo;       // e - p: e = 16-aligned end of this unit's grid
    uint32_t nf;       // niters << 12 | tail << 4 | flags (tail: bytes of F_t before e, the
                       // span's grid end, when this unit ends there; else 0)
    uint32_t raw;      // this lane's dword li & 7 of the unit's raw record: span index (dword 5)
                       // and segment (dword 7) are gathered from it when the unit ends
    static constexpr uint32_t kValid = 1, kSingle = 2, kHead = 4, kSane = 8;
    static constexpr uint32_t kNitersShift = 12, kTailShift = 4;
    __device__ __forceinline__ uint32_t niters() const { return nf >> kNitersShift; }
    __device__ __forceinline__ uint32_t tail() const { return (nf >> kTailShift) & 127u; }
    __device__ __forceinline__ bool valid() const { return nf & kValid; }
    __device__ __forceinline__ bool single() const { return nf & kSingle; }
    __device__ __forceinline__ bool head() const { return nf & kHead; }
    __device__ __forceinline__ bool sane() const { return nf & kSane; }
};

// Unit (segment `seg` of span [base + off, +len), or the whole span) as a record.
__device__ __forceinline__ UnitRec make_unit(const uint8_t *base, uint64_t off, uint32_t len, uint32_t aux,
                                             bool sane, uint32_t item, uint32_t seg) {
    const uint8_t *p0 = base + off;
    const uint32_t vlen = len + grid_pad(p0, len);
    const uint32_t nseg = seg == kWhole ? 1u : nseg_of(vlen);
    const bool single = nseg == 1, head = single || seg == 0;
    const uint32_t eo0 = vlen - (single ? 0u : (nseg - 1 - seg) * kSegBytes);  // e - p0
    uint32_t po = head ? 0u : eo0 - kSegBytes;                                // p - p0
    if (head) {  // a head fragment taken by the span's thread: the unit starts at G1
        const SpanHead h = span_head(p0, len);
        if (h.drop) po = (uint32_t)h.g1o;
    }
    const uint32_t eo = eo0 - po;
    const uint32_t niters = len ? (eo + (uint32_t)((uintptr_t)(p0 + po) & 15u) + kBlockBytes - 1) / kBlockBytes : 0u;
    const uint64_t o = off + po;
    UnitRec r;
    r.a = make_uint4((uint32_t)o, (uint32_t)(o >> 32), eo, len - po);
    r.b = make_uint4(aux, item,
                     UnitDesc::kValid | (single ? UnitDesc::kSingle : 0u) | (head ? UnitDesc::kHead : 0u) |
                         (sane ? UnitDesc::kSane : 0u) | (niters << 8),
                     single ? 0u : (nseg - 1 - seg) * (kSegBytes / kBlockBytes));
    return r;
}

// Blocks [k0, k1) of unit r (niters nb) as a record of their own: its end
// moves back by nb - k1 blocks (added to its shift), its start (k0 > 0) to
// block k0's grid point, which is 16-B aligned (the grid is anchored at the
// 16-aligned unit end), so the piece's own grid is the unit's.  A piece is
// never stored whole (not single): its value is shifted and XORed into the
// span's accumulator.  k0 == k1: an empty record (flags 0).
__device__ __forceinline__ UnitRec unit_piece(const UnitRec &r, uint32_t k0, uint32_t k1) {
    const uint32_t nb = r.b.z >> 8;
    if (k0 == 0 && k1 == nb) return r;
    UnitRec q{};
    if (k0 == k1) return q;
    const uint32_t delta = k0 ? r.a.z - kBlockBytes * (nb - k0) : 0u;  // block k0's G - p
    const uint64_t o = ((uint64_t)r.a.x | ((uint64_t)r.a.y << 32)) + delta;
    q.a = make_uint4((uint32_t)o, (uint32_t)(o >> 32), r.a.z - kBlockBytes * (nb - k1) - delta, r.a.w - delta);
    q.b = make_uint4(r.b.x, r.b.y, (r.b.z & (UnitDesc::kValid | UnitDesc::kSane)) | ((k1 - k0) << 8),
                     r.b.w + (nb - k1));
    return q;
}

// Raw fetch of unit u.  The record is the same for every lane of a group, so
// lane j of the group holds only its dword j (one VGPR while the loads are in
// flight); decode_unit gathers the dwords when the unit is needed.  Nothing
// here uses the loaded value (a use would make the wave wait for every older
// load, the block prefetch included): units are fetched two ahead and decoded
// when their loads are long done.  One-unit-per-span batches (no plan) fetch
// only the span's offset (lanes 0/1).
template <bool UNITS>
__device__ __forceinline__ uint32_t fetch_unit(const SpanArgs &a, uint64_t u, uint64_t nunits, uint32_t li) {
    const uint32_t j = li & 7u;
    if (u >= nunits) return 0u;  // flags 0: no unit
    if (UNITS) return reinterpret_cast<const uint32_t *>(a.units + u)[j];
    const uint32_t *src = j < 2u && a.offsets ? reinterpret_cast<const uint32_t *>(a.offsets) + 2 * u + j : nullptr;
    return src ? *src : 0u;
}

// Decode unit u's record (raw: its lane-distributed dwords from fetch_unit).
template <bool UNITS>
__device__ __forceinline__ UnitDesc decode_unit(const SpanArgs &a, uint32_t raw, uint64_t u, uint64_t nunits,
                                                uint32_t lane) {
    const uint32_t g = lane & 32u;
    UnitDesc d;
    d.raw = raw;
    if (UNITS) {
        d.p = a.base + ((uint64_t)__shfl(raw, g | 0, 64) | ((uint64_t)__shfl(raw, g | 1, 64) << 32));
        d.eo = __shfl(raw, g | 2, 64);
        // (record dword 6: niters << 8 | flags; dword 3: E - p, past e for
        // every unit but the span's last, whose tail is e - E = t < 128)
        const uint32_t ew = __shfl(raw, g | 3, 64), r6 = __shfl(raw, g | 6, 64);
        const uint32_t tl = d.eo > ew ? d.eo - ew : 0u;
        d.nf = (r6 & 15u) | (tl << UnitDesc::kTailShift) | ((r6 >> 8) << UnitDesc::kNitersShift);
    } else {
        // unit = span u of `len` bytes at `off`: make_unit(kWhole) restated in
        // 32-bit arithmetic (everything but the address depends on p & 15 only;
        // the generic form cost ~200 VALU per switch)
        static_assert(kBlockBytes == 4096, "shifts below");
        const uint64_t off = a.offsets ? (uint64_t)__shfl(raw, g | 0, 64) | ((uint64_t)__shfl(raw, g | 1, 64) << 32)
                                       : u * a.stride;
        const bool sane = off <= a.base_bytes && a.len <= a.base_bytes - off;  // else: read nothing
        const uint32_t len = sane ? a.len : 0u;
        const uint32_t plo = (uint32_t)(uintptr_t)a.base + (uint32_t)off, kh = plo & 15u;
        const uint32_t vlen = len + ((0u - plo - len) & (kGridAlign - 1));  // grid_pad
        const uint32_t x = vlen + kh;  // Ea - ph
        const uint32_t g1o = x - kBlockBytes * ((x - 1) >> 12) - kh;  // span_head
        const uint32_t po = frag_drop(len, g1o, vlen) ? g1o : 0u;
        const uint32_t eo = vlen - po;
        const uint32_t niters = len ? (eo + ((kh + po) & 15u) + kBlockBytes - 1) >> 12 : 0u;
        d.p = a.base + (sane ? off : 0) + po;
        d.eo = eo;
        d.nf = u < nunits ? UnitDesc::kValid | UnitDesc::kSingle | ((vlen - len) << UnitDesc::kTailShift) |
                                (niters << UnitDesc::kNitersShift)
                          : 0u;  // flags 0: no unit
    }
    return d;
}

// (non-temporal: the planned path's blocks are whole lines since round 5,
// kGridAlign; config 3 -1.5 to -2 %, mixed pages -1.3 % against the row
// layout, profiles/r05_ablations/spans_line_grid_ab.txt)
constexpr bool kSpanNT = true;
// A 4 KiB block of a unit in K1's lane layout (round 5): lane li holds the
// 16-B pieces at G + 512 k + 16 li, k = 0..7, so each load instruction reads
// 512 contiguous bytes per group, non-temporal (crc32c_kernels.hip K1).
struct BlockWin {
    uint4 v[kK1Pieces];
};

// Issue the loads of block k of unit d for lane li.
__device__ __forceinline__ void load_block(BlockWin &w, const UnitDesc &d, uint32_t k, uint32_t li,
                                           const uint4 *zero) {
    // Offsets relative to the unit's first byte p: block start G - p = grel;
    // lane li's piece k is [grel + 512 k + 16 li, +16).  A piece that ends at
    // or before ph = floor16(p) reads the zero line (only head blocks have
    // such pieces); every other piece overlaps [ph, e), so no load leaves the
    // pages of the span.
    const int32_t grel = (int32_t)d.eo - (int32_t)(kBlockBytes * (d.niters() - k));
    const int32_t lrel = grel + (int32_t)(kK1LaneBytes * li);
    const uint8_t *q0 = d.p + lrel;
    const uint8_t *zl = reinterpret_cast<const uint8_t *>(zero);
    // piece-0 end - ph; a unit without blocks (no bytes, or no unit) reads
    // nothing but zeros
    const int32_t e0 = d.niters() ? lrel + 16 + (int32_t)((uintptr_t)d.p & 15u) : -(int32_t)kBlockBytes - 16;
#pragma unroll
    for (int j = 0; j < (int)kK1Pieces; ++j) {
        const uint8_t *q = e0 + j * (int32_t)kK1Piece > 0 ? q0 + j * kK1Piece : zl;
        w.v[j] = kSpanNT ? ld16_nt(q) : ld16(q);
    }
}

// F_t cleared: the span's grid ends at Ea = E + t (t < 128), so F_t lies in
// the last line of its last block, piece 7 of lanes 24..31 (lane li's piece
// 7 is the line's bytes [16 (li - 24), +16)); the bytes of that piece from E
// on, min(max(t - 16 (31 - li), 0), 16) of them, are cleared.
__device__ __forceinline__ uint4 mask_tail(uint4 v, uint32_t t, uint32_t li) {
    const int32_t cl = min(max((int32_t)t - 16 * (31 - (int32_t)li), 0), 16);  // bytes cleared
    const int32_t keep = 16 - cl;
    uint32_t m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int32_t kb = min(max(keep - 4 * i, 0), 4);
        m[i] = kb >= 4 ? ~0u : (1u << (8 * kb)) - 1u;
    }
    return make_uint4(v.x & m[0], v.y & m[1], v.z & m[2], v.w & m[3]);
}

// acc' = M_4096(acc) ^ (the block's lane value) = M_2048(M_2048(acc) ^ u_A) ^ u_B
// (u_A / u_B: the first / second half's chains, k1_lane_value; M_2048 = the
// chunk-16 image's tables 16..19).  NS: rows (piece pairs) 0..NS-1 lie wholly
// before p for every lane of the wave (their chains are of zeros and are
// skipped); fold: some group of the wave is past its unit's first block
// (wave-uniform; else every acc is 0 and is not folded).
// The chains of one half's pieces v[J0..3] (v[j] for j < J0 are zeros and
// are skipped), each ended by its shifted last step: the half's value.  (One
// half at a time: eight live chains beside the prefetched block pushed the
// span kernel past 128 VGPRs into scratch.)
template <int J0>
__device__ __forceinline__ uint32_t half_value(const uint4 *v, const LaneCtx &c) {
    constexpr uint32_t kShift[3] = {kAuxShift0, kAuxShift1, kAuxShift2};
    uint32_t x[4];
#pragma unroll
    for (int j = J0; j < 4; ++j) x[j] = v[j].x;
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
        for (int j = J0; j < 4; ++j) x[j] = step4_next(x[j], dw4(v[j], i), c);
    uint32_t u = 0;
#pragma unroll
    for (int j = J0; j < 4; ++j) u ^= j < 3 ? step4_last_shifted(x[j], kShift[j]) : step4_next(x[j], 0u, c);
    return u;
}

template <int NS>
__device__ __forceinline__ uint32_t block_fold(uint32_t acc, bool fold, const BlockWin &w, const LaneCtx &c) {
    const uint32_t ub = half_value<NS == 3 ? 2 : 0>(w.v + 4, c);
    if (NS >= 2 && !fold) return ub;
    uint32_t h = fold ? apply_op<4>(kAuxSpanFold, acc) : 0u;
    if (NS < 2) h ^= half_value<2 * (NS & 1)>(w.v, c);
    return apply_op<4>(kAuxSpanFold, h) ^ ub;
}

// Store (MODE 0) or stamp (MODE 2) the CRC of span `item`, which starts at p.
// Stamp writes the spill CRC into the image's exptime field, bytes 28..31 =
// p - 4 (storage.c:567), or into out[] when the caller stages the images (host
// path); ok[] (if any) marks stamped images.  A span that is not sane (outside
// the buffer, or a malformed image) was not read (the caller counts it).
template <int MODE>
__device__ __forceinline__ void emit(const SpanArgs &a, uint64_t item, uint32_t crc, bool sane, const uint8_t *p) {
    if (MODE == 0) {
        a.out[item] = sane ? crc : 0u;
    } else {
        if (a.ok) a.ok[item] = sane;
        if (!sane) return;
        if (a.out) {
            a.out[item] = crc;
        } else {
            // one dword store at any alignment (global memory takes unaligned
            // stores on gfx950; the compiler emits that for this memcpy)
            __builtin_memcpy(const_cast<uint8_t *>(p) - 4, &crc, 4);
        }
    }
}

// v * y mod P spread over a 32-lane group: lane i adds bit i of v (the x^i
// coefficient) times xi = x^i * y (this lane's element of a row of the segpow
// table), and the lanes XOR-reduce into lane 0.  v is read from lane 0 of the
// group.
__device__ __forceinline__ uint32_t mul_row_group(uint32_t v0, uint32_t xi, uint32_t li) {
    const uint32_t v = __shfl(v0, 0, 32);
    uint32_t term = (v << li) & 0x80000000u ? xi : 0u;
    term ^= lane_down<0>(term);
    term ^= lane_down<1>(term);
    term ^= lane_down<2>(term);
    term ^= lane_down<3>(term);
    term ^= lane_down<4>(term);
    return term;
}

// 16 waves per CU (128 VGPRs).  768 threads (168 VGPRs) measured slower
// (config 3: 5.99 vs 5.90 ms; config 5: 6.90 vs 5.93 ms per 300 pages):
// latency hiding of the dependent lookup chains needs the waves.
constexpr uint32_t kSpanBlock = 1024;

// The span kernel: R = raw([ph, e)) of every work unit, pieces as they lie.
// A unit that is a whole span stores R (span_acc[span], or out[span] without
// a plan); a segment unit XORs M_{64Ki * (nseg-1-s)}(R) into span_acc[span].
// k_final then turns R into the CRC or the verdict.
template <bool UNITS>
__global__ __launch_bounds__(kSpanBlock) void k_spans(SpanArgs a, const uint4 *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint64_t nunits = UNITS ? (uint64_t)*a.nunits : a.n;
    // Balanced plan (k_expand): group g takes the records [starts[g],
    // starts[g + 1]), an equal share of the batch's blocks; else group g takes
    // units g, g + G, g + 2G, ...
    const bool bal = UNITS && a.starts;
    const uint32_t g0 = blockIdx.x * (blockDim.x >> 5);
    // a workgroup without a unit leaves before loading 160 KiB of tables (the
    // overlap pass is usually empty, and small plans do not fill the grid)
    if (bal ? (g0 && a.starts[g0] >= nunits) : (uint64_t)g0 >= nunits) return;
    load_tables(smem, img, kLdsImageK1Bytes);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t li = lane & 31u;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t ngroups_total = (uint64_t)gridDim.x * (blockDim.x >> 5);
    const uint32_t g = g0 + ((threadIdx.x >> 6) << 1) + (lane >> 5);
    // Rounds (round 5): the balanced plan cuts the batch's blocks into
    // rounds x G equal shares in block order and group g takes shares g,
    // G + g, 2G + g, ..., so the groups stream through one round's range of
    // the batch (about 8 GiB: crc32c_shim.hip plan_rounds) at a time instead
    // of each through its own 1/G of all of it.  Each round restarts the
    // group's pipeline.
    const uint32_t nrounds = bal ? a.rounds : 1u;
    uint64_t u = g;
    uint64_t ub = nunits;  // the group's records (of this round) end here
    auto share = [&](uint32_t rd) {
        const uint64_t v = (uint64_t)rd * ngroups_total + g;
        u = v ? min(a.starts[v], (uint32_t)nunits) : 0u;
        ub = min(a.starts[v + 1], (uint32_t)nunits);
    };
    if (bal) share(0);
    const uint64_t ustep = bal ? 1u : ngroups_total;

    UnitDesc cur = decode_unit<UNITS>(a, fetch_unit<UNITS>(a, u, ub, li), u, nunits, lane);
    // Ring of the next four units' raw records, lane-distributed: lanes
    // 8s..8s+7 of a group hold slot s.  The unit after cur is in slot sl; a
    // switch decodes it and refills the slot with the unit four further on.
    // Nothing is copied out of the ring and no load is used right after it is
    // issued (vmcnt counts in issue order: either would make the wave wait
    // for the block prefetch too).
    uint32_t ring = fetch_unit<UNITS>(a, u + (1 + (li >> 3)) * ustep, ub, li);
    const uint32_t *const segpow_rows = a.segpow;
    uint32_t sl = 0;
    uint32_t k = 0;    // block index inside cur
    uint32_t acc = 0;  // lane accumulator over the blocks of cur
    BlockWin w0, w1;
    const uint4 *zero = a.zero + (blockIdx.x % kZeroSlots) * (4096 / 16);
    load_block(w0, cur, 0, li, zero);

    // Process the block held in `w` (block k of cur) after issuing the loads of
    // the group's next block into `wn`.
    auto step = [&](BlockWin &w, BlockWin &wn) {
        const bool last = k + 1 >= cur.niters();
        // next block: block k + 1 of cur, or block 0 of the unit in ring slot sl
        UnitDesc nd;
        if (__any(last)) {
            const uint32_t g = lane & 32u, sb = sl << 3;
            const uint32_t rw = __shfl(ring, g | sb | (li & 7u), 64);  // slot sl, dword li & 7
            nd = decode_unit<UNITS>(a, rw, u + ustep, nunits, lane);
        }
        if (last && (li >> 3) == sl) ring = fetch_unit<UNITS>(a, u + 5 * ustep, ub, li);
        // a segment unit's shift row, loaded after the (masked) ring refill and
        // before the block prefetch: the multiply below then waits for exactly
        // the block's loads issued after it, vmcnt(8), not for everything
        // (under a wave-uniform branch: loads under divergent branches leave
        // the waitcnt pass a merged state that drains the prefetch)
        uint32_t segk = 0, fx1 = 0;
        if (UNITS) {
            segk = __shfl(cur.raw, (lane & 32u) | 7u, 64);
            if (__builtin_amdgcn_readfirstlane(__any(last && !cur.single())))
                fx1 = segpow_rows[32 * (segk & (kSegpowLo - 1)) + li];
            __builtin_amdgcn_sched_barrier(0);  // (issued before the block prefetch, not sunk after it)
        }
        {
            UnitDesc t = cur;
            t.p = last ? nd.p : cur.p;
            t.eo = last ? nd.eo : cur.eo;
            t.nf = last ? nd.nf : cur.nf;
            load_block(wn, t, last ? 0u : k + 1, li, zero);
        }
        // Every path consumes the whole block (a path that skips rows, or a
        // group without a unit, would otherwise leave the block's loads
        // pending in the waitcnt pass's view, and the next write to those
        // registers became an s_waitcnt vmcnt(0) that drained the prefetch).
#pragma unroll
        for (int j = 0; j < (int)kK1Pieces; ++j)
            asm volatile("" ::"v"(w.v[j].x), "v"(w.v[j].y), "v"(w.v[j].z), "v"(w.v[j].w));
        if (cur.niters()) {
            if (__any(last && cur.tail())) w.v[kK1Pieces - 1] = mask_tail(w.v[kK1Pieces - 1], last ? cur.tail() : 0u, li);
            const int32_t grel = (int32_t)cur.eo - (int32_t)(kBlockBytes * (cur.niters() - k));  // G - p
            // rows wholly before p for every lane of the wave are skipped
            // (a group without a unit has niters == 0 and votes to skip)
            const uint32_t nskip = __all(grel + 3 * (int32_t)kRowBytes <= 0)   ? 3u
                                   : __all(grel + 2 * (int32_t)kRowBytes <= 0) ? 2u
                                   : __all(grel + (int32_t)kRowBytes <= 0)     ? 1u
                                                                               : 0u;
            // (the fold of a unit's first block is of acc = 0: skipped when no
            // group of the wave is past its first block, e.g. one-block units)
            const bool fold = __builtin_amdgcn_readfirstlane(__any(k != 0));
            switch (nskip) {
                case 0: acc = block_fold<0>(acc, fold, w, c); break;
                case 1: acc = block_fold<1>(acc, fold, w, c); break;
                case 2: acc = block_fold<2>(acc, fold, w, c); break;
                default: acc = block_fold<3>(acc, fold, w, c); break;
            }
        }
        if (last) {
            if (cur.valid()) {
                const uint32_t raw = group_reduce32_span(acc, lane);
                if (!UNITS) {
                    if (li == 0) a.out[u] = raw;
                } else {
                    const uint32_t item = __shfl(cur.raw, (lane & 32u) | 5u, 64);
                    if (cur.single()) {
                        if (li == 0) a.span_acc[item] = raw;
                    } else {
                        // a segment or piece ending segk blocks before the span's end:
                        // R(span) gets M_{4096 segk}(R) (the second factor, for units
                        // 16 MiB or more before the end only, is loaded here:
                        // one register fewer across the step, a drain only at such segment ends)
                        uint32_t v = mul_row_group(raw, fx1, li);
                        if (__any(segk >= kSegpowLo))
                            v = mul_row_group(v, segpow_rows[32 * (kSegpowLo + segk / kSegpowLo) + li], li);
                        if (li == 0) atomicXor(a.span_acc + item, v);
                    }
                }
            }
            acc = 0;
            k = 0;
            u += ustep;
            cur = nd;
            sl = (sl + 1u) & 3u;
        } else {
            ++k;
        }
    };

    for (uint32_t rd = 0;;) {
        // nothing issued before the loop stays pending into it (the waitcnt
        // pass would otherwise wait for it, vmcnt(0), at the top of every
        // iteration)
        __builtin_amdgcn_s_waitcnt(0);
        // One, wave-uniform exit at the bottom (a group that has finished
        // runs empty steps until the other has): a divergent or mid-loop exit
        // gives the loop header an un-waited predecessor, and the waitcnt
        // pass then drains the prefetch there (vmcnt(0)) on every iteration.
        for (;;) {
            step(w0, w1);
            step(w1, w0);
            if (!__builtin_amdgcn_readfirstlane(__any(cur.valid()))) break;
        }
        if (++rd >= nrounds) break;
        // (a round whose first share is empty is followed by empty ones: a
        // small plan -- K5's fallback list -- fills round 0 or less)
        if (a.starts[(uint64_t)rd * ngroups_total] >= (uint32_t)nunits) break;
        // the next round's share: a fresh pipeline (the ring and the block
        // prefetch of the finished share hold nothing of it)
        share(rd);
        cur = decode_unit<UNITS>(a, fetch_unit<UNITS>(a, u, ub, li), u, nunits, lane);
        ring = fetch_unit<UNITS>(a, u + (1 + (li >> 3)) * ustep, ub, li);
        sl = 0;
        k = 0;
        acc = 0;
        load_block(w0, cur, 0, li, zero);
    }
}

// Work units of span [p, p + len): its segments, less a head segment that
// was one block and whose fragment the span's thread takes (none for len 0).
__device__ __forceinline__ uint32_t span_units(const uint8_t *p, uint32_t len) {
    if (len == 0) return 0;
    const uint32_t vlen = len + grid_pad(p, len);
    const uint32_t ns = nseg_of(vlen);
    const SpanHead h = span_head(p, len);
    return ns - (h.drop && h.g1o == vlen - (uint64_t)(ns - 1) * kSegBytes ? 1u : 0u);
}

// 4 KiB blocks of those nu units: 16 per segment, and the head segment's
// niters (make_unit) when it is one of them.
__device__ __forceinline__ uint32_t span_blocks(const uint8_t *p, uint32_t len, uint32_t nu) {
    if (nu == 0) return 0;
    const uint32_t vlen = len + grid_pad(p, len);
    const uint32_t ns = nseg_of(vlen);
    constexpr uint32_t kSegBlocks = kSegBytes / kBlockBytes;
    if (nu < ns) return kSegBlocks * nu;
    const SpanHead h = span_head(p, len);
    const uint32_t po = h.drop ? (uint32_t)h.g1o : 0u;
    const uint32_t eo = vlen - (ns - 1) * kSegBytes - po;
    return (eo + (uint32_t)((uintptr_t)(p + po) & 15u) + kBlockBytes - 1) / kBlockBytes + kSegBlocks * (ns - 1);
}

// Units and blocks per span (packed, units | blocks << 32: one exclusive scan
// places the work units and the balanced plan's group boundaries), and
// the span's item record with its z (the header is parsed once per launch, and
// the foreign bytes of the head piece are read here: for packed images they
// share a line with the header this pass reads anyway; the tail's are
// cleared by the span kernel and not read, round 5).
// Span i's plan entries: one-block flag, unit count, item record, R = 0.
template <int MODE>
__device__ __forceinline__ void count_item(const SpanArgs &a, uint64_t i, const ItemDesc &it, const Tab8 &t8,
                                           uint64_t *nunit, uint4 *irec, uint8_t *fast, bool whole = false,
                                           uint32_t rwhole = 0u) {
    // a span whose unit is one whole block goes to k_blocks (no units)
    const uint8_t *g1;
    bool none;
    const bool one = it.sane && one_block(it.p, it.len, &g1, &none) && !none;
    fast[i] = one;
    const uint32_t nu = one ? 0u : span_units(it.p, it.len);
    nunit[i] = nu | (uint64_t)span_blocks(it.p, it.len, nu) << 32;
    const uint64_t off = (uint64_t)(it.p - a.base);
    uint32_t z = 0;
    if (it.sane) {
        // (a whole span's R from the wave, whole_chunks: z = R ^ Z of its pieces)
        z = corr_apply(span_corr_arg(it.p, it.len, MODE == 0 ? it.aux : 0u, t8, whole), t8, a.xpow) ^
            (whole ? rwhole : 0u);
        if (MODE == 1) z ^= mulmodp_dev(~it.aux, a.xpow[grid_pad(it.p, it.len)]);  // W
    }
    irec[i] = make_uint4((uint32_t)off, (uint32_t)(off >> 32) | (it.sane ? 0u : kInsane), it.len, z);
    a.span_acc[i] = 0u;
}

// R = raw of [ph, Ea) (the pieces as they lie, F_t = [E, Ea) cleared as the
// span kernel clears it) for every lane of the wave whose span is whole
// (span_corr's first case: the thread's alone).  A whole
// span's chain used to run in its lane while the lanes without one idled
// (one whole span in seven on the mixed pages: 0.11 of k_count's 0.21 ms);
// now the wave cuts the pieces of all its whole spans into 128-B chunks and
// every lane takes one: r_c = raw of its <= 8 pieces, shifted past the rest of
// its span (M_{Ea - end}, x^(8 n) from the xpow table), XORed into the span's
// slot (LDS, wave-private).  The chunks cover the pieces [ph, ceil16(E)) only
// (the rest of [ph, Ea) is zeros), the piece holding E cleared from E on.
// tests/test_count_whole_model.py restates it.
constexpr uint32_t kCountThreads = 256;
// (128-B chunks: half the x^(8n) multiplies of 64-B ones, mixed pages -0.6 %;
// 256-B chunks' longer lane chains were slower: k_count_chunk_size_ab.txt)
constexpr uint32_t kWholePieces = 8, kWholeChunk = 16 * kWholePieces;  // pieces / bytes per chunk
__device__ __forceinline__ uint32_t whole_chunks(gbyte *gb, bool whole, uint64_t ph, uint64_t e, uint64_t ea,
                                                 const Tab8 &t, const uint32_t *xp, uint32_t *slot) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t e16 = (e + 15u) & ~(uint64_t)15u;  // end of the pieces holding bytes of D
    const uint32_t nch = whole ? (uint32_t)((e16 - ph + kWholeChunk - 1u) / kWholeChunk) : 0u;
    uint32_t inc = nch;  // inclusive chunk count over the wave
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += v;
    }
    const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64), excl = inc - nch;
    slot[lane] = 0u;
    for (uint32_t base = 0; base < total; base += 64u) {
        const uint32_t q = base + lane;
        // owner = the first lane whose inclusive count exceeds q
        uint32_t s = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1)
            if ((uint32_t)__shfl((int)inc, (int)(s + step - 1u), 64) <= q) s += step;
        const uint32_t c = q - (uint32_t)__shfl((int)excl, (int)s, 64);
        const uint64_t sph = (uint32_t)__shfl((int)(uint32_t)ph, (int)s, 64) |
                             ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(ph >> 32), (int)s, 64) << 32);
        const uint64_t sea = (uint32_t)__shfl((int)(uint32_t)ea, (int)s, 64) |
                             ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(ea >> 32), (int)s, 64) << 32);
        const uint64_t se = (uint32_t)__shfl((int)(uint32_t)e, (int)s, 64) |
                            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(e >> 32), (int)s, 64) << 32);
        const uint64_t se16 = (se + 15u) & ~(uint64_t)15u;
        const bool act = q < total;
        const uint64_t c0 = sph + (uint64_t)kWholeChunk * c;
        const uint32_t np = act ? (uint32_t)min((se16 - c0) >> 4, (uint64_t)kWholePieces) : 0u;
        Piece pc[kWholePieces];
#pragma unroll
        for (uint32_t k = 0; k < kWholePieces; ++k) pc[k] = k < np ? ld_piece(gb + c0 + 16u * k) : Piece{0, 0};
        // the last piece of the span: bytes from E on cleared (its first 16 - cl kept)
        if (np && c0 + 16u * np == se16) {
            const uint32_t keep = 16u - (uint32_t)(se16 - se);
            const uint64_t mlo = keep >= 8 ? ~0ull : (1ull << (8 * keep)) - 1ull;
            const uint64_t mhi = keep <= 8 ? 0ull : keep >= 16 ? ~0ull : (1ull << (8 * (keep - 8))) - 1ull;
#pragma unroll
            for (uint32_t k = 0; k < kWholePieces; ++k)
                if (k + 1 == np) pc[k] = Piece{pc[k].lo & mlo, pc[k].hi & mhi};
        }
        uint32_t r = 0;
#pragma unroll
        for (uint32_t k = 0; k < kWholePieces; ++k) {
            const uint32_t nx = t.piece(r, pc[k]);
            r = k < np ? nx : r;
        }
        const uint64_t after = act ? sea - (c0 + 16u * np) : 0u;
        r = after ? mulmodp_dev(r, xpow8_dev(xp, after)) : r;
        if (act) atomicXor(&slot[s], r);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return whole ? slot[lane] : 0u;
}

template <int MODE>
__global__ __launch_bounds__(kCountThreads) void k_count(SpanArgs a, uint64_t *nunit, uint4 *irec, uint8_t *fast) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    __shared__ __attribute__((aligned(16))) uint32_t s8[kTab8Dwords];
    __shared__ uint32_t wslot[kCountThreads / 64][64];
    const uint64_t n = span_count(a);
    // (a K5 fallback list is usually a few hundred spans on a grid sized for
    // the batch: the workgroups past it leave before copying 20 KiB of tables)
    if ((uint64_t)blockIdx.x * blockDim.x >= n) return;
    const Tab8 t8 = load_tab8(s8, a.tab8);
    gbyte *const gb = (gbyte *)a.base;
    uint32_t *const slot = wslot[threadIdx.x >> 6];
    const uint64_t lane = threadIdx.x & 63u;
    // (a wave-uniform loop: every lane takes part in whole_chunks)
    for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x + (threadIdx.x - lane); i0 < n;
         i0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = i0 + lane;
        const bool valid = i < n;
        ItemDesc it{a.base, 0u, 0u, false};
        if (valid) it = fetch_item<MODE>(a, i);
        const uint32_t t = grid_pad(it.p, it.len);
        const uint64_t kh = (uintptr_t)it.p & 15u, off = (uint64_t)(it.p - a.base);
        const SpanHead h = span_head(it.p, it.len);
        const bool whole = valid && it.sane && it.len != 0 && h.drop && h.g1o == (uint64_t)it.len + t;
        const uint32_t r = whole_chunks(gb, whole, off - kh, off + it.len, off + it.len + t, t8, a.xpow, slot);
        if (valid) count_item<MODE>(a, i, it, t8, nunit, irec, fast, whole, r);
    }
}

// ---------------------------------------------------------------------------
// The plan's prefix sums (round 4: the library's own kernels instead of
// hipcub's scan and select, so that every kernel that runs several
// workgroups per CU carries the VGPR floor, crc32c_device.h).  Per span k_count
// (or the walk) leaves nunit[i] = units | blocks << 32 and fast[i]; tiles of
// kPlanTile spans are reduced (k_plan_tiles), the tile sums scanned by one
// workgroup (k_plan_scan), and k_expand rescans its tile to place every span:
// units and blocks are summed in 64 bits each (no carry between the fields),
// the fast spans' positions give the compacted list k_blocks reads.
// ---------------------------------------------------------------------------
struct PlanSum {
    uint64_t units, blocks;
    uint32_t fast, pad;
};
constexpr uint32_t kPlanThreads = 1024, kPlanPer = 2, kPlanTile = kPlanThreads * kPlanPer;

__device__ __forceinline__ PlanSum plan_of(uint64_t nu, uint8_t f) {
    return {(uint32_t)nu, nu >> 32, (uint32_t)f, 0u};
}
__device__ __forceinline__ PlanSum plan_add(const PlanSum &x, const PlanSum &y) {
    return {x.units + y.units, x.blocks + y.blocks, x.fast + y.fast, 0u};
}

// Exclusive scan of v over a kPlanThreads workgroup; *total = the sum of all.
// Every thread calls it (two barriers; `sh` holds the wave sums).
__device__ __forceinline__ PlanSum block_scan_excl(PlanSum v, PlanSum *sh, PlanSum *total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    PlanSum inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(inc.units, d, 64), b = __shfl_up(inc.blocks, d, 64);
        const uint32_t f = __shfl_up(inc.fast, d, 64);
        if (lane >= d) inc = plan_add(inc, PlanSum{u, b, f, 0u});
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    PlanSum before{0, 0, 0, 0}, all{0, 0, 0, 0};
    for (uint32_t k = 0; k < kPlanThreads / 64; ++k) {
        if (k < w) before = plan_add(before, sh[k]);
        all = plan_add(all, sh[k]);
    }
    __syncthreads();  // (sh is reused by the next call)
    *total = all;
    return plan_add(before, PlanSum{inc.units - v.units, inc.blocks - v.blocks, inc.fast - v.fast, 0u});
}

// Span i's count record (past n: zero).
__device__ __forceinline__ PlanSum plan_at(const uint64_t *nunit, const uint8_t *fast, uint64_t n, uint64_t i) {
    return i < n ? plan_of(nunit[i], fast[i]) : PlanSum{0, 0, 0, 0};
}

// Tile t's sum (thread-contiguous: thread k holds spans t*kPlanTile + kPlanPer k .. + kPlanPer - 1).
__global__ __launch_bounds__(kPlanThreads) void k_plan_tiles(const uint64_t *nunit, const uint8_t *fast, uint64_t n,
                                                            const uint32_t *dn, PlanSum *tile_sum) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    __shared__ PlanSum sh[kPlanThreads / 64];
    if (dn) n = *dn;
    const uint64_t ntiles = (n + kPlanTile - 1) / kPlanTile;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t i0 = t * kPlanTile + (uint64_t)threadIdx.x * kPlanPer;
        PlanSum s{0, 0, 0, 0};
#pragma unroll
        for (uint32_t k = 0; k < kPlanPer; ++k) s = plan_add(s, plan_at(nunit, fast, n, i0 + k));
        PlanSum tot;
        (void)block_scan_excl(s, sh, &tot);
        if (threadIdx.x == 0) tile_sum[t] = tot;
    }
}

// Exclusive scan of the tile sums of n spans (*dn when given) by one
// workgroup; *total = the grand total (units, blocks and fast spans of the
// whole batch).
__global__ __launch_bounds__(kPlanThreads) void k_plan_scan(const PlanSum *tile_sum, uint64_t n, const uint32_t *dn,
                                                           PlanSum *tile_pre, PlanSum *total) {
    MCRC_VGPR_FLOOR();
    __shared__ PlanSum sh[kPlanThreads / 64];
    if (dn) n = *dn;
    const uint64_t ntiles = (n + kPlanTile - 1) / kPlanTile;
    PlanSum carry{0, 0, 0, 0};
    for (uint64_t t0 = 0; t0 < ntiles; t0 += kPlanThreads) {
        const uint64_t t = t0 + threadIdx.x;
        PlanSum tot;
        const PlanSum ex = block_scan_excl(t < ntiles ? tile_sum[t] : PlanSum{0, 0, 0, 0}, sh, &tot);
        if (t < ntiles) tile_pre[t] = plan_add(carry, ex);
        carry = plan_add(carry, tot);
    }
    if (threadIdx.x == 0) *total = carry;
}

// Exclusive scan of m 32-bit counts by one workgroup (the device page walk:
// the index of each wbuf's first item; a few thousand wbufs per call).
// out[m] = the total.
__global__ __launch_bounds__(1024) void k_scan32(const uint32_t *in, uint64_t m, uint32_t *out) {
    MCRC_VGPR_FLOOR();
    __shared__ uint32_t sh[16];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (uint64_t i0 = 0; i0 < m; i0 += 1024) {
        const uint64_t i = i0 + threadIdx.x;
        const uint32_t v = i < m ? in[i] : 0u;
        uint32_t inc = v;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            if (lane >= d) inc += o;
        }
        if (lane == 63) sh[w] = inc;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (uint32_t k = 0; k < 16; ++k) {
            before += k < w ? sh[k] : 0u;
            all += sh[k];
        }
        __syncthreads();
        if (i < m) out[i] = carry + before + inc - v;
        carry += all;
    }
    if (threadIdx.x == 0) out[m] = carry;
}

// Write the unit records of span i at its units prefix.  Spans whose units would pass
// `cap` (possible only when spans overlap) are listed in `whole` and processed
// as one unit each by a second pass; *nvalid = records written before the
// first such span (zeroed by the caller: none fit).  Spans of more than kExpandInline segments are listed in `big`
// and expanded by k_expand_big, one workgroup per span.
constexpr uint32_t kExpandInline = 32;
// A device-counted list (K5's fallback: a few hundred images whose length
// bits flipped) lands in one or two tiles, so its long spans go to
// k_expand_big sooner: k_expand 0.031 -> 0.012 ms per 300-page verify; at 8
// for every batch config 3 got 2.4 % slower
// (profiles/r04_ablations/k_expand_inline_ab.txt).
constexpr uint32_t kExpandInlineDn = 8;

// First segment of span i that is a unit (1 when the head segment is not).
__device__ __forceinline__ uint32_t first_seg(const uint8_t *p, uint32_t len, uint32_t nunit) {
    return nunit ? nseg_of(len + grid_pad(p, len)) - nunit : 0u;
}

// Balanced plan (starts != nullptr).  T = the blocks of all units, G = the
// span kernel's 32-lane groups: group g's share starts at block g * per,
// per = ceil(T / G).  A unit holding such boundaries is written as pieces cut
// at them (unit_piece), so unit j, first block bs, lands at record j + C(bs),
// C(bs) = the boundaries before bs, and group g's first record is
// starts[g] = j_g + g (j_g: the unit holding block g * per).  A boundary at a
// unit's first block leaves an empty record, the end of group g - 1's list.
// Round robin (starts == nullptr): unit j is record j.
constexpr uint32_t kBalanceMinPer = 2;
struct Balance {
    uint32_t *starts;
    uint64_t per;  // blocks per group
    uint64_t gm;   // groups with blocks: boundaries 1 .. gm - 1
};

// (total: the batch's grand total from k_plan_scan)
__device__ __forceinline__ Balance balance_of(const PlanSum *total, uint64_t n, uint32_t groups, uint32_t *starts) {
    Balance b{starts, 1, 0};
    if (starts && n) {
        // (at least kBalanceMinPer blocks per group.  One per block cut every
        // unit of a small batch into one record per block, serially in its
        // span's thread of k_expand: ~0.3 ms for 50 images of 1-2 MiB before
        // k_expand_big took the long spans of a device-counted list
        // (kExpandInlineDn).  A segment's 16, the floor until round 5, left a
        // small batch on few groups: K5's fallback list of ~1400 blocks per
        // 300 pages ran as 88 groups of 16 serial blocks, k_spans 0.07 ms.)
        const uint64_t t = total->blocks;
        b.per = max((t + groups - 1) / groups, (uint64_t)kBalanceMinPer);
        b.gm = (t + b.per - 1) / b.per;
    }
    return b;
}

__device__ __forceinline__ uint64_t cuts_before(const Balance &b, uint64_t bs) {
    if (!b.starts || bs == 0 || b.gm == 0) return 0;
    return min((bs + b.per - 1) / b.per - 1, b.gm - 1);
}

// Write unit j (record r, first block bs) as its records.
__device__ __forceinline__ void put_unit(UnitRec *units, const Balance &b, uint64_t j, uint64_t bs, const UnitRec &r) {
    if (!b.starts) {
        units[j] = r;
        return;
    }
    uint64_t idx = j + cuts_before(b, bs);
    const uint32_t nb = r.b.z >> 8;
    uint32_t k0 = 0;
    for (uint64_t g = max((bs + b.per - 1) / b.per, (uint64_t)1); g < b.gm && g * b.per < bs + nb; ++g) {
        const uint32_t kb = (uint32_t)(g * b.per - bs);
        units[idx] = unit_piece(r, k0, kb);
        b.starts[g] = (uint32_t)(idx + 1);
        ++idx;
        k0 = kb;
    }
    units[idx] = unit_piece(r, k0, nb);
}

// Per tile (kPlanTile spans, thread-contiguous as k_plan_tiles): the tile's
// prefix from k_plan_scan plus the exclusive scan inside the tile places every
// span's units (p0), first block (b0) and, for a one-block span, its slot in
// the compacted list fastidx (k_blocks).  The units of a wave's spans are
// written by the whole wave (round 5): unit q of the wave's inline units
// goes to lane q mod 64, which finds its span by a search over the lanes'
// inclusive unit counts -- a span of 16 segments used to take 16 serial
// make_unit / put_unit rounds in its lane while the wave's other lanes
// idled.  A span's units after its first are whole segments, so unit j's
// first block is b0 + (j ? nb0 + S (j - 1) : 0), nb0 = the span's blocks
// less S (ns - 1), S = kSegBytes / 4 KiB.  tests/test_span_balance.py
// restates the placement.
__global__ __launch_bounds__(kPlanThreads) void k_expand(const uint8_t *base, const uint64_t *nunit, const uint8_t *fast,
                                                        const PlanSum *tile_pre, const PlanSum *total, const uint4 *irec,
                                                        uint64_t n, const uint32_t *dn, UnitRec *units, uint64_t cap,
                                                        uint32_t *nvalid, UnitRec *whole, uint32_t *nwhole, uint4 *big,
                                                        uint32_t *nbig, uint32_t *fastidx, uint32_t groups,
                                                        uint32_t *starts) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    __shared__ PlanSum sh[kPlanThreads / 64];
    // the wave's spans' unit and block bases, slot 64 k + lane
    __shared__ uint64_t wp0[kPlanThreads / 64][64 * kPlanPer], wb0[kPlanThreads / 64][64 * kPlanPer];
    if (dn) n = *dn;
    const uint64_t ntiles = (n + kPlanTile - 1) / kPlanTile;
    const Balance bal = balance_of(total, n, groups, starts);
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t inline_max = dn ? kExpandInlineDn : kExpandInline;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t i0 = t * kPlanTile + (uint64_t)threadIdx.x * kPlanPer;
        uint64_t ck[kPlanPer];
        uint8_t fk[kPlanPer];
        PlanSum s{0, 0, 0, 0};
#pragma unroll
        for (uint32_t k = 0; k < kPlanPer; ++k) {
            ck[k] = i0 + k < n ? nunit[i0 + k] : 0ull;
            fk[k] = i0 + k < n ? fast[i0 + k] : (uint8_t)0;
            s = plan_add(s, plan_of(ck[k], fk[k]));
        }
        PlanSum tot;
        PlanSum pre = plan_add(tile_pre[t], block_scan_excl(s, sh, &tot));
        uint32_t cnt[kPlanPer];  // units this lane's span k leaves to the wave
#pragma unroll
        for (uint32_t k = 0; k < kPlanPer; ++k) {
            const uint64_t i = i0 + k;
            const uint64_t p0 = pre.units, ns = (uint32_t)ck[k], b0 = pre.blocks;
            cnt[k] = 0;
            wp0[w][64 * k + lane] = p0;
            wb0[w][64 * k + lane] = b0;
            if (i < n) {
                if (fk[k]) fastidx[pre.fast] = (uint32_t)i;
                if (p0 + ns <= cap) {
                    if (ns > inline_max) {
                        big[atomicAdd(nbig, 1u)] = make_uint4((uint32_t)i, (uint32_t)p0, (uint32_t)b0, (uint32_t)(b0 >> 32));
                    } else {
                        cnt[k] = (uint32_t)ns;
                    }
                    // the last span whose units fit: the record count
                    if (i + 1 == n || p0 + ns + (uint32_t)nunit[i + 1] > cap)
                        *nvalid = (uint32_t)(p0 + ns + cuts_before(bal, b0 + (ck[k] >> 32)));
                } else {
                    // (one unit with the span's head rule: the same grid, so the same G1)
                    const uint4 r = irec[i];
                    const uint64_t off = r.x | ((uint64_t)(r.y & ~kInsane) << 32);
                    whole[atomicAdd(nwhole, 1u)] = make_unit(base, off, r.z, r.w, !(r.y & kInsane), (uint32_t)i, kWhole);
                }
            }
            pre = plan_add(pre, plan_of(ck[k], fk[k]));
        }
        // the wave's inline units, one per lane and round
        const uint32_t c = cnt[0] + cnt[1];
        static_assert(kPlanPer == 2, "two spans per lane below");
        uint32_t inc = c;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += v;
        }
        const uint32_t T = (uint32_t)__shfl((int)inc, 63, 64), excl = inc - c;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (wp0 / wb0 written above)
        for (uint32_t q0 = 0; q0 < T; q0 += 64u) {
            const uint32_t q = q0 + lane;
            // owner lane: the first whose inclusive count exceeds q
            uint32_t o = 0;
#pragma unroll
            for (uint32_t step = 32; step; step >>= 1)
                if ((uint32_t)__shfl((int)inc, (int)(o + step - 1u), 64) <= q) o += step;
            const uint32_t oe = (uint32_t)__shfl((int)excl, (int)o, 64);
            const uint32_t oc0 = (uint32_t)__shfl((int)cnt[0], (int)o, 64);
            if (q < T) {
                const uint32_t r0 = q - oe;
                const uint32_t k = r0 < oc0 ? 0u : 1u;
                const uint32_t j = r0 - (k ? oc0 : 0u);
                const uint64_t i = t * kPlanTile + (uint64_t)((threadIdx.x & ~63u) + o) * kPlanPer + k;
                const uint64_t p0 = wp0[w][64 * k + o], b0 = wb0[w][64 * k + o];
                const uint64_t cki = nunit[i];
                const uint32_t ns = (uint32_t)cki;
                const uint4 r = irec[i];
                const uint64_t off = r.x | ((uint64_t)(r.y & ~kInsane) << 32);
                const uint32_t s0 = first_seg(base + off, r.z, ns);
                const uint64_t nb0 = (cki >> 32) - (uint64_t)(kSegBytes / kBlockBytes) * (ns - 1);
                const uint64_t bs = b0 + (j ? nb0 + (uint64_t)(j - 1) * (kSegBytes / kBlockBytes) : 0u);
                put_unit(units, bal, p0 + j, bs, make_unit(base, off, r.z, r.w, !(r.y & kInsane), (uint32_t)i, s0 + j));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (before the next tile rewrites wp0 / wb0)
    }
}

// big[b] = {span, p0, b0 (lo, hi)} from k_expand.
__global__ void k_expand_big(const uint8_t *base, const uint64_t *nunit, const PlanSum *total, const uint4 *irec,
                             UnitRec *units, const uint4 *big, const uint32_t *nbig, uint64_t n, const uint32_t *dn,
                             uint32_t groups, uint32_t *starts) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    if (dn) n = *dn;
    const Balance bal = balance_of(total, n, groups, starts);
    const uint32_t nb = *nbig;
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint4 e = big[b];
        const uint32_t i = e.x;
        const uint64_t p0 = e.y, b0 = e.z | ((uint64_t)e.w << 32);
        const uint32_t ns = (uint32_t)nunit[i];
        const uint4 r = irec[i];
        const uint64_t off = r.x | ((uint64_t)(r.y & ~kInsane) << 32);
        const bool sane = !(r.y & kInsane);
        const uint32_t s0 = first_seg(base + off, r.z, ns);
        // every unit after the first is a whole segment
        const uint32_t nb0 = make_unit(base, off, r.z, r.w, sane, i, s0).b.z >> 8;
        for (uint32_t s = threadIdx.x; s < ns; s += blockDim.x)
            put_unit(units, bal, p0 + s, b0 + (s ? nb0 + (s - 1) * (kSegBytes / kBlockBytes) : 0u),
                     make_unit(base, off, r.z, r.w, sane, i, s0 + s));
    }
}

// nbad += the per-thread counts of a workgroup: one atomic per workgroup.
// (Atomics on one address serialise in L2: one per bad item of a verify with
// 1 % corrupt items took 0.4 ms per 300 pages.)  Every thread of the block
// calls it.
__device__ __forceinline__ void count_bad(unsigned long long *nbad, uint32_t nb) {
    __shared__ uint32_t sum;
    if (threadIdx.x == 0) sum = 0;
    __syncthreads();
    nb += __shfl_xor(nb, 1);
    nb += __shfl_xor(nb, 2);
    nb += __shfl_xor(nb, 4);
    nb += __shfl_xor(nb, 8);
    nb += __shfl_xor(nb, 16);
    nb += __shfl_xor(nb, 32);
    if (__lane_id() == 0 && nb) atomicAdd(&sum, nb);
    __syncthreads();
    if (threadIdx.x == 0 && sum) atomicAdd(nbad, (unsigned long long)sum);
}

// Every span's result from its R (one thread per span):
//   planned (UNITS): R = span_acc[i], z from the item record: MODE 1 checks
//   R == W, MODE 0/2 compute ~M_{-t}(R ^ Z);
//   one unit per span (MODE 0, no plan): R = out[i], Z computed here.
template <int MODE, bool UNITS>
__global__ void k_final(SpanArgs a, const uint4 *irec) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    __shared__ __attribute__((aligned(16))) uint32_t s8[UNITS ? 1 : kTab8Dwords];
    Tab8 t8{s8};
    if (!UNITS) t8 = load_tab8(s8, a.tab8);
    uint32_t nb = 0;  // bad spans seen by this thread
    const uint64_t n = UNITS ? span_count(a) : a.n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *p;
        uint32_t len, R, z = 0;
        bool sane;
        if (UNITS) {
            const uint4 r = irec[i];
            p = a.base + (r.x | ((uint64_t)(r.y & ~kInsane) << 32));
            sane = !(r.y & kInsane);
            len = r.z;
            z = r.w;
            R = a.span_acc[i];
        } else {
            const uint64_t off = a.offsets ? a.offsets[i] : i * a.stride;
            sane = off <= a.base_bytes && a.len <= a.base_bytes - off;  // as decode_unit
            p = a.base + (sane ? off : 0);
            len = a.len;
            const SpanHead h = span_head(p, len);
            R = sane && !(h.drop && h.g1o == len + grid_pad(p, len)) ? a.out[i] : 0u;  // (else not given to k_spans)
            if (sane) z = span_corr(p, len, a.crc_in ? a.crc_in[i] : 0u, t8, a.xpow);
        }
        if (MODE == 1) {
            const bool good = sane && R == z;
            a.ok[i] = good;
            nb += !good;
        } else {
            const uint32_t t = grid_pad(p, len);
            uint32_t v = R ^ z;
            if (t) v = mulmodp_dev(v, a.xpow[kXpowInv + t]);
            emit<MODE>(a, i, ~v, sane, p);
            nb += !sane;
        }
    }
    count_bad(a.nbad, nb);
}

// Small batches: one launch.  Up to kSmallMax spans, one 32-lane group per
// span, 32 spans per workgroup: the group reads the whole span [ph, Ea) in
// 4 KiB blocks anchored at Ea (no plan, no segments, no head fragment), reduces
// it to R, and its lanes compute Z from the span image's own tables
// (raw16 by dword steps, the x^(8n) multiplies) and emit.  The planned path's
// seven launches (count, scan, expand, span kernel x 2, final) cost ~80 us per
// call whatever the batch; a storage.c wbuf stamp (1007 images) or an IO-batch
// verify is one call of this kernel.
constexpr uint32_t kSmallMax = 8192;

// Register after the 16 bytes of v from a zero register, on the span image's
// replicated slice-by-4 tables (this lane's copy).
__device__ __forceinline__ uint32_t raw16_img(Piece v, const LaneCtx &c) {
    uint32_t x = (uint32_t)v.lo;
    x = step4_next(x, (uint32_t)(v.lo >> 32), c);
    x = step4_next(x, (uint32_t)v.hi, c);
    x = step4_next(x, (uint32_t)(v.hi >> 32), c);
    return step4_next(x, 0u, c);
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_small(SpanArgs a, const uint4 *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    load_tables(smem, img, kLdsImageK1Bytes);
    const uint32_t lane = threadIdx.x & 63u, li = lane & 31u;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 5) + (threadIdx.x >> 5);
    const bool valid = i < a.n;
    ItemDesc it{a.base, 0u, 0u, false};
    if (valid) it = fetch_item<MODE>(a, i);
    const uint32_t len = it.sane ? it.len : 0u;
    const uint32_t t = tail_pad(it.p, len), eo = len + t;
    const uint32_t niters = len ? (eo + (uint32_t)((uintptr_t)it.p & 15u) + kBlockBytes - 1) / kBlockBytes : 0u;
    const uint32_t nmax = __builtin_amdgcn_readfirstlane(max(niters, (uint32_t)__shfl_xor(niters, 32, 64)));
    const uint4 *zero = a.zero + (blockIdx.x % kZeroSlots) * (4096 / 16);
    uint32_t acc = 0;
    // block k + 1 is loaded before block k is reduced (two register sets)
    auto issue = [&](BlockWin &w, uint32_t k) {
        UnitDesc d;
        d.p = it.p;
        d.eo = eo;
        // (past the span: zeros; no tail mask: k_small's grid is 16-B, its Z has raw(F_t))
        d.nf = k < niters ? (niters << UnitDesc::kNitersShift) | UnitDesc::kValid : 0u;
        d.raw = 0;
        load_block(w, d, k, li, zero);
    };
    auto reduce = [&](const BlockWin &w, uint32_t k) {
        const uint32_t v = block_fold<0>(acc, true, w, c);
        if (k < niters) acc = v;
    };
    BlockWin w0, w1;
    if (nmax) issue(w0, 0);
    for (uint32_t k = 0; k < nmax; k += 2) {
        issue(w1, k + 1);
        reduce(w0, k);
        if (k + 1 >= nmax) break;
        issue(w0, k + 2);
        reduce(w1, k + 1);
    }
    const uint32_t R = group_reduce32_span(acc, lane);
    uint32_t nb = 0;
    if (valid) {
        // Z on k_small's own 16-B grid (its blocks keep F_t): M_{len+t}(~c ^ raw(F_h)) ^ raw(F_t)
        const uint32_t cin = MODE == 0 ? it.aux : 0u;
        uint32_t z = mulmodp_dev(~cin, a.xpow[t]);  // (len 0: R = 0, crc = c)
        if (len) {
            const uint32_t kh = (uint32_t)((uintptr_t)it.p & 15u);
            uint32_t y = ~cin;
            if (kh) y ^= raw16_img(shl_bytes(ld_piece(it.p - kh), 16 - kh), c);
            z = mulmodp_dev(y, xpow8_dev(a.xpow, (uint64_t)len + t));
            if (t) z ^= raw16_img(clear_below(ld_piece(it.p + len + t - 16), 16 - t), c);
        }
        if (MODE == 1) {
            const bool good = it.sane && R == (z ^ mulmodp_dev(~it.aux, a.xpow[t]));
            if (li == 0) a.ok[i] = good;
            nb = li == 0 && !good;
        } else {
            uint32_t v = R ^ z;
            if (t) v = mulmodp_dev(v, a.xpow[kXpowInv + t]);
            if (li == 0) emit<MODE>(a, i, ~v, it.sane, it.p);
            nb = li == 0 && !it.sane;
        }
    }
    // one atomic per wave with a bad span (all 160 KiB of LDS hold the tables,
    // so no workgroup-level sum as in count_bad)
    const uint64_t m = __ballot(nb != 0);
    if (m && lane == (uint32_t)(__ffsll((unsigned long long)m) - 1)) {
        atomicAdd(a.nbad, (unsigned long long)__popcll(m));
        // the add must be performed before this workgroup is counted done:
        // __syncthreads is a workgroup-scope release and does not wait for
        // another wave's outstanding global atomics, so without this fence
        // the last workgroup could read nbad before the add lands (a lost
        // count this call, a phantom one the next)
        __threadfence();
    }
    if (a.host_nbad) {
        // the last workgroup to finish hands the count to the host and leaves
        // the counters at zero for the next call: no memset before the launch
        // and no copy after it (two dispatches of a ~35 us synchronous call)
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
                __threadfence();
                *a.host_nbad = atomicExch(a.nbad, 0ull);
                atomicExch(a.done, 0u);
                __threadfence_system();
            }
        }
    }
}

// ===========================================================================
// K4: one-block units (K1's loop over gathered blocks)
// ===========================================================================
//
// A span whose unit is exactly one 4 KiB block starting on its grid (its head
// fragment went to its thread: every 4133-B item of configs 2r and 5) needs
// none of the span kernel's unit machinery.  k_blocks runs K1's loop (MODE
// 14: four steps reduced by one tree, no row folds) over those blocks, with
// each group's block address gathered per span instead of base + i * stride,
// and writes R (no initial value, no final XOR): out[i] without a plan,
// span_acc[i] with one.  A span's descriptor is loaded two steps before its
// block: vmcnt counts in issue order, so when the address is needed only the
// newer block loads may still be pending.
struct BlkRegs {
    K1Regs d;       // the block, in K1's lane layout
    uint4 rec;      // descriptor of the block this buffer loads next
    uint32_t rs;    // (planned) its span
    uint32_t sidx;  // (planned) the span of the block two loads later
    uint32_t cur;   // (planned) the span of the block in d
    uint32_t tl;    // the block's span ends tl bytes before the block's end (F_t, mask_tail)
};

template <bool IDENT, bool OFFS>
__global__ __launch_bounds__(1024) void k_blocks(SpanArgs a, const uint4 *__restrict__ img, const uint4 *irec,
                                                 const uint32_t *fastidx, const uint32_t *nfast) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // without a plan block j is span j; with one, span fastidx[j] of the nfast
    // spans k_count found to be one block
    const uint64_t n = IDENT ? a.n : (uint64_t)*nfast;
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t gstep = gridDim.x * waves;
    const uint64_t ngroups = (n + 1) / 2;
    uint64_t grp = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6));
    if ((uint64_t)blockIdx.x * waves >= ngroups) return;
    load_tables(smem, img, kLdsImageK1Bytes);
    if (grp >= ngroups) return;
    const uint32_t lane = threadIdx.x & 63u, li = lane & 31u, g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    const uint8_t *zero = reinterpret_cast<const uint8_t *>(a.zero + (blockIdx.x % kZeroSlots) * (4096 / 16));
    auto item_of = [&](uint64_t gi) { return gi * 2 + g; };
    // block index of step gi (past the batch: a repeat of a step of this
    // wave, cache-hot, as in K1's last prefetch; its result is not stored)
    // (32-bit: the shim keeps n below 2^32)
    const uint32_t n32 = (uint32_t)n, ng32 = (uint32_t)ngroups, gstep32 = (uint32_t)gstep;
    auto j_of = [&](uint64_t gi64) -> uint32_t {
        const uint32_t gi = (uint32_t)gi64;
        const uint32_t gu = gi < ng32 ? gi : gi - gstep32 < ng32 ? gi - gstep32 : ng32 - 1;
        const uint32_t j = gu * 2 + g;
        return j < n32 ? j : n32 - 1;
    };
    // descriptor of block j (planned: of its span sj)
    auto rec_of = [&](uint32_t j, uint32_t sj) -> uint4 {
        if (IDENT) {
            // (offsets or stride is a template choice: a load under a branch
            // leaves the waitcnt pass a merged state that drains the prefetch)
            const uint64_t off = OFFS ? a.offsets[j] : j * a.stride;
            return make_uint4((uint32_t)off, (uint32_t)(off >> 32), a.len, 0u);
        }
        return irec[sj];
    };
    // A span here is one whole block and has a unit (one_block), so its block
    // is [Ea - 4096, Ea) whichever case of one_block holds.
    auto block_of = [&](const uint4 &r) -> const uint8_t * {
        const uint64_t off = r.x | ((uint64_t)(r.y & ~kInsane) << 32);
        bool sane = !(r.y & kInsane);
        if (IDENT) sane = off <= a.base_bytes && r.z <= a.base_bytes - off;  // (as decode_unit)
        const uint8_t *e = a.base + off + r.z;
        const uint8_t *blk = e + ((0u - (uint32_t)(uintptr_t)e) & (kGridAlign - 1)) - kBlockBytes;  // (pointer
        return sane ? blk : zero;  // arithmetic: an integer round trip would make these flat loads)
    };
    // t = Ea - E of the block's span (its F_t is the block's last t bytes)
    auto tail_of = [&](const uint4 &r) -> uint32_t {
        return (0u - ((uint32_t)(uintptr_t)a.base + r.x + r.z)) & (kGridAlign - 1);
    };
    // Loads run ahead of their use (vmcnt counts in issue order, so when a
    // value is needed only newer loads may be pending): the span index four
    // steps ahead, the descriptor two, the block one.
    auto ld = [&](BlkRegs &b, uint64_t gi) {
        if (IDENT && !OFFS) {  // (fixed stride: nothing to load ahead)
            const uint4 r = rec_of(j_of(gi), 0u);
            b.tl = tail_of(r);
            b.d.template load_at<kSpanNT>(block_of(r), li * kK1LaneBytes);
        } else {
            const uint8_t *blk = block_of(b.rec);
            b.tl = tail_of(b.rec);
            if (!IDENT) {
                b.cur = b.rs;
                b.rs = b.sidx;
            }
            b.rec = rec_of(j_of(gi + 2 * gstep), b.rs);
            if (!IDENT) b.sidx = fastidx[j_of(gi + 4 * gstep)];
            b.d.template load_at<kSpanNT>(blk, li * kK1LaneBytes);
        }
        // (as K1: the loads stay at the top of the step instead of being sunk
        // into the chains, where the next step would wait on them at once)
        __builtin_amdgcn_sched_barrier(0);
    };
    auto part0 = [&](BlkRegs &b) {
        b.d.d[kK1Pieces - 1] = mask_tail(b.d.d[kK1Pieces - 1], b.tl, li);
        return reduce_level<0>(k1_lane_value(b.d, c), (lane & 1u) == 0u);
    };
    uint32_t *dst = IDENT ? a.out : a.span_acc;
    auto store = [&](uint32_t raw, uint64_t gi, uint32_t span, bool on) {
        const uint64_t item = item_of(gi);
        if (on && gi < ngroups && item < n) dst[IDENT ? item : span] = raw;
    };
    BlkRegs ra, rb;
    if (!IDENT || OFFS) {
        if (!IDENT) {
            ra.rs = fastidx[j_of(grp)];
            rb.rs = fastidx[j_of(grp + gstep)];
            ra.sidx = fastidx[j_of(grp + 2 * gstep)];
            rb.sidx = fastidx[j_of(grp + 3 * gstep)];
        }
        ra.rec = rec_of(j_of(grp), ra.rs);
        rb.rec = rec_of(j_of(grp + gstep), rb.rs);
    }
    const uint64_t nsteps = (ngroups - grp + gstep - 1) / gstep;
    ld(ra, grp);
    uint64_t k = 0;
    for (; k + 4 <= nsteps; k += 4) {
        ld(rb, grp + gstep);
        const uint32_t va = part0(ra), sa = ra.cur;
        ld(ra, grp + 2 * gstep);
        const uint32_t vb = part0(rb), sb = rb.cur;
        const uint32_t vab = group_pair_level1(va, vb, lane);
        ld(rb, grp + 3 * gstep);
        const uint32_t vc = part0(ra), sc = ra.cur;
        ld(ra, grp + 4 * gstep);
        const uint32_t vd = part0(rb), sd = rb.cur;
        const uint32_t raw = group_reduce32_quad_span(vab, group_pair_level1(vc, vd, lane), lane);
        const uint32_t sp = li == 0 ? sa : li == 1 ? sb : li == 2 ? sc : sd;
        store(raw, grp + (li & 3u) * gstep, sp, li < 4);
        grp += 4 * gstep;
    }
    for (; k + 2 <= nsteps; k += 2) {
        ld(rb, grp + gstep);
        const uint32_t va = part0(ra), sa = ra.cur;
        ld(ra, grp + 2 * gstep);
        const uint32_t vb = part0(rb), sb = rb.cur;
        const uint32_t raw = group_reduce32_pair_span(va, vb, lane);
        store(raw, li == 0 ? grp : grp + gstep, li == 0 ? sa : sb, li < 2);
        grp += 2 * gstep;
    }
    if (nsteps & 1) {
        uint32_t v = part0(ra);
        v = reduce_level<1>(v, (lane & 3u) == 0u);
        v = reduce_level<2>(v, (lane & 7u) == 0u);
        v = reduce_level<3>(v, (lane & 15u) == 0u);
        store(reduce_level4_span(v, (lane & 31u) == 0u), grp, ra.cur, li == 0);
    }
}

// ===========================================================================
// K5: shared pieces (item images or equal spans whose span is one 4 KiB
// window after a short head; the kernel is k_lines below)
// ===========================================================================
//
// Images that are sane but not of K5's shape go to a fallback list that the
// planned path takes afterwards; malformed images are marked bad by K5.

struct ItemsOut {
    uint32_t *fb;   // items for the planned path (sane, not one block)
    uint32_t *nfb;  // their count
    const uint32_t *route;  // k_census's verdict (nullptr: take the batch); 0: every image to the planned path
    uint2 *rt;      // MODE 2: per item {M_t(f), t | kRtFused}, {0, 0} if not fused (for k_fix)
    uint32_t xm128;      // k_lines: x^(-8 * 128) (MODE 0: the CRC from M_128(V))
    uint32_t nsr;        // k_lines: steps per run (a wave's run is 2 nsr consecutive images)
};
constexpr uint32_t kRtFused = 0x80000000u;

// The dword at A of the head fragment: bytes below p cleared (pa = p - A)
// and the four bytes of inj (~c for an initial CRC c: a register seeded with
// ~c, crc32c.c:166) XORed into the bytes of [p, p + 4) it holds.
__device__ __forceinline__ uint32_t head_dword(uint32_t v, int32_t pa, uint32_t inj) {
    if (pa >= 4) return 0u;
    if (pa >= 0) return (v & (~0u << (8 * pa))) ^ (inj << (8 * pa));
    if (pa > -4) return v ^ (inj >> (8 * -pa));
    return v;
}
// Bytes [16 - t, 16) of v cleared (t < 16).
__device__ __forceinline__ uint4 clear_high(uint4 v, uint32_t t) {
    const uint64_t mh = t >= 8 ? 0ull : ~0ull >> (8 * t);
    const uint64_t ml = t <= 8 ? ~0ull : ~0ull >> (8 * (t - 8));
    return make_uint4(v.x & (uint32_t)ml, v.y & (uint32_t)(ml >> 32), v.z & (uint32_t)mh, v.w & (uint32_t)(mh >> 32));
}
// M_t(v) for t < 16: t zero bytes through this lane's replicated slice-by-4
// tables (t / 4 dword steps, then byte steps on T0).
__device__ __forceinline__ uint32_t zeros_lds(uint32_t v, uint32_t t, const LaneCtx &c) {
    for (uint32_t q = 0; q < (t >> 2); ++q) v = step4_next(v, 0u, c);
    for (uint32_t r = 0; r < (t & 3u); ++r)
        v = lds_ld(kAux4Bytes + 0x10000u + ((v & 0xffu) << 8) + 128u + c.lane4) ^ (v >> 8);
    return v;
}

constexpr uint32_t kStFused = 0x10u, kStSane = 0x20u, kStValid = 0x40u;
constexpr uint32_t kEpoch = 32;                                 // steps per epoch: 64 images per wave

struct ItemBuf {
    K1Regs d;     // the window, in K1's lane layout (pieces 512 k + 16 li)
    uint32_t st;  // its image: t | kStFused | kStSane | kStValid
};

// ===========================================================================
// K5, line-anchored (k_lines, round 4)
// ===========================================================================
//
// Round 3's K5 (k_items, removed in round 5; git show 7745007) read each
// image's header and head fragment at the start of an epoch and the image's
// 16-B-anchored block up to 32 steps later, by when the
// lines they share (the block's first line, the previous block's last line,
// which holds this image's header) have left L2: config 5 fetched 1.08x its
// span bytes, config 2r 1.065x (profiles/r04_ablations).  Here no line is
// read by both a block and a per-lane prep:
//   - the block of span D = [p, E) is the window [A, A + 4096), A =
//     ceil128(p + 4): the whole lines [A, B) of D, B = floor128(E), and zeros
//     past B (31 or 32 lines: the fused shape; lanes 28-31 of row 3 read the
//     zero line for a 31-line window);
//   - the epoch lane of the image takes its head [p, A) (4..131 bytes, ~c
//     injected at p: r_h = register from ~c over [p, A)) and its tail
//     [B, Et), Et = ceil16(E), bytes from E on cleared (r_t);
//   - a wave's epoch is a run of 2 nsr CONSECUTIVE images (lane L prepares
//     image L of the run, step s checksums images 2s and 2s + 1), so one
//     image's tail and the next image's head and header -- the same one or
//     two lines -- are read by neighbouring lanes of one instruction;
//   - the group's R = raw of the window goes back to the image's epoch lane,
//     which at the end of the run forms
//       V = M_{Et-A}(r_h) ^ M_{Et-A-4096}(R) ^ r_t = M_pad(f),
//     f the register after D from ~c, pad = Et - E: crc32c(c, D) =
//     ~M_{-pad}(V); a verify is good iff V == M_pad(~stored).  Round 6: the
//     lane forms W = M_128(V) = M_d(M_4096(r_h) ^ R) ^ M_128(r_t), d = Et - A
//     - 3968 in [0, 272), with the table operators (M_2048 twice, the tree
//     levels M_16..M_128 by the bits of d, zeros_lds below 16) instead of two
//     bitwise multiplies by x^(8 (Et - A)) and x^(8 (Et - A - 4096)) (the
//     second negative for a 31-line window with a short tail, hence the
//     M_128): a verify is good iff W == M_128(M_pad(~stored)), the CRC is
//     ~M_{-pad-128}(W).
// tests/test_items_lines_model.py restates it on the CPU.
constexpr uint32_t kLineBytes = 128;
constexpr uint32_t kHeadPieces = 10;  // 16-B pieces of [floor16(p), A): A - p <= 131
constexpr uint32_t kTailPieces = 9;   // of [B, Et): Et - B < 128 + 16
constexpr uint32_t kSt31 = 0x80u;     // the window holds 31 lines (row 3, lanes 28-31: zeros)

// The fused shape: B - A (bytes of whole lines inside the span after the
// head) is 31 or 32 lines.
__host__ __device__ __forceinline__ bool lines_fused(int64_t lines_bytes) {
    return lines_bytes >= (int64_t)(kBlockBytes - kLineBytes) && lines_bytes <= (int64_t)kBlockBytes;
}

template <int MODE, bool OFFS>
__global__ __launch_bounds__(1024) void k_lines(SpanArgs a, const uint4 *__restrict__ img, ItemsOut io) {
    // MODE 0: equal spans of a.len bytes by offsets (OFFS) or stride, MODE 1/2:
    // item images (verify / stamp) by offsets
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint64_t n = a.n;
    const uint64_t nsr = io.nsr;
    const uint64_t run_imgs = 2ull * nsr;
    const uint64_t waves = blockDim.x >> 6;
    const uint64_t W = gridDim.x * waves;
    const uint64_t w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)waves + (threadIdx.x >> 6));
    // Runs, dealt round robin (round 5): run k of wave w is the images
    // [(k W + w) 2 nsr, +2 nsr), so at any time the waves' windows lie
    // within W runs (~1 GB at 4165-B images) of each other.  Round 4 gave
    // each wave a contiguous chunk of ceil(n / W) images with staggered
    // first runs (-2.5 % at 300 pages); at 1000 pages (67 GB) those 4096
    // streams, 16 MB apart, ran 3.5-7 % slower per page than 300 pages did,
    // and the round-robin order took config 5 at 1000 pages from
    // 11.32-11.76 to 10.92-10.93 ms, 300 pages and config 2r level or better
    // (profiles/r05_ablations/k5_run_order_ab.txt).
    // tests/test_items_lines_model.py checks that the runs cover every image
    // exactly once.
    const uint64_t cend = n;
    auto run_start = [&](uint64_t k) -> uint64_t { return (k * W + w0) * run_imgs; };
    auto run_steps = [&](uint64_t k) -> uint64_t {
        (void)k;
        return nsr;
    };
    if ((uint64_t)blockIdx.x * waves * run_imgs >= n) return;
    if (MODE != 0 && io.route && *io.route == 0) {  // the census sent the batch to the planned path
        if (blockIdx.x == 0 && threadIdx.x == 0) *io.nfb = (uint32_t)n;
        return;
    }
    load_tables(smem, img, kLdsImageK1Bytes);
    if (run_start(0) >= cend) return;
    const uint32_t lane = threadIdx.x & 63u, li = lane & 31u, g = lane >> 5;
    LaneCtx c;
    c.lane4 = li << 2;
    c.lane4hi = c.lane4 | 0x10000u;
    gbyte *const gb = (gbyte *)a.base;
    gbyte *const gz = (gbyte *)(a.zero + (blockIdx.x % kZeroSlots) * (4096 / 16));
    const uint32_t base_lo = (uint32_t)(uintptr_t)a.base;  // (alignments: the offsets are from a.base)
    uint32_t nb = 0;  // bad (malformed or mismatching) images seen by this lane

    // (r: the wave's round, 0, 1, 2, ...)
    auto item_of = [&](uint64_t r) -> uint64_t { return run_start(r) + lane; };
    auto valid_of = [&](uint64_t r) { return lane < 2 * run_steps(r) && item_of(r) < cend; };
    auto off_of = [&](uint64_t r) -> uint64_t {
        // (offsets or stride is a template choice: a load on one side of a
        // branch leaves the waitcnt pass a merged state that waits for it)
        return valid_of(r) ? (OFFS ? a.offsets[item_of(r)] : item_of(r) * a.stride) : 0;
    };
    // MODE 0: x^(-8 (t + 128)), t < 16, lane-distributed (lane j holds t = j & 15)
    const uint32_t xinv = MODE == 0 ? mulmodp_dev(a.xpow[kXpowInv + (lane & 15u)], io.xm128) : 0u;
    uint64_t noff = off_of(0);  // this lane's image offset in the wave's next run
    uint32_t ncin = MODE == 0 && a.crc_in && valid_of(0) ? a.crc_in[item_of(0)] : 0u;

    // this lane's image of the run
    uint32_t eglo = 0, eghi = 0, est = 0;  // window start A (offset from a.base), status
    uint32_t p_kh = 0, p_inj = ~0u, p_stored = 0, p_nh = 0, p_nt = 0, p_eta = 0;
    uint64_t p_pho = 0, p_b = 0;
    uint32_t r_h = 0, r_t = 0, er = 0;
    uint4 pc[kHeadPieces], tc[kTailPieces];
    auto prep_head = [&](uint64_t r) {
        const bool valid = valid_of(r);
        const uint64_t off = noff;
        ItemHdr h{0u, 0u, 0u, 0u};
        ItemDesc it{a.base, 0u, 0u, false};
        p_inj = ~0u;  // ~c: the register's initial value, XORed in at p
        if (MODE == 0) {
            it.sane = valid && off <= a.base_bytes && a.len <= a.base_bytes - off;
            it.len = a.len;
            if (a.crc_in) p_inj = ~ncin;
        } else {
            const bool hdr_ok = valid && off + 48 <= a.base_bytes;
            if (hdr_ok) h = parse_hdr(gb + off);
            it = item_desc(a, off, h, hdr_ok);
        }
        p_stored = h.exptime;
        const uint32_t len = it.sane ? it.len : 0u;
        const uint64_t po = MODE == 0 ? off : off + 32;  // span start (offset)
        const uint64_t pe = po + len;                     // span end
        const uint32_t pa = base_lo + (uint32_t)po, ea = base_lo + (uint32_t)pe;
        const uint64_t A = po + 4 + ((0u - (pa + 4u)) & (kLineBytes - 1));
        const uint64_t B = pe - (ea & (kLineBytes - 1));
        const uint32_t pad = (0u - ea) & (kTailAlign - 1);
        const bool fused = it.sane && len >= 4 && lines_fused((int64_t)B - (int64_t)A);
        p_kh = pa & 15u;
        p_pho = po - p_kh;
        p_b = B;
        p_nh = fused ? (uint32_t)(A - p_pho) >> 4 : 0u;
        p_nt = fused ? (uint32_t)(pe + pad - B) >> 4 : 0u;
        p_eta = (uint32_t)(pe + pad - A);  // Et - A
        eglo = (uint32_t)A;
        eghi = (uint32_t)(A >> 32);
        est = pad | (fused ? kStFused : 0u) | (it.sane ? kStSane : 0u) | (valid ? kStValid : 0u) |
              (fused && B - A < kBlockBytes ? kSt31 : 0u);
    };
    auto head_loads = [&]() {
#pragma unroll
        for (uint32_t k = 0; k < kHeadPieces; ++k) pc[k] = ld16(k < p_nh ? gb + p_pho + 16 * k : gz);
    };
    // r_h = register from ~c over [p, A): bytes below p cleared, ~c injected at p
    auto head_chain = [&]() {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t k = 0; k < kHeadPieces; ++k) {
            const uint32_t w[4] = {pc[k].x, pc[k].y, pc[k].z, pc[k].w};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const int32_t pa = (int32_t)p_kh - (int32_t)(16 * k + 4 * j);
                const uint32_t d = head_dword(w[j], pa, p_inj);
                const uint32_t nx = (k == 0 && j == 0) ? d : step4_next(x, d, c);
                x = k < p_nh ? nx : x;
            }
        }
        r_h = p_nh ? step4_next(x, 0u, c) : 0u;
    };
    // (the last piece's bytes from E on are cleared: pad of them)
    auto tail_loads = [&]() {
#pragma unroll
        for (uint32_t k = 0; k < kTailPieces; ++k) tc[k] = ld16(k < p_nt ? gb + p_b + 16 * k : gz);
    };
    auto tail_chain = [&]() {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t k = 0; k < kTailPieces; ++k) {
            const uint4 v = k + 1 == p_nt ? clear_high(tc[k], est & 15u) : tc[k];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t nx = (k == 0 && j == 0) ? w[j] : step4_next(x, w[j], c);
                x = k < p_nt ? nx : x;
            }
        }
        r_t = p_nt ? step4_next(x, 0u, c) : 0u;
    };
    // Loads of step s into b: its window and its status.  Past the run
    // (s >= ns: the prefetch of the run's last step, whose result is not
    // used) the window is the workgroup's zero slot, in L2: a repeat of the
    // run's last window fetched it from HBM again (non-temporal loads), one
    // step in 1 + nsr, 3 % of config 5's bytes.  K1's layout
    // and policy (round 5): lane li holds the window's 16-B pieces at
    // 512 k + 16 li, each instruction reads whole lines, non-temporal (the
    // window's lines are read by nothing else: the heads and tails lie
    // outside [A, B)): config 2r 0.743-0.766 -> 0.693-0.694 ms, config 5
    // 3.58-3.59 -> 3.50 ms and stamp 3.85-3.86 -> 3.75-3.76 ms per 300 pages
    // (profiles/r05_ablations/k5_lines_pieces_nt_ab.txt).
    auto ld = [&](ItemBuf &b, uint32_t s, uint32_t ns) {
        const int src = (int)(2 * min(s, ns - 1) + g);
        const uint64_t lo = (uint32_t)__shfl((int)eglo, src, 64), hi = (uint32_t)__shfl((int)eghi, src, 64);
        b.st = (uint32_t)__shfl((int)est, src, 64);
        const bool real = s < ns;  // (wave-uniform)
        gbyte *blk = ((b.st & kStFused) && real ? gb + (lo | (hi << 32)) : gz) + 16 * li;
        const bool z7 = (b.st & kSt31) && real && li >= 24u;  // piece 7 past B (the window's last line): zeros
#pragma unroll
        for (int k = 0; k < (int)kK1Pieces - 1; ++k) b.d.d[k] = ld16_nt(blk + k * kK1Piece);
        b.d.d[kK1Pieces - 1] = ld16_nt(z7 ? gz + 16 * li : blk + (kK1Pieces - 1) * kK1Piece);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto part0 = [&](ItemBuf &b) { return reduce_level<0>(k1_lane_value(b.d, c), (lane & 1u) == 0u); };
    // The epoch lanes collect R of their images from the lanes that finished
    // them (steps s0 .. s0 + cnt - 1 in lanes 0 .. cnt - 1 of each group).
    auto collect = [&](uint32_t r, uint32_t s0, uint32_t cnt) {
        const uint32_t sl = lane >> 1;
        const int src = (int)((lane & 1u) * 32u + (sl - s0));
        const uint32_t v = (uint32_t)__shfl((int)r, sl - s0 < cnt ? src : 0, 64);
        er = sl - s0 < cnt ? v : er;
    };
    // End of a run: every epoch lane finishes its image.
    auto finish_run = [&](uint64_t r) {
        const bool valid = valid_of(r);
        const uint64_t item = item_of(r);
        const bool fused = est & kStFused, sane = est & kStSane;
        const uint32_t pad = est & 15u;
        // (every lane: a lane-distributed value read under a branch would come
        // from lanes the branch left inactive)
        const uint32_t xt = MODE == 0 ? (uint32_t)__shfl((int)xinv, (int)pad, 64) : 0u;
        uint32_t v = 0;  // W = M_128(V) = M_{pad + 128}(f)
        if (fused) {
            const uint32_t dl = p_eta - (kBlockBytes - kLineBytes);  // d = Et - A - 3968
            uint32_t y = apply_op<4>(kAuxSpanFold, apply_op<4>(kAuxSpanFold, r_h)) ^ er;
            if (dl & 256u) y = apply_op<4>(kAuxTree + 12, apply_op<4>(kAuxTree + 12, y));
            if (dl & 128u) y = apply_op<4>(kAuxTree + 12, y);
            if (dl & 64u) y = apply_op<4>(kAuxTree + 8, y);
            if (dl & 32u) y = apply_op<4>(kAuxTree + 4, y);
            if (dl & 16u) y = apply_op<4>(kAuxTree, y);
            v = zeros_lds(y, dl & 15u, c) ^ apply_op<4>(kAuxTree + 12, r_t);
        }
        if (valid) {
            if (MODE == 0) {
                a.out[item] = fused ? ~mulmodp_dev(v, xt) : 0u;
                nb += !sane;  // (out of the buffer: not read, out 0, counted)
            } else if (MODE == 1) {
                if (fused || !sane) {
                    const bool good = fused && v == apply_op<4>(kAuxTree + 12, zeros_lds(~p_stored, pad, c));
                    a.ok[item] = good;
                    nb += !good;
                }
            } else {
                io.rt[item] = fused ? make_uint2(v, pad | kRtFused) : make_uint2(0u, 0u);
                if (!sane) {
                    if (a.ok) a.ok[item] = 0;
                    ++nb;
                }
            }
        }
        if (MODE != 0) {
            const bool fb = valid && sane && !fused;
            const uint64_t m = __ballot(fb);  // the fallback list: one atomic per wave with entries
            if (m) {
                const uint32_t first = (uint32_t)__ffsll((unsigned long long)m) - 1u;
                uint32_t base = 0;
                if (lane == first) base = atomicAdd(io.nfb, (uint32_t)__popcll(m));
                base = __shfl(base, (int)first, 64);
                if (fb) io.fb[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)item;
            }
        }
    };
    ItemBuf ra, rb;
    for (uint64_t r = 0; run_start(r) < cend; ++r) {
        const uint64_t left = cend - run_start(r);
        const uint32_t ns = (uint32_t)min(run_steps(r), (left + 1) / 2);
        prep_head(r);
        // the head and tail lines of neighbouring images are the same lines:
        // both loads at once, so one image's tail and the next image's head
        // are fetched together (tail loads after the head chain came ~2 us
        // later and fetched the shared line again: 1.036x for config 2r)
        head_loads();
        tail_loads();
        __builtin_amdgcn_sched_barrier(0);  // (not sunk towards the tail chain)
        // the next run's offsets (and initial CRCs), consumed one run later
        noff = off_of(r + 1);
        if (MODE == 0) ncin = a.crc_in && valid_of(r + 1) ? a.crc_in[item_of(r + 1)] : 0u;
        head_chain();
        ld(ra, 0, ns);  // (after the head chain: its registers are free again)
        tail_chain();
        er = 0;
        uint32_t s = 0;
        for (; s + 4 <= ns; s += 4) {
            ld(rb, s + 1, ns);
            const uint32_t va = part0(ra);
            ld(ra, s + 2, ns);
            const uint32_t vb = part0(rb);
            const uint32_t vab = group_pair_level1(va, vb, lane);
            ld(rb, s + 3, ns);
            const uint32_t vc = part0(ra);
            ld(ra, s + 4, ns);
            const uint32_t vd = part0(rb);
            collect(group_reduce32_quad_span(vab, group_pair_level1(vc, vd, lane), lane), s, 4);
        }
        for (; s + 2 <= ns; s += 2) {
            ld(rb, s + 1, ns);
            const uint32_t va = part0(ra);
            ld(ra, s + 2, ns);
            const uint32_t vb = part0(rb);
            collect(group_reduce32_pair_span(va, vb, lane), s, 2);
        }
        if (s < ns) {
            const uint32_t v = part0(ra);
            // (part0 ran level 0; levels 1..4 of the span tree)
            uint32_t t = reduce_level<1>(v, (lane & 3u) == 0u);
            t = reduce_level<2>(t, (lane & 7u) == 0u);
            t = reduce_level<3>(t, (lane & 15u) == 0u);
            t = reduce_level4_span(t, (lane & 31u) == 0u);
            collect(t, s, 1);
        }
        finish_run(r);
    }
    // one atomic per wave for the bad count
    nb += __shfl_xor(nb, 1);
    nb += __shfl_xor(nb, 2);
    nb += __shfl_xor(nb, 4);
    nb += __shfl_xor(nb, 8);
    nb += __shfl_xor(nb, 16);
    nb += __shfl_xor(nb, 32);
    if (lane == 0 && nb) atomicAdd(a.nbad, (unsigned long long)nb);
}


// The last step of a K5 stamp (MODE 2), one thread per image: from W =
// M_{t + 128}(f), f the register after the span from ~0, the CRC is
// ~M_{-t-128}(W) (xm128 = x^(-8 * 128)), stamped into
// the image's exptime as the spill CRC (storage.c:567).  A separate pass:
// within k_lines an image's stamp could race with another wave's read of the
// same bytes when images overlap.  (MODE 0 spans get their CRC from the epoch
// lanes of k_lines itself.)
__global__ void k_fix(SpanArgs a, const uint2 *rt, const uint32_t *route, uint32_t xm128) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    if (route && *route == 0) return;  // (k_lines took no image)
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < a.n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint2 r = rt[i];
        if (r.y & kRtFused) {
            const uint32_t crc = ~mulmodp_dev(mulmodp_dev(r.x, xm128), a.xpow[kXpowInv + (r.y & 15u)]);
            uint8_t *p = const_cast<uint8_t *>(a.base) + a.offsets[i] + 32;
            // non-temporal: plain stores left 16 M dirty 32-B sectors in the
            // caches, written back while the next batch streamed (its
            // k_lines<2> 0.11 ms slower per 300 pages); so the write-backs
            // happen here (k_fix 0.17 -> 0.25 ms), stamp -1.2 % in all
            // (profiles/r04_ablations/k_fix_nontemporal_ab.txt)
            for (int b = 0; b < 4; ++b) __builtin_nontemporal_store((uint8_t)(crc >> (8 * b)), p - 4 + b);
            if (a.ok) a.ok[i] = 1;
        }
    }
}

// K5 or the planned path, decided on the device (round 4; it was the host's
// guess from the batch's average image size, which a mix of short and long
// images can match): the headers of up to kCensus images spread evenly over
// the batch, and *route = 1 when at least 15/16 of them have K5's shape (one
// 4 KiB block after a short head fragment).  Below that the images K5 leaves
// to its fallback cost a second pass, and the planned path takes the batch
// (k_lines then lists every image).  One workgroup, one header per thread.
constexpr uint32_t kCensus = 1024;
template <int MODE>
__global__ __launch_bounds__(kCensus) void k_census(SpanArgs a, uint32_t *route) {
    MCRC_VGPR_FLOOR();
    __shared__ uint32_t cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const uint64_t n = a.n, s = min(n, (uint64_t)kCensus);
    if (threadIdx.x < s) {
        const uint64_t i = threadIdx.x * n / s;
        const ItemDesc it = fetch_item<MODE>(a, i);
        const uint64_t pa = (uintptr_t)it.p, A = (pa + 4 + kLineBytes - 1) & ~(uint64_t)(kLineBytes - 1);
        const uint64_t B = (pa + it.len) & ~(uint64_t)(kLineBytes - 1);
        const bool fused = it.len >= 4 && lines_fused((int64_t)B - (int64_t)A);
        if (it.sane && fused) atomicAdd(&cnt, 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) *route = 16ull * cnt >= 15ull * s ? 1u : 0u;
}

// Fallback lists: gather the listed items' offsets / scatter their results.
// (route 0, k_census: k_lines took no image, the list is every image: the
// identity)
__global__ void k_gather_offs(const uint64_t *offsets, const uint32_t *idx, const uint32_t *nidx, uint64_t *out,
                              const uint32_t *route) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    const uint32_t nn = *nidx;
    const bool all = route && *route == 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x)
        out[i] = offsets[all ? i : idx[i]];
}
__global__ void k_scatter_ok(const uint8_t *ok_in, const uint32_t *idx, const uint32_t *nidx, uint8_t *ok,
                             const uint32_t *route) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    const uint32_t nn = *nidx;
    const bool all = route && *route == 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x)
        ok[all ? i : idx[i]] = ok_in[i];
}

// Chained CRC over an iov list (the chunked-item read verify of
// storage.c:163-170: crc = crc32c(0, iov0 + 32, ...), then
// crc = crc32c(crc, iov_x) for every chunk).  Given crc_i = crc32c(0, iov_i),
// crc32c(c, B) = crc32c(0, B) ^ M_|B|(c), so chain c folds
//   acc = M_{len_i}(acc) ^ crc_i   over its iovs [first[c], first[c+1]).
// One thread per chain.
__global__ void k_chain(const uint32_t *iov_crc, const uint32_t *lens, uint32_t len, const uint64_t *first,
                        uint64_t nchains, uint32_t *out, const uint32_t *xpow) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchains;
         c += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t acc = 0;
        for (uint64_t i = first[c]; i < first[c + 1]; ++i) {
            const uint32_t l = lens ? lens[i] : len;
            if (acc) acc = mulmodp_dev(acc, xpow8_dev(xpow, l));
            acc ^= iov_crc[i];
        }
        out[c] = acc;
    }
}

// Device-side page walk (storage_compact_readback, storage.c:950-1070): the
// buffer is a sequence of wbuf-sized reads; in each, items are packed from
// offset 0, nkey == 0 ends the wbuf, the next item is at + ITEM_ntotal, and the
// walk stops when fewer than sizeof(item) = 48 bytes remain.  Two passes:
//   k_walk<false>: count the items of wbuf w into cnt[w];
//   (exclusive scan of the counts: prefix[w] = the index of wbuf w's first item)
//   k_walk<true>: walk again and write item prefix[w] + c's offset and, for a
//     planned verify, its plan entries (count_item: what k_count would write
//     after reading the header a second time), so no k_count pass follows.
// Round 4: the count pass also keeps the first kslot offsets of each wbuf
// (out.slots), and the emit pass of a verify that needs offsets only (K5)
// copies them instead of walking a wbuf again (the second walk re-read every
// header line from HBM: 0.15 ms per 300 pages); a wbuf of more than kslot
// items is walked again as before.
// One wave per wbuf.  The walk is a dependent chain, so each round trip
// guesses: lane j reads the header at off + j * s, s = the last item's
// ITEM_ntotal.  Lane j's guess is right iff every lane before it holds an item
// of exactly s bytes; the first lane m where that fails (a ballot) still sits
// on a true item boundary, so lanes [0, m) are items, lane m is one too unless
// it ends the wbuf (nkey == 0, or fewer than 48 bytes left), and the walk goes
// on from lane m's item end with s = its ntotal.  Whatever the data, the
// result is the sequential walk's (tests/test_walk_model.py restates it);
// equal-sized items cost one round trip per 64 of them.  Round 6: after a
// round trip whose guesses broke at lane 0 or 1 the next one guesses once
// (lane 0 alone reads a header), and widens again when that guess holds.
constexpr uint32_t kWalkWaves = 4;  // waves (wbufs) per workgroup

struct WalkOut {
    uint32_t *cnt;           // count pass: items per wbuf
    const uint32_t *prefix;  // emit pass: index of each wbuf's first item (nw + 1 entries)
    uint64_t *offs;          // emit pass: item offsets from base
    uint64_t *nunit;         // emit pass, planned verify (else nullptr): k_count's entries
    uint4 *irec;
    uint8_t *fast;
    unsigned long long *err; // emit pass: wbufs whose two walks disagree (must stay 0)
    uint64_t *slots;         // count pass: the first kslot item offsets of wbuf w at w * kslot
    uint32_t kslot;          // (0: none kept)
};

// a: base, base_bytes (the walked bytes), region (= wbuf), and for the plan
// entries xpow, tab8, span_acc.
template <bool EMIT>
__global__ __launch_bounds__(64 * kWalkWaves) void k_walk(SpanArgs a, uint64_t nw, WalkOut out) {
    MCRC_VGPR_FLOOR();  // (several workgroups per CU: crc32c_device.h)
    __shared__ __attribute__((aligned(16))) uint32_t s8[EMIT ? kTab8Dwords : 1];
    Tab8 t8{s8};
    const bool plan = EMIT && out.irec;
    if (plan) t8 = load_tab8(s8, a.tab8);
    const uint32_t j = threadIdx.x & 63u;
    const uint64_t wbuf = a.region;
    // the wave's wbuf index as a scalar: the walk state (off, s, c) is then
    // wave-uniform in the compiler's view too, and the loops are scalar loops
    // (with the index in a VGPR the walk went wrong on large page sets)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t w = (uint64_t)blockIdx.x * kWalkWaves + wave; w < nw; w += (uint64_t)gridDim.x * kWalkWaves) {
        const uint64_t start = w * wbuf, size = a.base_bytes - start < wbuf ? a.base_bytes - start : wbuf;
        const uint8_t *wb = a.base + start;
        const uint64_t first = EMIT ? out.prefix[w] : 0;
        // the count pass's item count of this wbuf: the emit pass never writes
        // past it (into the next wbuf's slots) and checks that it walks the
        // same number of items (the walk invariant; see DESIGN.md section 3 on
        // the round-2 readlane variants that broke it)
        const uint64_t expect = EMIT ? out.prefix[w + 1] - first : 0;
        if (EMIT && !plan && out.slots && expect <= out.kslot) {  // the count pass kept them all
            for (uint64_t i = j; i < expect; i += 64) out.offs[first + i] = out.slots[w * out.kslot + i];
            continue;
        }
        uint64_t off = 0, s = 0;  // wave-uniform: next item, stride guess (0: none yet)
        uint32_t c = 0;           // items walked so far
        // guesses this round trip: 64, or 1 after a round trip whose guesses
        // broke at once (round 6: a wbuf of mixed sizes breaks every guess at
        // its first lane, and 63 wasted header reads per item flooded HBM --
        // 19 us per round trip on the mixed pages; one read per item until a
        // size repeats)
        uint32_t wid = 1;
        while (off + 48 <= size) {
            const uint64_t o = off + j * s;
            const bool in = j < wid && (j == 0 || s != 0) && o + 48 <= size;  // (s < 2^33: no overflow)
            ItemHdr h{0u, 0u, 0u, 0u};
            if (in) h = parse_hdr(wb + o);
            const uint64_t nt = h.ntotal(a.cfl);
            const bool item = in && h.nkey != 0;
            // m = the first lane whose successor's guess is wrong (wid: none;
            // lanes past wid guessed nothing)
            const uint64_t brk = __ballot(!(item && nt == s)) & (wid >= 64u ? ~0ull : (1ull << wid) - 1ull);
            const uint32_t m = brk ? (uint32_t)__ffsll((unsigned long long)brk) - 1u : wid;
            // lane m (if any) is on a true boundary: an item, or the end of the
            // wbuf.  Its flag and size are read out of lane m into scalars
            // (v_readlane: the walk state is scalar).  Round 6: the walk kept
            // its state in VGPRs through round 5, broadcast with ds_bpermute,
            // because readlane variants had gone wrong on large page sets in
            // round 2 -- the 64-bit shift hazard of the header parse (DESIGN.md
            // 3.6), since removed; the bpermutes' LDS round trips were most of
            // a narrow round trip's time
            const uint32_t src = m < wid ? m : 0u;
            const bool last_item = m < wid && __builtin_amdgcn_readlane((int)item, (int)src) != 0;
            const uint64_t nt_m = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)nt, (int)src) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(nt >> 32), (int)src)
                                   << 32);
            const uint32_t k = m < wid ? m + (last_item ? 1u : 0u) : wid;  // items this round trip
            if (!EMIT && out.slots && j < k && c + j < out.kslot) out.slots[w * out.kslot + c + j] = start + o;
            if (EMIT && j < k && c + j < expect) {
                const uint64_t i = first + c + j;
                out.offs[i] = start + o;
                if (plan) count_item<1>(a, i, item_desc(a, start + o, h, true), t8, out.nunit, out.irec, out.fast);
            }
            c += k;
            if (m == wid) {
                off += wid * s;  // every guess right: the size repeats
                wid = 64u;
            } else if (!last_item) {
                break;  // lane m ends the wbuf
            } else {
                off += m * s + nt_m;
                s = nt_m;
                wid = m <= 1u ? 1u : 64u;
            }
        }
        if (!EMIT && j == 0) out.cnt[w] = c;
        if (EMIT && j == 0 && c != expect) atomicAdd(out.err, 1ull);
    }
}

}  // namespace mcrc_dev
