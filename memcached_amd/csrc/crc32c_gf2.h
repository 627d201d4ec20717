// crc32c_gf2.h -- host-side GF(2) operator algebra for CRC-32C (Castagnoli).
//
// The reference computes CRC-32C with a reflected register and the polynomial
// 0x82f63b78 (crc32c.c:50).  Its hardware path merges three interleaved
// streams with "zeros operators": 32x32 GF(2) matrices that advance a CRC
// register over n zero bytes, applied through four byte-indexed tables
// (crc32c.c:58-137).  This header is the build's own statement of that algebra;
// it produces every constant table the HIP kernels and the host shim use:
//
//   Z            one zero byte:      r' = T0[r & 0xff] ^ (r >> 8)
//   M_n = Z^n    n zero bytes;       M_n(r) = r * x^(8n) mod P
//   raw(D)       register after D from a zero register (linear in D)
//   crc32c(c, D) = ~( M_|D|(~c) ^ raw(D) )
//
// Everything here is plain integer arithmetic and runs once per table set.
#pragma once

#include <stdint.h>
#include <string.h>

namespace mcrc {

constexpr uint32_t kPoly = 0x82f63b78u;  // reflected Castagnoli, crc32c.c:50

// Register advanced by one zero bit: r * x mod P in the reflected basis.
inline uint32_t zero_bit(uint32_t r) { return (r >> 1) ^ ((r & 1u) ? kPoly : 0u); }

// Byte-wise Sarwate table: T0[b] = register after byte b from a zero register.
inline void build_t0(uint32_t t0[256]) {
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t r = b;
        for (int k = 0; k < 8; ++k) r = zero_bit(r);
        t0[b] = r;
    }
}

// A linear map on 32-bit CRC registers, stored by columns: col[i] = op(1 << i).
struct Gf2Op {
    uint32_t col[32];

    uint32_t apply(uint32_t v) const {
        uint32_t acc = 0;
        for (int i = 0; v; ++i, v >>= 1)
            if (v & 1u) acc ^= col[i];
        return acc;
    }
    // (this o other)(v) = this(other(v))
    Gf2Op after(const Gf2Op &other) const {
        Gf2Op out;
        for (int i = 0; i < 32; ++i) out.col[i] = apply(other.col[i]);
        return out;
    }
    static Gf2Op identity() {
        Gf2Op out;
        for (int i = 0; i < 32; ++i) out.col[i] = 1u << i;
        return out;
    }
    static Gf2Op one_zero_byte() {
        Gf2Op out;
        for (int i = 0; i < 32; ++i) {
            uint32_t r = 1u << i;
            for (int k = 0; k < 8; ++k) r = zero_bit(r);
            out.col[i] = r;
        }
        return out;
    }
    // M_n: advance over n zero bytes (square-and-multiply over Z).
    static Gf2Op zeros(uint64_t n) {
        Gf2Op result = identity();
        Gf2Op sq = one_zero_byte();
        while (n) {
            if (n & 1u) result = sq.after(result);
            n >>= 1;
            if (n) sq = sq.after(sq);
        }
        return result;
    }
    // Inverse map (Gauss-Jordan over GF(2)); M_n is invertible because the
    // polynomial has a constant term, so M_{-n} undoes n zero bytes.
    Gf2Op inverse() const {
        uint32_t a[32], b[32];  // rows of the matrix (bit j of row i = column j bit i) and of I
        for (int i = 0; i < 32; ++i) {
            a[i] = 0;
            for (int j = 0; j < 32; ++j) a[i] |= ((col[j] >> i) & 1u) << j;
            b[i] = 1u << i;
        }
        for (int c = 0; c < 32; ++c) {
            int r = c;
            while (r < 32 && !((a[r] >> c) & 1u)) ++r;
            if (r == 32) return identity();  // singular (cannot happen for M_n)
            uint32_t t = a[r]; a[r] = a[c]; a[c] = t;
            t = b[r]; b[r] = b[c]; b[c] = t;
            for (int i = 0; i < 32; ++i)
                if (i != c && ((a[i] >> c) & 1u)) {
                    a[i] ^= a[c];
                    b[i] ^= b[c];
                }
        }
        Gf2Op out;  // b holds the inverse by rows; convert back to columns
        for (int j = 0; j < 32; ++j) {
            out.col[j] = 0;
            for (int i = 0; i < 32; ++i) out.col[j] |= ((b[i] >> j) & 1u) << i;
        }
        return out;
    }
    // Four byte-slice tables so that apply(v) = t[0][v&255] ^ t[1][(v>>8)&255]
    // ^ t[2][(v>>16)&255] ^ t[3][v>>24]  (the form of crc32c.c:121-137).
    void byte_tables(uint32_t t[4][256]) const {
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) t[k][b] = apply(b << (8 * k));
    }
};

// Reflected-basis polynomial product a(x) * b(x) mod P (bit 31 is x^0).
inline uint32_t mulmodp(uint32_t a, uint32_t b) {
    uint32_t prod = 0;
    for (uint32_t m = 0x80000000u; m; m >>= 1) {
        if (a & m) prod ^= b;
        b = zero_bit(b);
    }
    return prod;
}

// x^(8n) mod P, reflected: multiplying a register by it advances n zero bytes.
inline uint32_t xpow8n(uint64_t n) {
    uint32_t result = 0x80000000u;  // x^0
    uint32_t sq = 0x00800000u;      // x^8
    while (n) {
        if (n & 1u) result = mulmodp(result, sq);
        n >>= 1;
        if (n) sq = mulmodp(sq, sq);
    }
    return result;
}

// x^(-8n) mod P: multiplying a register by it undoes n zero bytes.
inline uint32_t xpow8n_inv(uint64_t n) { return Gf2Op::zeros(n).inverse().apply(0x80000000u); }

// ---------------------------------------------------------------------------
// LDS table images for the HIP kernels (layouts documented in crc32c_device.h).
//   chunk = CH, bytes per lane per row.  Operator o = 0..6 fills aux tables
//   4o..4o+3: o <= 5 is M_{chunk * 2^o}, o = 6 is M_{128 * chunk}
//   (the 4-row block fold of the span kernels).
// ---------------------------------------------------------------------------
constexpr int kAux4Dwords = 28 * 256;                      // SLICE 4 aux: 28 KiB
constexpr int kImage4Dwords = kAux4Dwords + 2 * 16384;     // SLICE 4: 156 KiB
constexpr int kAuxTree = 0;
constexpr int kAuxFold = 24;

inline void aux_ops(uint32_t chunk, Gf2Op ops[7]) {
    for (int k = 0; k < 6; ++k) ops[k] = Gf2Op::zeros((uint64_t)chunk << k);
    ops[6] = Gf2Op::zeros((uint64_t)chunk * 128);
}

inline void build_lds_image4(uint32_t *img, uint32_t chunk) {
    memset(img, 0, sizeof(uint32_t) * kImage4Dwords);
    Gf2Op ops[7];
    aux_ops(chunk, ops);
    for (int o = 0; o < 7; ++o) {
        uint32_t tabs[4][256];
        ops[o].byte_tables(tabs);
        for (int k = 0; k < 4; ++k)
            for (uint32_t e = 0; e < 256; ++e) img[(4 * o + k) * 256 + e] = tabs[k][e];
    }
    uint32_t t[4][256];  // t[k][b]: byte b then k zero bytes
    build_t0(t[0]);
    for (int k = 1; k < 4; ++k)
        for (int b = 0; b < 256; ++b) t[k][b] = t[0][t[k - 1][b] & 0xffu] ^ (t[k - 1][b] >> 8);
    uint32_t *set_a = img + kAux4Dwords, *set_b = set_a + 16384;
    for (int e = 0; e < 256; ++e)
        for (int l = 0; l < 32; ++l) {
            set_a[e * 64 + l] = t[3][e];
            set_a[e * 64 + 32 + l] = t[2][e];
            set_b[e * 64 + l] = t[1][e];
            set_b[e * 64 + 32 + l] = t[0][e];
        }
}

// K1 image (160 KiB): the slice-by-4 image with the row fold absorbed into the
// last dword step of the first three row chains.  Row r of a lane (R = 4 rows
// of 32 * chunk bytes) must end up advanced by (3 - r) * 32 * chunk bytes; a
// zeros operator is linear, so it can be applied to the step's table values
// instead of to the chain's result:  S_r[j][b] = M_{(3-r)*32*chunk}(T_{3-j}[b])
// (table j is indexed by byte j of the step input).  S_2 and S_1 replace aux
// operators 5 and 6 (tables 20..27, unused by K1), S_0 takes tables 156..159
// ([156 KiB, 160 KiB)).  crc32c_device.h kAuxShift* names the slots.
constexpr int kImageK1Dwords = 160 * 256;

inline void build_lds_image_k1(uint32_t *img, uint32_t chunk) {
    build_lds_image4(img, chunk);
    uint32_t t[4][256];
    build_t0(t[0]);
    for (int k = 1; k < 4; ++k)
        for (int b = 0; b < 256; ++b) t[k][b] = t[0][t[k - 1][b] & 0xffu] ^ (t[k - 1][b] >> 8);
    const int slot[3] = {156, 24, 20};  // tables of S_0, S_1, S_2
    for (int r = 0; r < 3; ++r) {
        const Gf2Op m = Gf2Op::zeros((uint64_t)(3 - r) * 32 * chunk);
        for (int j = 0; j < 4; ++j)
            for (int b = 0; b < 256; ++b) img[(slot[r] + j) * 256 + b] = m.apply(t[3 - j][b]);
    }
}

// Span image (160 KiB): the K1 image with aux tables 16..19 (tree level 4,
// M_{16 chunk}) replaced by the block fold M_{128 chunk} (4 rows of 32 lanes).
// The span kernels apply level 3 twice for level 4 (once per unit, a few
// lanes) and fold every 4 KiB block into the lane accumulator with the freed
// tables; the row folds come from the shifted last-step tables as in K1.
inline void build_lds_image_span(uint32_t *img, uint32_t chunk) {
    build_lds_image_k1(img, chunk);
    uint32_t tabs[4][256];
    Gf2Op::zeros((uint64_t)chunk * 128).byte_tables(tabs);
    for (int k = 0; k < 4; ++k)
        for (uint32_t e = 0; e < 256; ++e) img[(16 + k) * 256 + e] = tabs[k][e];
}

}  // namespace mcrc
