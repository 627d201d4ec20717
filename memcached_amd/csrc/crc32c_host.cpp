// crc32c_host.cpp -- host CRC-32C used by the scalar drop-in symbol.
#include "crc32c_host.h"

#include <mutex>

#include "crc32c_gf2.h"

#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#elif defined(__aarch64__)
#include <arm_acle.h>
#include <sys/auxv.h>
#ifndef HWCAP_CRC32
#define HWCAP_CRC32 (1ul << 7)
#endif
#endif

namespace mcrc {

namespace {

std::once_flag g_once;
uint32_t g_slice[8][256];           // g_slice[k][b]: byte b followed by k zero bytes
constexpr size_t kStreamBlock = 4096;  // bytes per stream per round of the 3-way loop
uint32_t g_shift_block[4][256];     // M_{kStreamBlock}
uint32_t g_shift_small[4][256];     // M_{kSmallBlock}
constexpr size_t kSmallBlock = 256;
uint64_t g_big[8][256];             // big-endian word tables: g_slice[k][b] byte-reversed into bits 32..63

void build_all() {
    build_t0(g_slice[0]);
    for (int k = 1; k < 8; ++k)
        for (int b = 0; b < 256; ++b) {
            const uint32_t prev = g_slice[k - 1][b];
            g_slice[k][b] = g_slice[0][prev & 0xffu] ^ (prev >> 8);
        }
    for (int k = 0; k < 8; ++k)
        for (int b = 0; b < 256; ++b) g_big[k][b] = (uint64_t)__builtin_bswap32(g_slice[k][b]) << 32;
    Gf2Op::zeros(kStreamBlock).byte_tables(g_shift_block);
    Gf2Op::zeros(kSmallBlock).byte_tables(g_shift_small);
}

inline uint32_t apply4(const uint32_t t[4][256], uint32_t v) {
    return t[0][v & 0xffu] ^ t[1][(v >> 8) & 0xffu] ^ t[2][(v >> 16) & 0xffu] ^ t[3][v >> 24];
}

inline uint64_t load64(const unsigned char *p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

// Register-level slice-by-8 (no pre/post inversion).
uint32_t reg_sw(uint32_t r, const unsigned char *p, size_t n) {
    while (n && ((uintptr_t)p & 7u)) {
        r = g_slice[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
        --n;
    }
    for (; n >= 8; n -= 8, p += 8) {
        const uint64_t x = load64(p) ^ r;
        r = g_slice[7][x & 0xffu] ^ g_slice[6][(x >> 8) & 0xffu] ^ g_slice[5][(x >> 16) & 0xffu] ^
            g_slice[4][(x >> 24) & 0xffu] ^ g_slice[3][(x >> 32) & 0xffu] ^
            g_slice[2][(x >> 40) & 0xffu] ^ g_slice[1][(x >> 48) & 0xffu] ^ g_slice[0][x >> 56];
    }
    while (n--) r = g_slice[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
    return r;
}

// The big-endian slice-by-8 of crc32c.c:467-498 (crc32c_sw_big), evaluated
// with this host's native 64-bit loads, as the reference's exported function
// is: the register is kept byte-reversed in the upper half of a 64-bit word,
// each aligned data word (native load) is XORed in, and byte j of the word
// (j = 0 the low-order byte) indexes the word table of j trailing zero bytes.
// On a big-endian host that is CRC-32C; on a little-endian host it is the
// reference's same (non-CRC) function, which callers only reach through
// crc32c_sw_big itself (crc32c_sw dispatches by endianness, crc32c.c:507-513).
uint32_t reg_sw_big(uint32_t r, const unsigned char *p, size_t n) {
    while (n && ((uintptr_t)p & 7u)) {
        r = g_slice[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
        --n;
    }
    if (n >= 8) {
        uint64_t w = (uint64_t)__builtin_bswap32(r) << 32;
        for (; n >= 8; n -= 8, p += 8) {
            w ^= load64(p);
            uint64_t acc = 0;
            for (int j = 0; j < 8; ++j) acc ^= g_big[j][(w >> (8 * j)) & 0xffu];
            w = acc;
        }
        r = (uint32_t)__builtin_bswap64(w);
    }
    while (n--) r = g_slice[0][(r ^ *p++) & 0xffu] ^ (r >> 8);
    return r;
}

// The CRC32C instruction: SSE4.2 crc32 on x86-64; on arm64 the ARMv8 CRC
// extension's crc32cb / crc32cx (crc32c.c:285-336 uses the latter the same way).
#if defined(__x86_64__)
#define HOST_CRC_TARGET __attribute__((target("sse4.2")))
HOST_CRC_TARGET inline uint64_t hw_u64(uint64_t r, uint64_t v) { return _mm_crc32_u64(r, v); }
HOST_CRC_TARGET inline uint64_t hw_u8(uint64_t r, unsigned char b) { return _mm_crc32_u8((uint32_t)r, b); }
#elif defined(__aarch64__)
// (GCC spells the extension "+crc", clang "crc")
#if defined(__clang__)
#define HOST_CRC_TARGET __attribute__((target("crc")))
#else
#define HOST_CRC_TARGET __attribute__((target("+crc")))
#endif
HOST_CRC_TARGET inline uint64_t hw_u64(uint64_t r, uint64_t v) { return __crc32cd((uint32_t)r, v); }
HOST_CRC_TARGET inline uint64_t hw_u8(uint64_t r, unsigned char b) { return __crc32cb((uint32_t)r, b); }
#endif

#if defined(HOST_CRC_TARGET)
// Three streams of `blk` bytes per round: the crc32 instruction has a latency of
// three and a throughput of one (x86-64; arm64 cores are alike), so three
// independent chains keep it busy.
HOST_CRC_TARGET uint64_t three_way(uint64_t r, const unsigned char *&p, size_t &n, size_t blk,
                                  const uint32_t (*shift)[256]) {
    while (n >= 3 * blk) {
        uint64_t a = r, b = 0, c = 0;
        const unsigned char *pa = p, *pb = p + blk, *pc = p + 2 * blk;
        for (size_t i = 0; i < blk; i += 8) {
            a = hw_u64(a, load64(pa + i));
            b = hw_u64(b, load64(pb + i));
            c = hw_u64(c, load64(pc + i));
        }
        r = apply4(shift, apply4(shift, (uint32_t)a) ^ (uint32_t)b) ^ (uint32_t)c;
        p += 3 * blk;
        n -= 3 * blk;
    }
    return r;
}

HOST_CRC_TARGET uint32_t reg_hw(uint32_t r32, const unsigned char *p, size_t n) {
    uint64_t r = r32;
    while (n && ((uintptr_t)p & 7u)) {
        r = hw_u8(r, *p++);
        --n;
    }
    r = three_way(r, p, n, kStreamBlock, g_shift_block);
    r = three_way(r, p, n, kSmallBlock, g_shift_small);
    for (; n >= 8; n -= 8, p += 8) r = hw_u64(r, load64(p));
    while (n--) r = hw_u8(r, *p++);
    return (uint32_t)r;
}
#endif

}  // namespace

void host_tables_init() { std::call_once(g_once, build_all); }

bool host_has_hw_crc() {
#if defined(__x86_64__)
    unsigned eax, ebx, ecx, edx;
    if (!__get_cpuid(1, &eax, &ebx, &ecx, &edx)) return false;
    return (ecx >> 20) & 1u;  // SSE4.2
#elif defined(__aarch64__)
    return (getauxval(AT_HWCAP) & HWCAP_CRC32) != 0;  // crc32c.c:266-275 probes the same
#else
    return false;
#endif
}

uint32_t crc32c_host_sw(uint32_t crc, const void *buf, size_t len) {
    host_tables_init();
    return ~reg_sw(~crc, static_cast<const unsigned char *>(buf), len);
}

uint32_t crc32c_host_sw_big(uint32_t crc, const void *buf, size_t len) {
    host_tables_init();
    return ~reg_sw_big(~crc, static_cast<const unsigned char *>(buf), len);
}

uint32_t crc32c_host_hw(uint32_t crc, const void *buf, size_t len) {
    host_tables_init();
#if defined(HOST_CRC_TARGET)
    return ~reg_hw(~crc, static_cast<const unsigned char *>(buf), len);
#else
    return ~reg_sw(~crc, static_cast<const unsigned char *>(buf), len);
#endif
}

uint32_t crc32c_host_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    // crc(A||B) = ~(M_|B|(~crc(A)) ^ raw(B)), raw(B) = ~crc_b ^ M_|B|(~0)
    // => crc(A||B) = M_|B|(crc_a) ^ crc_b   (the ~ terms cancel by linearity)
    return mulmodp(crc_a, xpow8n(len_b)) ^ crc_b;
}

}  // namespace mcrc
