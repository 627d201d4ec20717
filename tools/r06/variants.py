"""Build A/B variants of libmcrc32c.so from edited copies of the sources
(ab/NAME/src -> ab/NAME/libmcrc32c.so), so that the product sources carry no
build switch.  Each variant is a list of (file, old, new) text edits; a
missing `old` text fails the build.

    python tools/r06/variants.py NAME [NAME ...]      # cur, lnst, lnc, git:REV
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# The in-kernel stamp (round-6 review item 3): k_lines<2>'s epoch lane stores
# the CRC into exptime at the end of its run (and ok = 1), no k_fix pass.
_LN_FINISH_OLD = """                io.rt[item] = fused ? make_uint2(v, pad | kRtFused) : make_uint2(0u, 0u);
                if (!sane) {"""
_LN_FINISH_NEW = """                if (fused) {
                    const uint32_t crc = ~mulmodp_dev(v, a.xpow[kXpowInv + pad]);
                    uint8_t *q = const_cast<uint8_t *>(a.base) + p_pho + p_kh - 4;  // exptime (off + 28)
                    STAMP_STORE
                    if (a.ok) a.ok[item] = 1;
                }
                if (!sane) {"""
_LN_SHIM_OLD = "    if (MODE == 2) {\n        // k_fix (the stamps"
_LN_SHIM_NEW = "    if (MODE == 2 && false) {\n        // k_fix (the stamps"
_NT = ("for (int b = 0; b < 4; ++b) __builtin_nontemporal_store((uint8_t)(crc >> (8 * b)), q + b);")
_PLAIN = "for (int b = 0; b < 4; ++b) q[b] = (uint8_t)(crc >> (8 * b));"

# K5's runs dealt in chunks of 16 consecutive runs (about one 4 MiB wbuf of
# 4165-B images) instead of one run at a time: the locality a K5 that walks
# its own wbufs would have
_RUN_OLD = "    auto run_start = [&](uint64_t k) -> uint64_t { return (k * W + w0) * run_imgs; };"
_RUN_NEW = ("    auto run_start = [&](uint64_t k) -> uint64_t { return (((k >> 4) * W + w0) * 16 + (k & 15)) * run_imgs; };")

# K1 with the table image's 32 replicas used as 16 (lanes l and l + 16 read
# the same replica: the two-way bank conflicts of a half-replicated image, the
# room an LDS-DMA K1 would stage into), same instructions otherwise
_K1_LANE_OLD = "    c.lane4 = li << 2;\n    c.lane4hi = c.lane4 | 0x10000u;\n    const uint64_t waves = blockDim.x >> 6;"
_K1_LANE_NEW = "    c.lane4 = (li & 15u) << 2;\n    c.lane4hi = c.lane4 | 0x10000u;\n    const uint64_t waves = blockDim.x >> 6;"

# load_block with one address per lane and the loads' immediate offsets when
# every piece of every lane of the wave lies at or past its span's first
# piece (every block but a unit's head block): no per-piece select
_LB_OLD = """#pragma unroll
    for (int j = 0; j < (int)kK1Pieces; ++j) {
        const uint8_t *q = e0 + j * (int32_t)kK1Piece > 0 ? q0 + j * kK1Piece : zl;
        w.v[j] = kSpanNT ? ld16_nt(q) : ld16(q);
    }
}"""
_LB_NEW = """    if (__builtin_amdgcn_readfirstlane(__all(e0 > 0))) {
#pragma unroll
        for (int j = 0; j < (int)kK1Pieces; ++j) w.v[j] = kSpanNT ? ld16_nt(q0 + j * kK1Piece) : ld16(q0 + j * kK1Piece);
    } else {
#pragma unroll
        for (int j = 0; j < (int)kK1Pieces; ++j) {
            const uint8_t *q = e0 + j * (int32_t)kK1Piece > 0 ? q0 + j * kK1Piece : zl;
            w.v[j] = kSpanNT ? ld16_nt(q) : ld16(q);
        }
    }
}"""

# k_spans<true>'s record cursor and share end in 32 bits (a plan holds fewer
# than 2^32 records): two VGPRs fewer where the kernel spills
_U32_OLD = """    uint64_t u = g;
    uint64_t ub = nunits;  // the group's records (of this round) end here"""
_U32_NEW = """    // (UNITS: a plan holds fewer than 2^32 records -- 32-bit cursors, two
    // VGPRs fewer)
    using Idx = typename std::conditional<UNITS, uint32_t, uint64_t>::type;
    Idx u = g;
    Idx ub = (Idx)nunits;  // the group's records (of this round) end here"""
_U32S_OLD = "    const uint64_t ustep = bal ? 1u : ngroups_total;"
_U32S_NEW = "    const Idx ustep = bal ? 1u : (Idx)ngroups_total;"

# the lane index re-derived (v_mbcnt, volatile: not hoisted) where a unit
# switch uses it, so that no lane constant is live across the block loop
_RM_OLD = """        UnitDesc nd;
        if (__any(last)) {
            const uint32_t g = lane & 32u, sb = sl << 3;
            const uint32_t rw = __shfl(ring, g | sb | (li & 7u), 64);  // slot sl, dword li & 7
            nd = decode_unit<UNITS>(a, rw, u + ustep, nunits, lane);
        }
        if (last && (li >> 3) == sl) ring = fetch_unit<UNITS>(a, u + 5 * ustep, ub, li);"""
_RM_NEW = r"""        UnitDesc nd;
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const uint32_t lj = ln & 31u;
        if (__any(last)) {
            const uint32_t g = ln & 32u, sb = sl << 3;
            const uint32_t rw = __shfl(ring, g | sb | (lj & 7u), 64);  // slot sl, dword li & 7
            nd = decode_unit<UNITS>(a, rw, u + ustep, nunits, ln);
        }
        if (last && (lj >> 3) == sl) ring = fetch_unit<UNITS>(a, u + 5 * ustep, ub, lj);"""

# k_spans: a block's first and last 512-B piece rows (lines a span's head or
# tail block may share with its neighbour span, which the same group takes
# next in a balanced plan) with the default policy, the rest non-temporal
_EDGE_OLD = """        w.v[j] = kSpanNT ? ld16_nt(q) : ld16(q);"""
_EDGE_NEW = """        w.v[j] = kSpanNT && j != 0 && j != (int)kK1Pieces - 1 ? ld16_nt(q) : ld16(q);"""

VARIANTS = {
    "cur": [],
    "edgecache": [("crc32c_kernels.hip", _EDGE_OLD, _EDGE_NEW)],
    "remat": [("crc32c_kernels.hip", _RM_OLD, _RM_NEW)],
    "u32remat": [("crc32c_kernels.hip", _U32_OLD, _U32_NEW), ("crc32c_kernels.hip", _U32S_OLD, _U32S_NEW),
                 ("crc32c_kernels.hip", _RM_OLD, _RM_NEW)],
    "u32": [("crc32c_kernels.hip", _U32_OLD, _U32_NEW), ("crc32c_kernels.hip", _U32S_OLD, _U32S_NEW)],
    "lbfast": [("crc32c_kernels.hip", _LB_OLD, _LB_NEW)],
    "k1half": [("crc32c_kernels.hip", _K1_LANE_OLD, _K1_LANE_NEW)],
    "chunk16": [("crc32c_kernels.hip", _RUN_OLD, _RUN_NEW)],
    # byte-wise non-temporal stores, as k_fix's
    "lnst": [("crc32c_kernels.hip", _LN_FINISH_OLD, _LN_FINISH_NEW.replace("STAMP_STORE", _NT)),
             ("crc32c_shim.hip", _LN_SHIM_OLD, _LN_SHIM_NEW)],
    # byte-wise default-policy stores
    "lnc": [("crc32c_kernels.hip", _LN_FINISH_OLD, _LN_FINISH_NEW.replace("STAMP_STORE", _PLAIN)),
            ("crc32c_shim.hip", _LN_SHIM_OLD, _LN_SHIM_NEW)],
}


def build(name):
    """NAME from VARIANTS, or git:REV -- the sources of commit REV (built into ab/REV)."""
    rev = name[4:] if name.startswith("git:") else None
    out = os.path.join(ROOT, "ab", rev or name)
    src = os.path.join(out, "src")
    shutil.rmtree(out, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "memcached_amd", "csrc"), os.path.join(src, "memcached_amd", "csrc"),
                    ignore=shutil.ignore_patterns("_obj"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(src, "include"))
    csrc = os.path.join(src, "memcached_amd", "csrc")
    if rev:
        for d, files in (("memcached_amd/csrc", os.listdir(csrc)), ("include", os.listdir(os.path.join(src, "include")))):
            for f in files:
                text = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{d}/{f}"], check=True, capture_output=True).stdout
                open(os.path.join(src, d, f), "wb").write(text)
    for f, old, new in ([] if rev else VARIANTS[name]):
        p = os.path.join(csrc, f)
        text = open(p).read()
        if old not in text:
            raise SystemExit(f"{name}: edit target not found in {f}")
        open(p, "w").write(text.replace(old, new, 1))
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-c", os.path.join(csrc, "crc32c_host.cpp"), "-o",
                    os.path.join(out, "host.o")], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                    os.path.join(csrc, "crc32c_shim.hip"), "-o", os.path.join(out, "shim.o")], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(out, "libmcrc32c.so"), os.path.join(out, "shim.o"), os.path.join(out, "host.o"),
                    "-lpthread"], check=True)
    for o in ("host.o", "shim.o"):
        os.remove(os.path.join(out, o))
    print(f"built ab/{rev or name}/libmcrc32c.so")


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
