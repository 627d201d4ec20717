"""The gfx950 code object inside libmcrc32c.so: register allocation of every
product kernel (no GPU needed).

The page-walk experiment (tools/walk_hazard.hip) found a
kernel whose identical instruction stream walks wrongly when it is allocated
24 VGPRs and several workgroups share a CU, and exactly with 32, 40 or 48.
Every kernel therefore allocates at least 32 VGPRs (MCRC_VGPR_FLOOR,
crc32c_device.h); this test reads the allocation back from the built
library's kernel metadata.  Round 4: the planned path's prefix sums and the
walk's scan are the library's own kernels (k_plan_tiles, k_plan_scan,
k_scan32) instead of hipcub's, so the check covers every kernel in the code
object, not only the mcrc_dev ones.
"""
import os
import re
import shutil
import subprocess

import pytest

from memcached_amd import _lib

LLVM = "/opt/rocm/lib/llvm/bin"


def _code_object(tmp_path):
    lib = _lib.LIB_PATH
    if not os.path.exists(lib):
        pytest.skip("libmcrc32c.so not built")
    bundler = os.path.join(LLVM, "clang-offload-bundler")
    if not (shutil.which("objcopy") and os.path.exists(bundler)):
        pytest.skip("objcopy / clang-offload-bundler not available")
    fat = tmp_path / "fatbin.bin"
    co = tmp_path / "gfx950.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fat)], check=True)
    subprocess.run([bundler, "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def _kernels(co):
    notes = subprocess.run([os.path.join(LLVM, "llvm-readobj"), "--notes", str(co)], check=True,
                           capture_output=True, text=True).stdout
    out = {}
    for blk in notes.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
        agpr = int(blk.split()[1])
        lds = int(re.search(r"\.group_segment_fixed_size:\s+(\d+)", blk).group(1))
        out[name] = (vgpr, agpr, lds)
    return out


def test_every_kernel_allocates_at_least_32_vgprs(tmp_path):
    ks = _kernels(_code_object(tmp_path))
    # no third-party kernel (hipcub / rocprim) is left in the code object
    assert all("mcrc_dev" in n for n in ks), [n for n in ks if "mcrc_dev" not in n]
    # every kernel of crc32c_kernels.hip is in the library
    for k in ("k_fixed", "k_spans", "k_count", "k_expand", "k_expand_big", "k_final", "k_small", "k_blocks",
              "k_fix", "k_gather_offs", "k_scatter_ok", "k_chain", "k_walk", "k_plan_tiles",
              "k_plan_scan", "k_scan32", "k_census", "k_lines"):
        assert any(re.search(rf"\d{k}E", n) or re.search(rf"\d{k}I", n) for n in ks), k
    low = {n: v for n, (v, a, _) in ks.items() if ((v + 7) // 8) * 8 < 32}
    assert not low, f"kernels allocating fewer than 32 VGPRs: {low}"
    # and no kernel pays occupancy for the floor: the small per-thread kernels
    # stay within 64 VGPRs (8 waves per SIMD)
    for n, (v, a, lds) in ks.items():
        if any(f"{len(k)}{k}" in n for k in ("k_fix", "k_gather_offs", "k_scatter_ok", "k_chain")):
            assert v <= 64, (n, v)


_SHIFT64 = re.compile(r"\s(v_(?:lshlrev|lshrrev|ashrrev)_[bi]64)\s+(v\[\d+:\d+\]),\s*(\S+),")


def _disasm_by_function(co):
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)], check=True,
                         capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur:
            out[cur].append(line)
    return out


def test_no_64bit_shift_takes_its_amount_from_the_top_vgpr(tmp_path):
    """The named cause of the 24-VGPR header miscompute (DESIGN.md section
    3.7, tools/shift64_top_vgpr.hip): a 64-bit VALU shift whose amount operand
    is the last VGPR of the wave's allocation.  No instruction of the library
    may take that form, whatever the VGPR floor."""
    co = _code_object(tmp_path)
    ks = _kernels(co)
    fns = _disasm_by_function(co)
    bad, nshift = [], 0
    for name, (vgpr, _a, _l) in ks.items():
        top = f"v{((vgpr + 7) // 8) * 8 - 1}"
        assert name in fns, name
        for ins in fns[name]:
            m = _SHIFT64.search(ins)
            if m:
                nshift += 1
                if m.group(3) == top:
                    bad.append((name, ins.strip()))
    assert nshift > 0  # (the scan sees the library's shifts)
    assert not bad, bad


def test_parse_hdr_has_no_64bit_shift(tmp_path):
    """parse_hdr (crc32c_kernels.hip) funnels the header bytes with
    v_alignbyte_b32: a probe kernel holding only the parse, for both pointer
    types the library instantiates, has no 64-bit VALU shift."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "memcached_amd", "csrc")
    src = tmp_path / "probe.hip"
    src.write_text(
        '#include "crc32c_kernels.hip"\n'
        "using namespace mcrc_dev;\n"
        "__global__ void probe_flat(const uint8_t *p, uint32_t *o) {\n"
        "    const ItemHdr h = parse_hdr(p + threadIdx.x * 13u);\n"
        "    o[threadIdx.x] = h.exptime ^ h.nbytes * 3u ^ h.flags * 5u ^ h.nkey * 7u;\n"
        "}\n"
        "__global__ void probe_global(const uint8_t *p, uint32_t *o) {\n"
        "    gbyte *g = (gbyte *)p;\n"
        "    const ItemHdr h = parse_hdr(g + threadIdx.x * 13u);\n"
        "    o[threadIdx.x] = h.exptime ^ h.nbytes * 3u ^ h.flags * 5u ^ h.nkey * 7u;\n"
        "}\n")
    asm = tmp_path / "probe.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", csrc, "--cuda-device-only", "-S",
                    str(src), "-o", str(asm)], check=True, capture_output=True)
    # (the include brings the library's own kernels along: only the probes' bodies count)
    bodies = {}
    for blk in re.split(r"\n(?=_Z\S*:)", asm.read_text()):
        m = re.match(r"(_Z\S*probe_\w+?Pj):", blk)
        if m:
            bodies[m.group(1)] = blk.split("\t.section")[0]
    assert len(bodies) == 2, list(bodies)
    for name, body in bodies.items():
        assert "v_alignbyte_b32" in body and re.search(r"(global|flat)_load_dwordx4", body), name
        shifts = [ln.strip() for ln in body.splitlines() if re.search(r"\sv_(lshlrev|lshrrev|ashrrev)_[bi]64\s", ln)]
        assert not shifts, (name, shifts)


def test_no_build_switch_alternatives_in_the_product_sources():
    """One build of the product: no #if/#ifdef feature switch selects an
    untested alternative kernel path (round-4 review item 5)."""
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "memcached_amd", "csrc")
    bad = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h", ".cpp")):
            for i, line in enumerate(open(os.path.join(csrc, f)), 1):
                if re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b.*MCRC_", line):
                    bad.append(f"{f}:{i}: {line.strip()}")
    assert not bad, bad
