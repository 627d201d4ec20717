"""The C-ABI library loads and exports every symbol include/*.h declares, and
its host-side scalar surface (crc32c.h) matches the reference's answers.
No GPU needed."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from memcached_amd import _lib
from memcached_amd import crc32c as mc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _declared():
    names = set()
    for h in ("crc32c.h", "crc32c_batch.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(crc32c\w*)\s*\(", src))
        names |= set(re.findall(r"extern\s+\w+\s+(crc32c\w*)\s*;", src))
    names -= {"crc32c_spans"}
    return names


def test_every_declared_symbol_is_exported():
    declared = _declared()
    assert "crc32c" in declared and "crc32c_batch" in declared
    for name in declared:
        ctypes.c_void_p.in_dll(_lib.lib, name) if name == "crc32c" else getattr(_lib.lib, name)
    assert declared <= set(_lib.EXPORTED)


def test_crc_func_is_a_data_symbol_set_by_init():
    ptr = ctypes.c_void_p.in_dll(_lib.lib, "crc32c")
    assert ptr.value  # _lib.load() ran crc32c_init()


def test_scalar_kats():
    for case in json.load(open(os.path.join(GOLD, "kat.json"))):
        data = bytes.fromhex(case["hex"])
        assert mc.crc32c(case["crc_in"], data) == case["expect"], case["name"]
        assert mc.crc32c_sw(case["crc_in"], data) == case["expect"], case["name"]


def test_scalar_all_lengths():
    g = np.load(os.path.join(GOLD, "spans.npz"))
    raw = g["buf"].tobytes()
    f = _lib.scalar_crc32c()
    buf = ctypes.create_string_buffer(raw, len(raw))
    base = ctypes.addressof(buf)
    for n in range(g["crc0"].shape[0]):
        for off in range(8):
            assert f(0, base + off, n) == g["crc0"][n, off]
            assert f(int(g["cin"][n, off]), base + off, n) == g["crcin"][n, off]


def test_sw_big_matches_the_reference_symbol():
    """crc32c_sw_big (crc32c.c:467-498) equals the reference's own exported
    function on this host (tests/golden/swbig.npz), at every length 0..300,
    five long lengths and every 8-byte alignment, with and without crc_in."""
    g = np.load(os.path.join(GOLD, "swbig.npz"))
    f = _lib.lib.crc32c_sw_big
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    raw = g["buf"].tobytes()
    buf = ctypes.create_string_buffer(raw, len(raw))
    base = ctypes.addressof(buf)
    assert base % 8 == 0  # as when the vectors were made (the word loop is address-aligned)
    for i, n in enumerate(g["lens"]):
        for off in range(8):
            assert f(0, base + off, int(n)) == g["crc0"][i, off], (int(n), off)
            assert f(int(g["cin"][i, off]), base + off, int(n)) == g["crcin"][i, off], (int(n), off)


def test_errors_are_named():
    assert _lib.lib.crc32c_strerror(_lib.CRC32C_ENODEV) == b"no gfx950 device"
    assert _lib.lib.crc32c_strerror(_lib.CRC32C_EINVAL) == b"invalid argument"


def test_batch_rejects_null_descriptor():
    assert _lib.lib.crc32c_batch(None, 0, None) == _lib.CRC32C_EINVAL


def test_no_gpu_means_enodev_not_a_cpu_fallback():
    """Every batch entry point fails loudly without a gfx950 device (CPU leg
    only: skipped where a GPU is visible)."""
    if _lib.lib.crc32c_gpu_count() > 0:
        pytest.skip("a gfx950 device is visible")
    buf = np.zeros(1 << 16, np.uint8)
    offs = np.zeros(4, np.uint64)
    lens = np.full(4, 100, np.uint32)
    out = np.zeros(4, np.uint32)
    s = _lib.Spans(buf.ctypes.data, buf.size, offs.ctypes.data, 0, lens.ctypes.data, 0, None, out.ctypes.data, 4)
    nbad, nitems = ctypes.c_uint64(0), ctypes.c_uint64(0)
    ok = np.zeros(4, np.uint8)
    first = np.array([0, 2, 4], np.uint64)
    calls = {
        "crc32c_batch": lambda: _lib.lib.crc32c_batch(ctypes.byref(s), 0, None),
        "crc32c_batch_multi": lambda: _lib.lib.crc32c_batch_multi(ctypes.byref(s), 1),
        "crc32c_verify_items": lambda: _lib.lib.crc32c_verify_items(buf.ctypes.data, buf.size, 0, offs.ctypes.data,
                                                                    4, ok.ctypes.data, ctypes.byref(nbad), 0, None),
        "crc32c_stamp_items": lambda: _lib.lib.crc32c_stamp_items(buf.ctypes.data, buf.size, 0, offs.ctypes.data,
                                                                  4, ok.ctypes.data, ctypes.byref(nbad), 0, None),
        "crc32c_verify_pages": lambda: _lib.lib.crc32c_verify_pages(buf.ctypes.data, buf.size, 1 << 12, None, None,
                                                                    0, ctypes.byref(nitems), ctypes.byref(nbad),
                                                                    0, None),
        "crc32c_batch_chains": lambda: _lib.lib.crc32c_batch_chains(ctypes.byref(s), first.ctypes.data, 2,
                                                                    out.ctypes.data, 0, None),
    }
    for name, call in calls.items():
        assert call() == _lib.CRC32C_ENODEV, name
    assert _lib.lib.crc32c_host_alloc(4096) is None
    assert (out == 0).all()  # nothing was computed on the CPU


def test_python_constants_match_the_header():
    """Every #define CRC32C_* of include/crc32c_batch.h has the same value in
    memcached_amd/_lib.py (the ctypes mirror the tests and bench use)."""
    import re
    hdr = open(os.path.join(ROOT, "include", "crc32c_batch.h")).read()
    defs = dict(re.findall(r"#define (CRC32C_\w+) \(?(-?(?:0x)?[0-9a-fA-F]+)u?\)?", hdr))
    assert len(defs) >= 11
    assert not hasattr(_lib, "CRC32C_ALIGNED16")  # retired: no kernel read it
    for name, val in defs.items():
        assert getattr(_lib, name) == int(val, 0), name


def test_batch_accepts_the_retired_aligned16_keyword():
    """batch(aligned16=...) still parses (a DeprecationWarning, no effect):
    with a GPU the CRCs are the oracle's, without one the call fails with
    ENODEV, not a TypeError."""
    from tests import oracle
    buf = np.random.default_rng(3).integers(0, 256, 1 << 14, dtype=np.uint8)
    offs = np.array([0, 16, 4096], np.uint64)
    lens = np.array([100, 4096, 33], np.uint32)
    with pytest.warns(DeprecationWarning):
        try:
            got = mc.batch(buf, offsets=offs, lens=lens, aligned16=True)
        except _lib.Crc32cError as e:
            assert e.rc == _lib.CRC32C_ENODEV and _lib.lib.crc32c_gpu_count() == 0
            return
    np.testing.assert_array_equal(got, oracle.batch(buf, offs, lens))
