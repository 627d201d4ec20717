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


def test_errors_are_named():
    assert _lib.lib.crc32c_strerror(_lib.CRC32C_ENODEV) == b"no gfx950 device"
    assert _lib.lib.crc32c_strerror(_lib.CRC32C_EINVAL) == b"invalid argument"


def test_batch_rejects_null_descriptor():
    assert _lib.lib.crc32c_batch(None, 0, None) == _lib.CRC32C_EINVAL
