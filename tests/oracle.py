"""ctypes binding of the CPU oracle (oracle/liboracle.so) for the tests.

Test infrastructure only: the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        L = ctypes.CDLL(path)
        for name in ("oracle_crc32c", "oracle_crc32c_bitwise"):
            f = getattr(L, name)
            f.restype = ctypes.c_uint32
            f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_shift_zeros.restype = ctypes.c_uint32
        L.oracle_shift_zeros.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_crc32c_combine.restype = ctypes.c_uint32
        L.oracle_crc32c_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_crc32c_batch.restype = None
        L.oracle_crc32c_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_uint64]
        L.oracle_item_crc.restype = ctypes.c_uint32
        L.oracle_item_crc.argtypes = [ctypes.c_void_p]
        L.oracle_item_crc_cfl.restype = ctypes.c_uint32
        L.oracle_item_crc_cfl.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_item_ntotal_cfl.restype = ctypes.c_uint32
        L.oracle_item_ntotal_cfl.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_verify_span.restype = ctypes.c_uint64
        L.oracle_verify_span.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64]
        L.oracle_verify_span_cfl.restype = ctypes.c_uint64
        L.oracle_verify_span_cfl.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_uint32]
        _lib = L
    return _lib


def _arr(data):
    if isinstance(data, (bytes, bytearray)):
        return np.frombuffer(bytes(data), np.uint8)
    return np.ascontiguousarray(data).view(np.uint8).reshape(-1)


def crc32c(crc: int, data) -> int:
    a = _arr(data)
    return int(lib().oracle_crc32c(crc & 0xFFFFFFFF, a.ctypes.data, a.size))


def crc32c_bitwise(crc: int, data) -> int:
    a = _arr(data)
    return int(lib().oracle_crc32c_bitwise(crc & 0xFFFFFFFF, a.ctypes.data, a.size))


def batch(buf, offsets, lens, crc_in=None):
    buf = _arr(buf)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint64)
    out = np.empty(offsets.size, np.uint32)
    cin = None if crc_in is None else np.ascontiguousarray(crc_in, np.uint32)
    lib().oracle_crc32c_batch(buf.ctypes.data, offsets.ctypes.data, lens.ctypes.data,
                              None if cin is None else cin.ctypes.data, out.ctypes.data, offsets.size)
    return out


def verify_span(buf, max_items=1 << 20, cflags_bytes=4):
    buf = _arr(buf)
    offs = np.empty(max_items, np.uint64)
    ok = np.empty(max_items, np.uint8)
    n = lib().oracle_verify_span_cfl(buf.ctypes.data, buf.size, offs.ctypes.data, ok.ctypes.data, max_items,
                                     cflags_bytes)
    return offs[:n], ok[:n]


def item_crc(buf, off, cflags_bytes=4):
    """Spill CRC (storage.c:567) of the image at buf[off:]."""
    buf = _arr(buf)
    return int(lib().oracle_item_crc_cfl(buf.ctypes.data + int(off), cflags_bytes))
