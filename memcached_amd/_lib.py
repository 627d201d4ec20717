"""ctypes binding of libmcrc32c.so (include/crc32c.h + include/crc32c_batch.h).

The library is the product; this module only marshals arguments.  There is no
Python or CPU fallback for the batch entry points: if the library is missing,
importing this module raises, and a batch call without a gfx950 device raises
Crc32cError(CRC32C_ENODEV).
"""
from __future__ import annotations

import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# MCRC_LIB selects another build of the same library (A/B of two builds in one run)
LIB_PATH = os.environ.get("MCRC_LIB") or os.path.join(PKG, "libmcrc32c.so")

CRC32C_OK = 0
CRC32C_ENODEV = -1
CRC32C_EHIP = -2
CRC32C_EINVAL = -3
CRC32C_ENOMEM = -4
CRC32C_ERANGE = -5
CRC32C_EWALK = -6

CRC32C_DEVICE = 0x1
CRC32C_ASYNC = 0x2
CRC32C_CFLAGS64 = 0x8
CRC32C_MAX_SPAN = 0x7FFF0000  # longest span (include/crc32c_batch.h)

# every symbol include/*.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "crc32c", "crc32c_init", "crc32c_sw", "crc32c_sw_little", "crc32c_sw_big",
    "crc32c_gpu_count", "crc32c_batch", "crc32c_batch_multi", "crc32c_verify_items", "crc32c_stamp_items",
    "crc32c_verify_pages", "crc32c_batch_chains", "crc32c_host_alloc", "crc32c_host_free",
    "crc32c_batch_submit", "crc32c_batch_wait", "crc32c_strerror", "crc32c_last_kernel_ms",
    "crc32c_shard_cuts", "crc32c_queue_stats", "crc32c_host_register", "crc32c_host_unregister",
    "crc32c_set_small_max",
)


class Crc32cError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        msg = lib.crc32c_strerror(rc).decode() if lib is not None else str(rc)
        super().__init__(f"{what}: {msg} ({rc})" if what else f"{msg} ({rc})")
        self.rc = rc


class Spans(ctypes.Structure):
    _fields_ = [
        ("base", ctypes.c_void_p),
        ("base_bytes", ctypes.c_uint64),
        ("offsets", ctypes.c_void_p),
        ("stride", ctypes.c_uint64),
        ("lens", ctypes.c_void_p),
        ("len", ctypes.c_uint32),
        ("crc_in", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("n", ctypes.c_uint64),
    ]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -m memcached_amd.build`")
    # the HIP runtime already loaded by torch (same soname) is reused when present
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    lib.crc32c_init.restype = None
    lib.crc32c_init.argtypes = []
    for name in ("crc32c_sw", "crc32c_sw_little"):
        f = getattr(lib, name)
        f.restype = ctypes.c_uint32
        f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    lib.crc32c_gpu_count.restype = ctypes.c_int
    lib.crc32c_batch.restype = ctypes.c_int
    lib.crc32c_batch.argtypes = [ctypes.POINTER(Spans), ctypes.c_uint, ctypes.c_void_p]
    lib.crc32c_batch_multi.restype = ctypes.c_int
    lib.crc32c_batch_multi.argtypes = [ctypes.POINTER(Spans), ctypes.c_int]
    lib.crc32c_verify_items.restype = ctypes.c_int
    lib.crc32c_verify_items.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint,
                                        ctypes.c_void_p]
    lib.crc32c_stamp_items.restype = ctypes.c_int
    lib.crc32c_stamp_items.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.c_uint, ctypes.c_void_p]
    lib.crc32c_verify_pages.restype = ctypes.c_int
    lib.crc32c_verify_pages.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint, ctypes.c_void_p]
    lib.crc32c_batch_chains.restype = ctypes.c_int
    lib.crc32c_batch_chains.argtypes = [ctypes.POINTER(Spans), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_uint, ctypes.c_void_p]
    lib.crc32c_host_alloc.restype = ctypes.c_void_p
    lib.crc32c_host_alloc.argtypes = [ctypes.c_size_t]
    lib.crc32c_host_free.restype = None
    lib.crc32c_host_free.argtypes = [ctypes.c_void_p]
    lib.crc32c_batch_submit.restype = ctypes.c_int
    lib.crc32c_batch_submit.argtypes = [ctypes.POINTER(Spans), ctypes.c_uint, ctypes.POINTER(ctypes.c_void_p)]
    lib.crc32c_batch_wait.restype = ctypes.c_int
    lib.crc32c_batch_wait.argtypes = [ctypes.c_void_p]
    lib.crc32c_strerror.restype = ctypes.c_char_p
    lib.crc32c_strerror.argtypes = [ctypes.c_int]
    lib.crc32c_last_kernel_ms.restype = ctypes.c_float
    lib.crc32c_shard_cuts.restype = ctypes.c_int
    lib.crc32c_shard_cuts.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                      ctypes.c_void_p]
    lib.crc32c_queue_stats.restype = ctypes.c_int
    lib.crc32c_queue_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
    lib.crc32c_host_register.restype = ctypes.c_int
    lib.crc32c_host_register.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.crc32c_host_unregister.restype = ctypes.c_int
    lib.crc32c_host_unregister.argtypes = [ctypes.c_void_p]
    lib.crc32c_set_small_max.restype = ctypes.c_uint64
    lib.crc32c_set_small_max.argtypes = [ctypes.c_uint64]
    lib.crc32c_init()
    return lib


lib = _load()

# the crc_func data symbol: a function pointer the callers invoke directly
CRC_FUNC = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t)
_crc_ptr = ctypes.c_void_p.in_dll(lib, "crc32c")


def scalar_crc32c():
    """The function currently stored in the `crc32c` data symbol."""
    if not _crc_ptr.value:
        raise RuntimeError("crc32c_init() has not run")
    return CRC_FUNC(_crc_ptr.value)


def check(rc: int, what: str = "") -> None:
    if rc != CRC32C_OK:
        raise Crc32cError(rc, what)
