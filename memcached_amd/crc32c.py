"""Python face of the drop-in library, mirroring the reference interface.

Scalar calls follow crc32c.h (reference crc32c.h:15-21): ``crc32c(crc, buf)``
continues a CRC-32C over ``buf`` (first call with crc = 0, chaining allowed)
and ``crc32c_sw`` is the table-driven variant.  Batch calls wrap
include/crc32c_batch.h and run the gfx950 kernels:

* ``batch``        out[i] = crc32c(crc_in[i] or 0, span i)  (storage.c:567, :172)
* ``verify_items`` stored-CRC check of packed item images (storage.c:160-178)
* ``stamp_items``  spill CRC written into each image's exptime (storage.c:567)
* ``verify_pages`` walk + verify whole pages on the device (storage.c:950-1070)
* ``batch_chains`` chained CRCs of chunked items over iov lists (storage.c:163-170)
* ``batch_multi``  host batch split across GPUs by bytes

Host inputs are numpy arrays (or bytes); device inputs are torch tensors on a
HIP device, enqueued on torch's current stream.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import CRC32C_ASYNC, CRC32C_CFLAGS64, CRC32C_DEVICE, Crc32cError, check, lib

__all__ = ["crc32c", "crc32c_sw", "batch", "verify_items", "stamp_items", "verify_pages", "batch_chains", "batch_multi",
           "shard_cuts", "queue_stats", "set_small_max", "gpu_count", "Crc32cError"]


def _host_buf(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(data, dtype=np.uint8)
    else:
        arr = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return arr


def crc32c(crc: int, data) -> int:
    """crc32c(crc, buf, len) through the `crc32c` function-pointer symbol."""
    arr = _host_buf(data)
    return int(_lib.scalar_crc32c()(crc & 0xFFFFFFFF, arr.ctypes.data, arr.size))


def crc32c_sw(crc: int, data) -> int:
    arr = _host_buf(data)
    return int(lib.crc32c_sw(crc & 0xFFFFFFFF, arr.ctypes.data, arr.size))


def gpu_count() -> int:
    return int(lib.crc32c_gpu_count())


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _ptr(x):
    if x is None:
        return None
    if _is_torch(x):
        return x.data_ptr()
    return x.ctypes.data


def _check_dev(t, name, n, dtypes):
    """A device descriptor array: contiguous, on the device, one of `dtypes`
    (names), at least n elements (the kernels read n of them unchecked)."""
    import torch
    if not (_is_torch(t) and t.is_cuda and t.is_contiguous()):
        raise ValueError(f"{name}: device batches need a contiguous device tensor")
    if str(t.dtype).replace("torch.", "") not in dtypes:
        raise TypeError(f"{name}: dtype {t.dtype} (need one of {', '.join(dtypes)})")
    if t.numel() < n:
        raise ValueError(f"{name}: {t.numel()} elements for {n} spans")
    return torch


def batch(buf, offsets=None, stride: int = 0, lens=None, length: int = 0, crc_in=None, out=None,
          stream=None, asynchronous: bool = False, aligned16=None):
    """Batched CRC-32C of spans of ``buf``.

    Span i = buf[off_i : off_i + len_i] with off_i = offsets[i] (or i*stride)
    and len_i = lens[i] (or ``length``).  Host numpy inputs take the pinned
    staging path; torch device tensors run in place on the current stream.
    Returns ``out`` (uint32, one CRC per span).  ``aligned16`` is accepted and
    ignored, as the C ABI ignores its retired flag bit 0x4 (the kernels test
    alignment themselves).
    """
    if aligned16 is not None:
        import warnings
        warnings.warn("batch(aligned16=...) is ignored (alignment is detected per batch)", DeprecationWarning,
                      stacklevel=2)
    dev = _is_torch(buf) and buf.is_cuda
    if offsets is not None:
        n = len(offsets)
    elif lens is not None:
        n = len(lens)
    else:
        raise ValueError("need offsets or lens to know the batch size")
    if dev:
        import torch
        if not buf.is_contiguous():
            raise ValueError("buf: device batches need a contiguous device tensor")
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=buf.device)
        _check_dev(out, "out", n, ("int32", "uint32"))
        if offsets is not None:
            _check_dev(offsets, "offsets", n, ("int64", "uint64"))
        for name, t in (("lens", lens), ("crc_in", crc_in)):
            if t is not None:
                _check_dev(t, name, n, ("int32", "uint32"))
        base_bytes = buf.numel() * buf.element_size()
        if stream is None:
            stream = torch.cuda.current_stream(buf.device).cuda_stream
    else:
        buf = _host_buf(buf)
        base_bytes = buf.size
        offsets = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint32)
        crc_in = None if crc_in is None else np.ascontiguousarray(crc_in, dtype=np.uint32)
        if out is None:
            out = np.empty(n, dtype=np.uint32)
        for name, a in (("lens", lens), ("crc_in", crc_in), ("out", out)):
            if a is not None and a.size < n:
                raise ValueError(f"{name}: {a.size} elements for {n} spans")
        if out.dtype not in (np.uint32, np.int32) or not out.flags.c_contiguous:
            raise TypeError("out: need a contiguous uint32 array")
    s = _lib.Spans(_ptr(buf), base_bytes, _ptr(offsets), stride, _ptr(lens), length, _ptr(crc_in),
                   _ptr(out), n)
    flags = CRC32C_DEVICE if dev else 0
    if dev and asynchronous:
        flags |= CRC32C_ASYNC
    check(lib.crc32c_batch(ctypes.byref(s), flags, stream if dev else None), "crc32c_batch")
    return out


def batch_multi(buf, offsets=None, stride: int = 0, lens=None, length: int = 0, crc_in=None, ngpus: int = 0):
    """Host batch split across ``ngpus`` devices (0 = all) by bytes."""
    buf = _host_buf(buf)
    offsets = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint32)
    crc_in = None if crc_in is None else np.ascontiguousarray(crc_in, dtype=np.uint32)
    n = len(offsets) if offsets is not None else len(lens)
    out = np.empty(n, dtype=np.uint32)
    s = _lib.Spans(_ptr(buf), buf.size, _ptr(offsets), stride, _ptr(lens), length, _ptr(crc_in),
                   _ptr(out), n)
    check(lib.crc32c_batch_multi(ctypes.byref(s), ngpus), "crc32c_batch_multi")
    return out


def verify_items(buf, item_offsets, region_bytes=0, stream=None, cflags64=False):
    """Verify packed item images; returns (ok uint8 array / tensor, nbad).

    ``region_bytes``: the write-buffer size; an item whose header claims a
    span crossing a multiple of it is reported bad without being read
    (extstore never splits an item across wbufs).  0 = no such bound.
    ``cflags64``: images of a LARGE_CLIENT_FLAGS build (8-byte client flags)."""
    dev = _is_torch(buf) and buf.is_cuda
    nbad = ctypes.c_uint64(0)
    fl = CRC32C_CFLAGS64 if cflags64 else 0
    if dev:
        import torch
        n = item_offsets.numel()
        _check_dev(item_offsets, "item_offsets", n, ("int64", "uint64"))
        ok = torch.empty(n, dtype=torch.uint8, device=buf.device)
        if stream is None:
            stream = torch.cuda.current_stream(buf.device).cuda_stream
        rc = lib.crc32c_verify_items(buf.data_ptr(), buf.numel() * buf.element_size(), region_bytes,
                                     item_offsets.data_ptr(), n, ok.data_ptr(), ctypes.byref(nbad),
                                     CRC32C_DEVICE | fl, stream)
    else:
        buf = _host_buf(buf)
        offs = np.ascontiguousarray(item_offsets, dtype=np.uint64)
        ok = np.empty(offs.size, dtype=np.uint8)
        rc = lib.crc32c_verify_items(buf.ctypes.data, buf.size, region_bytes, offs.ctypes.data, offs.size,
                                     ok.ctypes.data, ctypes.byref(nbad), fl, None)
    check(rc, "crc32c_verify_items")
    return ok, int(nbad.value)


def stamp_items(buf, item_offsets, region_bytes=0, stream=None, cflags64=False):
    """Write the spill CRC of every item image into its exptime field, in place
    (storage.c:567 for a whole wbuf at once).  Returns (ok, nbad): ok marks
    stamped images, nbad counts malformed ones (left untouched)."""
    dev = _is_torch(buf) and buf.is_cuda
    nbad = ctypes.c_uint64(0)
    fl = CRC32C_CFLAGS64 if cflags64 else 0
    if dev:
        import torch
        n = item_offsets.numel()
        _check_dev(item_offsets, "item_offsets", n, ("int64", "uint64"))
        ok = torch.empty(n, dtype=torch.uint8, device=buf.device)
        if stream is None:
            stream = torch.cuda.current_stream(buf.device).cuda_stream
        rc = lib.crc32c_stamp_items(buf.data_ptr(), buf.numel() * buf.element_size(), region_bytes,
                                    item_offsets.data_ptr(), n, ok.data_ptr(), ctypes.byref(nbad),
                                    CRC32C_DEVICE | fl, stream)
    else:
        if not (isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.flags.writeable
                and buf.flags.c_contiguous):
            raise TypeError("stamp_items needs a writable contiguous uint8 numpy array (stamped in place)")
        offs = np.ascontiguousarray(item_offsets, dtype=np.uint64)
        ok = np.empty(offs.size, dtype=np.uint8)
        rc = lib.crc32c_stamp_items(buf.ctypes.data, buf.size, region_bytes, offs.ctypes.data, offs.size,
                                    ok.ctypes.data, ctypes.byref(nbad), fl, None)
    check(rc, "crc32c_stamp_items")
    return ok, int(nbad.value)


def verify_pages(buf, wbuf_bytes, stream=None, cflags64=False):
    """Walk every wbuf-sized read of ``buf`` on the device and verify each
    item found.  Returns (item offsets, ok flags, nbad) in walk order.

    One library call when the items fit a first guess of the capacity
    (images of >= 1 KiB on average); otherwise a second call with the exact
    count the first one reported."""
    dev = _is_torch(buf) and buf.is_cuda
    nitems, nbad = ctypes.c_uint64(0), ctypes.c_uint64(0)
    fl = CRC32C_CFLAGS64 if cflags64 else 0
    if dev:
        import torch
        if not buf.is_contiguous():
            raise ValueError("buf: need a contiguous device tensor")
        if stream is None:
            stream = torch.cuda.current_stream(buf.device).cuda_stream
        nbytes = buf.numel() * buf.element_size()
        nw = -(-nbytes // wbuf_bytes)
        cap = min(nbytes // 1024 + nw, nbytes // 50 + nw)
        while True:
            offs = torch.empty(cap, dtype=torch.int64, device=buf.device)
            ok = torch.empty(cap, dtype=torch.uint8, device=buf.device)
            check(lib.crc32c_verify_pages(buf.data_ptr(), nbytes, wbuf_bytes, offs.data_ptr(), ok.data_ptr(), cap,
                                          ctypes.byref(nitems), ctypes.byref(nbad), CRC32C_DEVICE | fl, stream),
                  "crc32c_verify_pages")
            n = nitems.value
            if n <= cap:
                return offs[:n], ok[:n], int(nbad.value)
            cap = n
    buf = _host_buf(buf)
    # an image is >= 50 bytes and each wbuf's last counted image may run past its end
    cap = buf.size // 50 + -(-buf.size // wbuf_bytes)
    offs = np.empty(cap, np.uint64)
    ok = np.empty(cap, np.uint8)
    check(lib.crc32c_verify_pages(buf.ctypes.data, buf.size, wbuf_bytes, offs.ctypes.data, ok.ctypes.data, cap,
                                  ctypes.byref(nitems), ctypes.byref(nbad), fl, None), "crc32c_verify_pages")
    n = nitems.value
    assert n <= cap, "item count above the proven bound"
    return offs[:n], ok[:n], int(nbad.value)


def batch_chains(buf, offsets, lens, chain_first, stream=None):
    """Chained CRC per iov list: chain c covers iovs [chain_first[c],
    chain_first[c+1]) of the spans (offsets[i], lens[i]) of ``buf`` and gets
    crc32c(...crc32c(crc32c(0, iov_a), iov_a+1)..., iov_b-1)."""
    dev = _is_torch(buf) and buf.is_cuda
    n, nchains = len(offsets), len(chain_first) - 1
    if dev:
        import torch
        if not buf.is_contiguous():
            raise ValueError("buf: need a contiguous device tensor")
        _check_dev(offsets, "offsets", n, ("int64", "uint64"))
        _check_dev(lens, "lens", n, ("int32", "uint32"))
        _check_dev(chain_first, "chain_first", nchains + 1, ("int64", "uint64"))
        iov_out = torch.empty(n, dtype=torch.int32, device=buf.device)
        out = torch.empty(nchains, dtype=torch.int32, device=buf.device)
        if stream is None:
            stream = torch.cuda.current_stream(buf.device).cuda_stream
        base_bytes = buf.numel() * buf.element_size()
    else:
        buf = _host_buf(buf)
        base_bytes = buf.size
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        chain_first = np.ascontiguousarray(chain_first, dtype=np.uint64)
        iov_out = np.empty(n, dtype=np.uint32)
        out = np.empty(nchains, dtype=np.uint32)
    s = _lib.Spans(_ptr(buf), base_bytes, _ptr(offsets), 0, _ptr(lens), 0, None, _ptr(iov_out), n)
    check(lib.crc32c_batch_chains(ctypes.byref(s), _ptr(chain_first), nchains, _ptr(out),
                                  CRC32C_DEVICE if dev else 0, stream if dev else None), "crc32c_batch_chains")
    return out


def shard_cuts(lens, parts: int):
    """crc32c_shard_cuts: the parts + 1 cut points of the byte-balanced split
    crc32c_batch_multi uses over spans of lengths ``lens`` (uint32)."""
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    cuts = np.empty(parts + 1, dtype=np.uint64)
    check(lib.crc32c_shard_cuts(lens.ctypes.data, 0, lens.size, parts, cuts.ctypes.data), "crc32c_shard_cuts")
    return cuts.astype(np.int64)


def queue_stats():
    """(launches, spans, jobs, solo_jobs) of the current device's coalescing queue."""
    v = [ctypes.c_uint64(0) for _ in range(4)]
    check(lib.crc32c_queue_stats(*[ctypes.byref(x) for x in v]), "crc32c_queue_stats")
    return tuple(int(x.value) for x in v)


def set_small_max(n: int) -> int:
    """Batches of at most n spans take the single-launch kernel (0: none); returns the previous value."""
    return int(lib.crc32c_set_small_max(n))
