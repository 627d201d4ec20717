"""Host-side mirror of the memcached item byte layout the CRC path covers.

Only the geometry that decides which bytes are checksummed is restated here
(reference /root/reference):

* ``struct _stritem`` (memcached.h:613-636): 48-byte header on LP64 --
  next/prev/h_next pointers (0..23), time (24), exptime (28), nbytes (32),
  refcount (36), it_flags (38), slabs_clsid (40), nkey (41), 6 pad bytes,
  then CAS (8 bytes, when ITEM_CAS), key + NUL, client flags (when
  ITEM_CFLAGS: sizeof(client_flags_t), 4 bytes, or 8 in a build with
  --enable-large-client-flags, memcached.h:96-100) and the value with its
  trailing ``\\r\\n``.
* ``ITEM_ntotal`` (memcached.h:149-152).
* ``STORE_OFFSET = offsetof(item, nbytes) = 32`` (storage.h:43): the spill CRC
  covers ``[32, ntotal)`` and is stored in ``exptime`` (storage.c:567), and the
  read-back verify recomputes it over the same span (storage.c:160-178).
* Write buffers pack item images back to back; an item never straddles a wbuf
  and the unused tail is zero-filled before flush (extstore.c:559-570,
  :652-670); a page is ``page_size / wbuf_size`` wbufs (64 MiB / 4 MiB).
"""
from __future__ import annotations

import struct

import numpy as np

ITEM_HDR = 48
STORE_OFFSET = 32
EXPTIME_OFF = 28
NBYTES_OFF = 32
FLAGS_OFF = 38
NKEY_OFF = 41
ITEM_CAS = 2
ITEM_CFLAGS = 256
WBUF_SIZE = 4 * 1024 * 1024
PAGE_SIZE = 64 * 1024 * 1024


def item_ntotal(nkey: int, nbytes: int, cas: bool, cflags: bool, cflags_bytes: int = 4) -> int:
    """ITEM_ntotal for a key of ``nkey`` bytes and ``nbytes`` of value+CRLF
    (``cflags_bytes`` = sizeof(client_flags_t): 4, or 8 with large client flags)."""
    return ITEM_HDR + nkey + 1 + nbytes + (cflags_bytes if cflags else 0) + (8 if cas else 0)


def make_item(key: bytes, value: bytes, cas: int | None = 1, client_flags: int = 0,
              time_hash: int = 0, cflags_bytes: int = 4) -> bytearray:
    """One item image as storage.c copies it into a wbuf (CRC field zeroed)."""
    data = value + b"\r\n"
    flags = (ITEM_CAS if cas is not None else 0) | (ITEM_CFLAGS if client_flags else 0)
    n = item_ntotal(len(key), len(data), cas is not None, bool(client_flags), cflags_bytes)
    img = bytearray(n)
    struct.pack_into("<IIiHHBB", img, 24, time_hash & 0xFFFFFFFF, 0, len(data), 1, flags, 1,
                     len(key))
    pos = ITEM_HDR
    if cas is not None:
        struct.pack_into("<Q", img, pos, cas)
        pos += 8
    img[pos:pos + len(key)] = key
    pos += len(key) + 1
    if client_flags:
        struct.pack_into("<Q" if cflags_bytes == 8 else "<I", img, pos, client_flags)
        pos += cflags_bytes
    img[pos:pos + len(data)] = data
    assert pos + len(data) == n
    return img


def ntotal_of(buf, off: int, cflags_bytes: int = 4) -> int:
    """ITEM_ntotal read back from an image at ``off`` (storage.c:960)."""
    nbytes, = struct.unpack_from("<i", buf, off + NBYTES_OFF)
    flags, = struct.unpack_from("<H", buf, off + FLAGS_OFF)
    return item_ntotal(int(buf[off + NKEY_OFF]), nbytes, bool(flags & ITEM_CAS), bool(flags & ITEM_CFLAGS),
                       cflags_bytes)


def pack_wbufs(items, wbuf_size: int = WBUF_SIZE):
    """Pack item images back to back into wbufs of ``wbuf_size`` bytes.

    Returns (buffer as np.uint8 array, item offsets as np.uint64).  A new wbuf
    starts when the next item does not fit; tails are zero (extstore.c:568).
    """
    chunks, offsets = [], []
    cur, used, base = bytearray(wbuf_size), 0, 0
    for img in items:
        if len(img) > wbuf_size:
            raise ValueError("item larger than a wbuf")
        if used + len(img) > wbuf_size:
            chunks.append(cur)
            base += wbuf_size
            cur, used = bytearray(wbuf_size), 0
        cur[used:used + len(img)] = img
        offsets.append(base + used)
        used += len(img)
    chunks.append(cur)
    return np.frombuffer(b"".join(chunks), dtype=np.uint8).copy(), np.asarray(offsets, np.uint64)


def spans_of(buf, offsets, cflags_bytes: int = 4):
    """(span offsets, span lengths) of the CRC span of every item."""
    offs = np.asarray(offsets, np.uint64)
    lens = np.array([ntotal_of(buf, int(o), cflags_bytes) - STORE_OFFSET for o in offs], np.uint64)
    return offs + STORE_OFFSET, lens


def store_crcs(buf: np.ndarray, offsets, crcs) -> None:
    """Write each item's CRC into its exptime field (storage.c:567)."""
    view = buf.view(np.uint8)
    for o, c in zip(np.asarray(offsets, np.uint64), np.asarray(crcs, np.uint32)):
        view[int(o) + EXPTIME_OFF:int(o) + EXPTIME_OFF + 4] = np.frombuffer(
            struct.pack("<I", int(c)), np.uint8)
