"""CPU restatement of K5 k_items (crc32c_kernels.hip): one pass per one-block
item image, the per-image work done by one lane per epoch.

Checked against the oracle for every alignment and every fused length:
* the fused shape (fused_vlen): one 4 KiB block [Ea - 4096, Ea) after a head
  fragment [p, G) of 4..128 bytes, G = Ea - 4096;
* the lane's fragment chain: the 16-B pieces of [floor16(p), G) as dwords,
  bytes below p cleared and ~0 XORed into [p, p + 4) (head_dword), folded
  dword by dword -- equal to the register from ~0 over [p, G);
* the block with its t foreign tail bytes cleared: R = raw of it;
* R ^ C with C = M_4096(r) is M_t(f), f the register after the whole span from
  ~0 (crc32c(0, D) = ~f); a verify adds M_t(~stored) to C, so R ^ C == 0 iff
  the stored CRC matches; the stamp's last step (k_fix) is ~M_{-t}(R ^ C);
* the header decode from five window dwords (alignbyte) against the layout.
"""
import struct

import numpy as np
import pytest

from memcached_amd import layout
from tests import oracle
from tests.span_model import M32, mulmodp, tail_pad, xpow8_inv

FRAG = 128
BLOCK = 4096


def reg(r, data):
    """The register after data from register r (crc32c without the final ~)."""
    return ~oracle.crc32c(~r & M32, bytes(data)) & M32


def raw(data):
    return reg(0, data)


def zeros(v, n):
    return oracle.lib().oracle_shift_zeros(v & M32, n)


def fused_vlen(vlen):
    return BLOCK + 4 <= vlen <= BLOCK + FRAG


def head_dword(v, pa):
    c, e = min(max(pa, 0), 4), min(max(pa + 4, 0), 4)
    keep = 0 if c >= 4 else (M32 << (8 * c)) & M32
    inj = M32 if e >= 4 else (1 << (8 * e)) - 1
    return (v & keep) ^ (inj & keep)


def step4(x, d):
    """step4_next: x advanced over four zero bytes, then d XORed in -- the
    dword-by-dword slice-by-4 fold (raw(A || B) = M_4(raw(A)) ^ raw(B) for a
    dword B is M_4(raw(A)) ^ step4(0, B) ... written as the kernel does)."""
    return zeros(x, 4) ^ d


def lane_fragment(buf, p, G):
    """The lane's chain of k_items' prep over [floor16(p), G)."""
    kh = p & 15
    ph = p - kh
    assert (G - ph) % 16 == 0
    np16 = (G - ph) // 16
    x = 0
    for k in range(np16):
        for j in range(4):
            A = ph + 16 * k + 4 * j
            v = int.from_bytes(bytes(buf[A:A + 4]), "little")
            d = head_dword(v, kh - (16 * k + 4 * j))
            x = d if (k == 0 and j == 0) else step4(x, d)
    # x is the dword stream folded without its last four-byte advance; the
    # kernel's final step4_next(x, 0) gives raw of the dwords
    return step4(x, 0) if np16 else 0


def kernel_items(buf, p, length, stored=None):
    """(R ^ C, t) as k_items computes it for span [p, p + length)."""
    t = tail_pad(p, length)
    vlen = length + t
    assert fused_vlen(vlen)
    G = p + vlen - BLOCK
    r = lane_fragment(buf, p, G)
    # the fragment chain is the register from ~0 over [p, G)
    assert r == reg(M32, buf[p:G])
    C = zeros(r, BLOCK)
    if stored is not None:
        C ^= zeros(~stored & M32, t)
    block = bytearray(buf[G:G + BLOCK])
    E = p + length
    for i in range(E - G, BLOCK):
        block[i] = 0  # the tail mask of lane 31's last piece
    return raw(block) ^ C, t


@pytest.mark.parametrize("kh", range(16))
def test_fused_R_xor_C_is_Mt_of_the_register(kh):
    rng = np.random.default_rng(kh)
    buf = rng.integers(0, 256, 3 * BLOCK, dtype=np.uint8).tobytes()
    for length in list(range(BLOCK + 1 - 15, BLOCK + 16)) + list(range(BLOCK + 100, BLOCK + FRAG + 1)) + [4133]:
        p = 160 + kh
        t = tail_pad(p, length)
        if not fused_vlen(length + t):
            continue
        D = buf[p:p + length]
        crc = oracle.crc32c(0, D)
        f = reg(M32, D)  # register after D from ~0: crc32c(0, D) = ~f
        assert crc == ~f & M32
        RC, t2 = kernel_items(buf, p, length)
        assert RC == zeros(f, t) and t2 == t
        # the stamp (k_fix): ~M_{-t}(R ^ C)
        assert ~mulmodp(RC, xpow8_inv(t)) & M32 == crc
        # verify: zero iff the stored CRC matches
        assert kernel_items(buf, p, length, stored=crc)[0] == 0
        assert kernel_items(buf, p, length, stored=crc ^ 1)[0] != 0


def test_fused_shapes_of_the_configs():
    """Every alignment of a 4133-B span (config 5's images) is fused; a
    fragment under 4 bytes is not, nor one past 128 bytes."""
    for kh in range(16):
        assert fused_vlen(4133 + tail_pad(kh, 4133))
    assert all(fused_vlen(L + tail_pad(kh, L)) for L in range(4100, 4210) for kh in range(16))
    assert not any(fused_vlen(L + tail_pad(kh, L)) for L in range(4080, 4097) for kh in range(16)
                   if L + tail_pad(kh, L) < BLOCK + 4)
    assert not any(fused_vlen(L + tail_pad(kh, L)) for L in range(4225, 4300) for kh in range(16))


def test_header_window_decode():
    """Five dwords of the 16-B aligned window at floor16(off + 28), lane i
    holding dword (sh >> 2) + i, give exptime, nbytes, it_flags and nkey by
    alignbyte -- for every alignment of the image."""
    rng = np.random.default_rng(9)
    for off in range(64, 64 + 16):
        img = layout.make_item(b"key0000042", rng.integers(0, 256, 300, dtype=np.uint8).tobytes(), cas=7,
                               client_flags=5)
        buf = bytearray(off) + img + bytearray(64)
        struct.pack_into("<I", buf, off + 28, 0xDEADBEEF)
        q = off + 28
        sh = q & 15
        q0 = q - sh
        w = [int.from_bytes(bytes(buf[q0 + 4 * ((sh >> 2) + i):q0 + 4 * ((sh >> 2) + i) + 4]), "little")
             for i in range(5)]
        assert q0 + 4 * ((sh >> 2) + 5) <= ((off + 48 + 15) // 16) * 16

        def alignbyte(hi, lo, b):
            return ((hi << 32 | lo) >> (8 * b)) & M32

        b = sh & 3
        assert alignbyte(w[1], w[0], b) == 0xDEADBEEF
        assert alignbyte(w[2], w[1], b) == struct.unpack_from("<I", buf, off + 32)[0]
        assert alignbyte(w[3], w[2], b) >> 16 == struct.unpack_from("<H", buf, off + 38)[0]
        assert (alignbyte(w[4], w[3], b) >> 8) & 0xFF == buf[off + 41]
