"""CPU restatement of K5 k_items (crc32c_kernels.hip): one pass per one-block
item image, the per-image work done by one lane per epoch.

Checked against the oracle for every alignment and every fused length:
* the fused shape (fused_vlen): one 4 KiB block [Ea - 4096, Ea) after a head
  fragment [p, G) of 4..128 bytes, G = Ea - 4096;
* the lane's fragment chain: the 16-B pieces of [floor16(p), G) as dwords,
  bytes below p cleared and ~c XORed into [p, p + 4) (head_dword; c = 0 for
  item images, the span's initial CRC for MODE 0), folded dword by dword --
  equal to the register from ~c over [p, G);
* the block with its t foreign tail bytes cleared: R = raw of it;
* R ^ C with C = M_4096(r) is M_t(f), f the register after the whole span from
  ~0 (crc32c(0, D) = ~f); a verify adds M_t(~stored) to C, so R ^ C == 0 iff
  the stored CRC matches; the last step of a stamp or a MODE 0 span (k_fix)
  is ~M_{-t}(R ^ C).
"""
import numpy as np
import pytest

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


def head_dword(v, pa, inj=M32):
    """Bytes below p cleared, the bytes of inj (~c) XORed into [p, p + 4)."""
    if pa >= 4:
        return 0
    if pa >= 0:
        return ((v & ((M32 << (8 * pa)) & M32)) ^ (inj << (8 * pa))) & M32
    if pa > -4:
        return v ^ (inj >> (8 * -pa))
    return v


def step4(x, d):
    """step4_next: x advanced over four zero bytes, then d XORed in -- the
    dword-by-dword slice-by-4 fold (raw(A || B) = M_4(raw(A)) ^ raw(B) for a
    dword B is M_4(raw(A)) ^ step4(0, B) ... written as the kernel does)."""
    return zeros(x, 4) ^ d


def lane_fragment(buf, p, G, inj=M32):
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
            d = head_dword(v, kh - (16 * k + 4 * j), inj)
            x = d if (k == 0 and j == 0) else step4(x, d)
    # x is the dword stream folded without its last four-byte advance; the
    # kernel's final step4_next(x, 0) gives raw of the dwords
    return step4(x, 0) if np16 else 0


def kernel_items(buf, p, length, stored=None, crc_in=0):
    """(R ^ C, t) as k_items computes it for span [p, p + length)."""
    t = tail_pad(p, length)
    vlen = length + t
    assert fused_vlen(vlen)
    G = p + vlen - BLOCK
    r = lane_fragment(buf, p, G, ~crc_in & M32)
    # the fragment chain is the register from ~c over [p, G)
    assert r == reg(~crc_in & M32, buf[p:G])
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
        # MODE 0 with an initial CRC c: ~c injected at p
        for c in (0x9C44184B, int(rng.integers(0, 1 << 32))):
            RCc, _ = kernel_items(buf, p, length, crc_in=c)
            assert ~mulmodp(RCc, xpow8_inv(t)) & M32 == oracle.crc32c(c, D)
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
