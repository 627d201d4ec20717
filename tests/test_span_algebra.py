"""CPU check of the span kernels' algebra (crc32c_kernels.hip "Pieces as they
lie", span_corr, mask_tail, k_final): with R = the XOR over a span's work
units of M_{Ea - e}(raw of the unit's 16-B pieces as they lie in memory, the
span's tail bytes [E, Ea) cleared) -- what k_spans accumulates -- and Z from
the span's thread,
    crc32c(c, D) = ~M_{-t}(R ^ Z)   and, for a verify,  R == W
for every alignment, length class (empty, short, one block, head fragment
taken or not, multi-segment) and initial CRC.  The expected CRC comes from the
oracle (pinned by the reference's vectors, tests/test_oracle.py)."""
import numpy as np
import pytest

from tests import oracle
from tests.span_model import (M32, SEG, mulmodp, span_head, tail_pad, units_of, xpow8, xpow8_inv)


@pytest.fixture(autouse=True, params=[(1024, 1024), (256, 1024), (128, 2048)], ids=lambda v: f"frag{v[0]}-whole{v[1]}")
def limits(request, monkeypatch):
    """The head-fragment and whole-span limits (kFragMax, kWholeMax) are build
    constants; the geometry and algebra must hold for any of them."""
    from tests import span_model
    monkeypatch.setattr(span_model, "FRAG_MAX", request.param[0])
    monkeypatch.setattr(span_model, "WHOLE_MAX", request.param[1])


def reg(r, data):
    """CRC register advanced from r over data (crc32c(c, D) = ~reg(~c, D))."""
    return ~oracle.crc32c(~r & M32, bytes(data)) & M32


def raw(data):
    return reg(0, data)


def kernel_R(buf, p, length):
    """What k_spans accumulates for span [p, p + length) of buf."""
    E = p + length
    Ea = E + tail_pad(p, length)
    R = 0
    for up, eo, niters, _single, _segk in units_of(0, p, length):
        e = up + eo
        lo = up - (up & 15) if niters else e  # load_block: pieces from floor16(p)
        piece = bytearray(buf[lo:e])
        if e > E:  # mask_tail: the last line's bytes from E on
            piece[E - lo:] = bytes(e - E)
        R ^= mulmodp(raw(piece), xpow8(Ea - e))
    return R


def span_corr(buf, p, length, c):
    """Z of span_corr, restated."""
    t = tail_pad(p, length)
    if length == 0:
        return mulmodp(~c & M32, xpow8(t))
    vlen = length + t
    g1o, drop = span_head(p, length)
    if drop and g1o == vlen:
        return mulmodp(reg(~c & M32, buf[p:p + length]), xpow8(t))
    if drop:
        z = mulmodp(reg(~c & M32, buf[p:p + g1o]), xpow8(vlen - g1o))
    else:
        kh = p & 15
        z = mulmodp(~c & M32 ^ raw(buf[p - kh:p]), xpow8(vlen))
    return z


CASES = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 63, 100, 1000, 1009, 1024, 1040, 2047, 4064, 4081, 4096, 4097, 4133,
         5000, 5100, 8192, 9000, 12345, SEG - 100, SEG + 16, SEG + 17, SEG + 1100, 2 * SEG + 50, 2 * SEG + 3000]


@pytest.mark.parametrize("length", CASES)
def test_crc_from_R_and_Z(length):
    rng = np.random.default_rng(length)
    buf = rng.integers(0, 256, 3 * SEG + 16384, dtype=np.uint8).tobytes()
    for _ in range(6):
        p = int(rng.integers(16, 4096 + 16))
        c = int(rng.integers(0, 1 << 32))
        R = kernel_R(buf, p, length)
        Z = span_corr(buf, p, length, c)
        t = tail_pad(p, length)
        v = R ^ Z
        if t:
            v = mulmodp(v, xpow8_inv(t))
        want = oracle.crc32c(c, buf[p:p + length])
        assert (~v & M32) == want, (p, length, c)
        # verify form (k_count MODE 1): W = Z(c = 0) ^ M_t(~stored), match iff R == W
        if length:
            stored = oracle.crc32c(0, buf[p:p + length])
            W = span_corr(buf, p, length, 0) ^ mulmodp(~stored & M32, xpow8(t))
            assert R == W
            W_bad = span_corr(buf, p, length, 0) ^ mulmodp(~(stored ^ 1) & M32, xpow8(t))
            assert R != W_bad
