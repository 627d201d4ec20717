"""CPU check of the span kernel's work-unit geometry, restated in integer
arithmetic (crc32c_kernels.hip make_unit / decode_unit / load_block): for every
unit, the 16-B pieces read from memory lie inside [floor16(p), e) of the unit
(so no load leaves the pages of the span), and over a span's segments they
cover every byte of [p, E) exactly once.  No GPU needed: this guards the load
addressing before a kernel runs."""
import numpy as np
import pytest

SEG = 64 * 1024
BLOCK = 4096
WHOLE = 0xFFFFFFFF


def nseg_of(vlen):
    return 1 if vlen <= SEG + 16 else (vlen - 16 + SEG - 1) // SEG


def make_unit(base, off, length, seg):
    """make_unit: (p, eo = e - p, Eo = E - p, niters) of one work unit."""
    p0 = base + off
    vlen = length + ((-(p0 + length)) & 15)
    nseg = 1 if seg == WHOLE else nseg_of(vlen)
    single = nseg == 1
    head = single or seg == 0
    eo0 = vlen - (0 if single else (nseg - 1 - seg) * SEG)
    po = 0 if head else eo0 - SEG
    eo = eo0 - po
    niters = (eo + ((p0 + po) & 15) + BLOCK - 1) // BLOCK if length else 0
    return p0 + po, eo, length - po, niters


def real_pieces(p, eo, niters, k):
    """Addresses of the pieces load_block reads from memory for block k."""
    grel = eo - BLOCK * (niters - k)
    out = []
    for li in range(32):
        lrel = grel + 32 * li
        e0 = lrel + 16 + (p & 15) if niters else -BLOCK - 16
        for r in range(4):
            er = e0 + 1024 * r
            if er > 0:
                out.append(p + lrel + 1024 * r)
            if er + 16 > 0:
                out.append(p + lrel + 1024 * r + 16)
    return out


@pytest.mark.parametrize("seed", range(6))
def test_span_loads_stay_in_the_span_and_cover_it(seed):
    rng = np.random.default_rng(seed)
    for _ in range(80):
        base = 4096 * int(rng.integers(1, 9)) + int(rng.choice([0, 16, 32, 1, 7]))
        length = int(rng.choice([0, 1, 3, 4, 15, 17, 100, 4096, 4133, 4165, 8192, 65536, 65552, 65553, 200000]))
        length = max(0, length + int(rng.integers(-3, 4)))
        off = int(rng.integers(0, 9000))
        P, E = base + off, base + off + length
        covered = np.zeros(length, np.int32)
        segs = [WHOLE] if rng.random() < 0.2 else range(nseg_of(length + ((-E) & 15)))
        for seg in segs:
            p, eo, Eo, niters = make_unit(base, off, length, seg)
            e = p + eo
            assert e % 16 == 0
            for k in range(niters):
                for a in real_pieces(p, eo, niters, k):
                    assert a % 16 == (p - (p & 15)) % 16
                    assert a >= p - (p & 15), "piece before floor16(p)"
                    assert a + 16 <= e, "piece past the unit's grid end"
                    lo, hi = max(a, P), min(a + 16, E, p + min(eo, Eo))
                    if hi > lo:
                        covered[lo - P:hi - P] += 1
            # the prefetch of a unit with no blocks reads nothing
            if niters == 0:
                assert real_pieces(p, eo, niters, 0) == []
        assert (covered == 1).all()
