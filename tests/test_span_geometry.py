"""CPU check of the span kernel's work-unit geometry (restated in
tests/span_model.py from crc32c_kernels.hip make_unit / span_units /
load_block): for every unit, the 16-B pieces read from memory lie inside
[floor16(p), e) of the unit (so no load leaves the pages of the span), and the
units of a span together with its head fragment (the bytes [p, G1) that the
span's thread reads when span_head drops them) cover every byte of [p, E)
exactly once.  No GPU needed: this guards the load addressing before a kernel
runs."""
import numpy as np
import pytest

from tests.span_model import BLOCK, SEG, WHOLE, make_unit, nseg_of, real_pieces, span_head, tail_pad, units_of


@pytest.fixture(autouse=True, params=[(1024, 1024), (256, 1024), (128, 2048)], ids=lambda v: f"frag{v[0]}-whole{v[1]}")
def limits(request, monkeypatch):
    """The head-fragment and whole-span limits (kFragMax, kWholeMax) are build
    constants; the geometry and algebra must hold for any of them."""
    from tests import span_model
    monkeypatch.setattr(span_model, "FRAG_MAX", request.param[0])
    monkeypatch.setattr(span_model, "WHOLE_MAX", request.param[1])


def check_units(base, off, length, units):
    P, E = base + off, base + off + length
    covered = np.zeros(length, np.int32)
    for p, eo, niters, _single, _segk in units:
        e = p + eo
        assert e % 16 == 0
        for k in range(niters):
            for a in real_pieces(p, eo, niters, k):
                assert a % 16 == (p - (p & 15)) % 16
                assert a >= p - (p & 15), "piece before floor16(p)"
                assert a + 16 <= e, "piece past the unit's grid end"
                lo, hi = max(a, P, p), min(a + 16, E)
                if hi > lo:
                    covered[lo - P:hi - P] += 1
        # the prefetch of a unit with no blocks reads nothing
        if niters == 0:
            assert real_pieces(p, eo, niters, 0) == []
    g1o, drop = span_head(P, length)
    if drop:  # the head fragment, read by the span's thread
        covered[:min(g1o, length)] += 1
    assert (covered == 1).all()


@pytest.mark.parametrize("seed", range(6))
def test_span_loads_stay_in_the_span_and_cover_it(seed):
    rng = np.random.default_rng(seed)
    for _ in range(80):
        base = 4096 * int(rng.integers(1, 9)) + int(rng.choice([0, 16, 32, 1, 7]))
        length = int(rng.choice([0, 1, 3, 4, 15, 17, 100, 1000, 1030, 4096, 4133, 4165, 5100, 8192, 65536,
                                 65552, 65553, 66560, 200000]))
        length = max(0, length + int(rng.integers(-3, 4)))
        off = int(rng.integers(0, 9000))
        if rng.random() < 0.2:  # one unit for the whole span (k_expand's overlap fallback)
            units = [make_unit(base, off, length, WHOLE)]
        else:
            units = units_of(base, off, length)
        check_units(base, off, length, units)


def test_head_fragment_rule():
    """The 4133-B spans of a packed page (config 5) always leave their ~50-B
    head to the thread, so every unit is exactly one full block."""
    for kh in range(16):
        for length in (4133, 4100, 4160):
            p = 4096 * 3 + kh
            units = units_of(0, p, length)
            assert len(units) == 1 and units[0][2] == 1 and units[0][1] == BLOCK
    # a span that fits one block is not given to the kernel
    for length in (1, 64, 1000, 1024 - 15):
        assert units_of(0, 7, length) == []
    # a long span keeps its segments; a head segment of one block whose bytes
    # are all in the fragment disappears
    for extra, lost in ((2000, 0), (100, 1), (5000, 0)):
        p, length = 5, 3 * SEG + extra
        vlen = length + tail_pad(p, length)
        assert len(units_of(0, p, length)) == nseg_of(vlen) - lost


def test_one_block_matches_the_unit_plan():
    """k_blocks takes a span iff the planner would give it exactly one unit of
    one whole block (and the same block), and no unit at all iff it has none."""
    from tests.span_model import one_block
    rng = np.random.default_rng(5)
    for _ in range(3000):
        p = int(rng.integers(0, 1 << 20))
        length = int(rng.choice([rng.integers(0, 9000), rng.integers(4000, 5200)]))
        fast, none, g1 = one_block(p, length)
        units = units_of(0, p, length)
        assert none == (len(units) == 0)
        one = len(units) == 1 and units[0][2] == 1 and (units[0][1] + (units[0][0] & 15)) == BLOCK
        assert (fast and not none) == one, (p, length)
        if one:  # the block k_blocks reads is the unit's block
            assert units[0][0] - (units[0][0] & 15) == g1
