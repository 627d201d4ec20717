"""CPU check of the span kernel's balanced plan (crc32c_kernels.hip
span_blocks, unit_piece, put_unit / k_expand, k_spans' group ranges),
restated in tests/span_model.py:
  * span_blocks (k_count's packed block count) is the sum of the units' niters;
  * group g's records [starts[g], starts[g + 1]) hold exactly the blocks
    [g * per, (g + 1) * per) of the batch, in order, whatever the cuts;
  * a piece reads the same blocks as its unit did (the grid is the unit's),
    and the span's R rebuilt from the records -- each shifted by its block
    count, as k_spans' multiply does -- is the R of the unit plan, so the CRC
    the oracle gives follows (tests/test_span_algebra.py)."""
import numpy as np
import pytest

from tests import oracle
from tests.span_model import (BALANCE_MIN_PER, BLOCK, M32, SEG, balanced_plan, mulmodp, span_blocks, span_units, tail_pad,
                              units_of, xpow8)


def reg(r, data):
    return ~oracle.crc32c(~r & M32, bytes(data)) & M32


def blocks_of(rec):
    """The byte ranges k_spans' load_block covers for each block of a record."""
    p, eo, nb, _single, _shift = rec
    return [p + eo - BLOCK * (nb - k) for k in range(nb)]


def random_spans(rng, n, maxlen):
    lens = np.minimum(64 * 1.25 ** rng.integers(0, 40, n) * rng.uniform(0.5, 1.5, n), maxlen).astype(int)
    lens[rng.random(n) < 0.05] = 0
    offs, spans, pos = [], [], 1
    for length in lens:
        pos += int(rng.integers(0, 40))
        spans.append((pos, int(length)))
        pos += int(length)
    return spans, pos + 256  # (slack past the last span: its grid ends up to 127 B after it)


@pytest.mark.parametrize("seed", range(6))
def test_span_blocks_is_the_units_niters(seed):
    rng = np.random.default_rng(seed)
    for _ in range(400):
        p = int(rng.integers(0, 4096))
        length = int(rng.choice([0, 1, 15, 100, 1000, 1100, 4080, 4096, 4133, 9000, SEG, SEG + 16, SEG + 17,
                                 3 * SEG + 123, int(rng.integers(0, 5 * SEG))]))
        assert span_blocks(p, length) == sum(u[2] for u in units_of(0, p, length)), (p, length)
        assert span_units(p, length) == len(units_of(0, p, length))
        # k_expand's unit placement without a running sum (round 5: a wave's
        # lanes write any unit of the wave's spans): units after the first are
        # whole segments, so unit j's first block is
        # b0 + (j ? nb0 + S (j - 1) : 0), nb0 = span_blocks - S (ns - 1), S = SEG / BLOCK
        units = units_of(0, p, length)
        ns = len(units)
        if ns:
            nb0 = span_blocks(p, length) - (SEG // BLOCK) * (ns - 1)
            bs = 0
            for j, u in enumerate(units):
                assert bs == (nb0 + (SEG // BLOCK) * (j - 1) if j else 0), (p, length, j)
                bs += u[2]


@pytest.mark.parametrize("groups", [1, 2, 3, 7, 64, 1000, 5000])
def test_groups_get_equal_contiguous_block_ranges(groups):
    rng = np.random.default_rng(groups)
    spans, _ = random_spans(rng, 300, 5 * SEG)
    records, starts, per = balanced_plan(spans, groups)
    # the unit plan's blocks, in order: (span, absolute block start)
    want = [(s, b) for s, (p, length) in enumerate(spans) for u in units_of(0, p, length)
            for b in blocks_of((u[0], u[1], u[2], u[3], 0))]
    t = len(want)
    assert per == max(-(-t // groups), BALANCE_MIN_PER)  # (kBalanceMinPer blocks at least)
    got = []
    for g in range(groups):
        if g * per >= t:
            assert g not in starts  # a group past the blocks: none (k_spans clamps to the record count)
            continue
        lo = starts[g]
        hi = starts.get(g + 1, len(records))
        blocks = [(s, b) for s, rec in records[lo:hi] if rec for b in blocks_of(rec)]
        assert blocks == want[g * per:(g + 1) * per], g
        # the only empty record of a group is its last (a boundary at a unit's start)
        assert all(rec for _, rec in records[lo:hi - 1])
        got += blocks
    assert got == want


@pytest.mark.parametrize("groups", [1, 5, 33, 400])
def test_R_from_pieces_is_R_from_units(groups):
    rng = np.random.default_rng(100 + groups)
    spans, size = random_spans(rng, 60, 3 * SEG)
    buf = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    records, _, _ = balanced_plan(spans, groups)

    def rec_raw(rec):
        p, eo, nb, _single, _shift = rec
        e = p + eo
        lo = p - (p & 15) if nb else e
        return reg(0, buf[lo:e])

    R = [0] * len(spans)
    for s, rec in records:
        if rec is None:
            continue
        p0, length = spans[s]
        Ea = p0 + length + tail_pad(p0, length)
        e = rec[0] + rec[1]
        assert Ea - e == BLOCK * rec[4]  # the shift k_spans multiplies by (4 KiB blocks)
        R[s] ^= mulmodp(rec_raw(rec), xpow8(BLOCK * rec[4]))
    for s, (p, length) in enumerate(spans):
        Ea = p + length + tail_pad(p, length)
        want = 0
        for up, eo, nb, _single, _segk in units_of(0, p, length):
            e = up + eo
            lo = up - (up & 15) if nb else e
            want ^= mulmodp(reg(0, buf[lo:e]), xpow8(Ea - e))
        assert R[s] == want, (s, p, length)
