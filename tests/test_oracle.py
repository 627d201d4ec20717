"""The oracle pinned against the reference's own answers.

kat.json holds the known answers of testapp.c:853-879 plus RFC 3720 vectors;
spans.npz and items.npz hold outputs of the reference crc32c.c itself
(tests/golden/make_golden.py).
"""
import json
import os

import numpy as np
import pytest

from . import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _kat():
    with open(os.path.join(GOLD, "kat.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _kat(), ids=lambda c: c["name"])
def test_kat(case):
    data = bytes.fromhex(case["hex"])
    assert oracle.crc32c(case["crc_in"], data) == case["expect"]
    assert oracle.crc32c_bitwise(case["crc_in"], data) == case["expect"]


def test_testapp_values_literal():
    # testapp.c:861-876, literally
    buf = bytes(range(256))
    c = oracle.crc32c(0, buf)
    assert c == 0x9C44184B
    c = oracle.crc32c(c, buf)
    assert c == 0xAE10EE5A
    assert oracle.crc32c(c, buf[1:255]) == 0xED37B906


def test_all_lengths_and_alignments():
    g = np.load(os.path.join(GOLD, "spans.npz"))
    buf, crc0, cin, crcin = g["buf"], g["crc0"], g["cin"], g["crcin"]
    raw = buf.tobytes()
    for n in range(crc0.shape[0]):
        for off in range(8):
            assert oracle.crc32c(0, raw[off:off + n]) == crc0[n, off]
            assert oracle.crc32c(int(cin[n, off]), raw[off:off + n]) == crcin[n, off]


def test_bitwise_matches_sliced_on_sample():
    g = np.load(os.path.join(GOLD, "spans.npz"))
    raw = g["buf"].tobytes()
    for n in (0, 1, 7, 8, 9, 63, 64, 65, 255, 1000, 4200):
        assert oracle.crc32c_bitwise(0, raw[3:3 + n]) == g["crc0"][n, 3]


def test_combine_and_shift():
    rng = np.random.default_rng(1)
    for _ in range(50):
        a = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        c0 = int(rng.integers(0, 2**32))
        ca = oracle.crc32c(c0, a)
        cb = oracle.crc32c(0, b)
        assert oracle.lib().oracle_crc32c_combine(ca, cb, len(b)) == oracle.crc32c(c0, a + b)


@pytest.mark.parametrize("name", ["cfg1", "varied"])
def test_items_spill_crc(name):
    g = np.load(os.path.join(GOLD, "items.npz"))
    buf, offs, crcs = g[f"{name}_buf"], g[f"{name}_offsets"], g[f"{name}_crc"]
    for o, c in zip(offs, crcs):
        assert oracle.lib().oracle_item_crc(buf[int(o):].ctypes.data) == c


def test_page_walk_matches_fixture():
    g = np.load(os.path.join(GOLD, "items.npz"))
    buf, offs = g["varied_buf"], g["varied_offsets"]
    wsz = int(g["varied_wbuf"])
    found = []
    for w in range(0, buf.size, wsz):
        o, ok = oracle.verify_span(buf[w:w + wsz])
        assert ok.all()
        found += [w + int(x) for x in o]
    assert found == [int(x) for x in offs]
