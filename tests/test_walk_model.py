"""CPU check of the device page walk's round-trip algebra (k_walk in
crc32c_kernels.hip, restated here): one wave per wbuf guesses that the next 64
items all have the last item's size, reads their headers in one round trip,
and keeps the guesses up to the first lane whose item breaks the run.  The
claim to check is that this gives exactly the sequential walk of
storage_compact_readback (storage.c:950-1070) for ANY bytes: runs of equal
sizes of every length around the wave width, runs broken by other sizes, a
zeroed nkey, corrupt sizes, wbufs ending a few bytes after an item.  No GPU
needed."""
import numpy as np
import pytest

from memcached_amd import layout

WAVE = 64


def ntotal(buf, off):
    """ITEM_ntotal as the kernels compute it (ItemHdr::ntotal): nbytes as an
    unsigned 32-bit field, the sum in 64 bits (a corrupt size ends the wbuf
    instead of stepping backwards)."""
    nbytes = int.from_bytes(bytes(buf[off + 32:off + 36]), "little")
    flags = int(buf[off + 38]) | int(buf[off + 39]) << 8
    return 48 + int(buf[off + 41]) + 1 + nbytes + (4 if flags & 256 else 0) + (8 if flags & 2 else 0)


def seq_walk(buf, start, size):
    """storage.c:950-1070: nkey == 0 or fewer than 48 bytes left ends the wbuf."""
    out, off = [], 0
    while off + 48 <= size and buf[start + off + 41] != 0:
        out.append(off)
        off += ntotal(buf, start + off)
    return out


def wave_walk(buf, start, size, G=1, adaptive=True):
    """k_walk's loop, lane by lane (returns the offsets and the round trips).
    G: guesses per lane per round trip (candidate q * 64 + j in lane j; the
    width is 64 G).  The kernel reads one (G = 1); four were measured in round
    6 and rejected (profiles/r06_ablations/walk_guesses_ab.txt), and the
    walk's algebra holds for any G.  adaptive (the kernel since round 6):
    after a round trip whose guesses broke at lane 0 or 1, the next one
    guesses with lane 0 alone, and widens again when that guess holds."""
    full = WAVE * G
    out, off, s, trips = [], 0, 0, 0
    W = 1 if adaptive else full
    while off + 48 <= size:
        trips += 1
        lanes = []
        for j in range(W):
            o = off + j * s
            inb = (j == 0 or s != 0) and o + 48 <= size
            nkey = int(buf[start + o + 41]) if inb else 0
            nt = ntotal(buf, start + o) if inb else 48 + 1  # (header of zeros)
            item = inb and nkey != 0
            lanes.append((o, item, nt))
        m = next((j for j, (_o, item, nt) in enumerate(lanes) if not (item and nt == s)), W)
        last_item = m < W and lanes[m][1]
        k = m + (1 if last_item else 0) if m < W else W
        out += [lanes[j][0] for j in range(k)]
        if m == W:
            off += W * s
            W = full
        elif not last_item:
            break
        else:
            off += m * s + lanes[m][2]
            s = lanes[m][2]
            W = 1 if (adaptive and m <= 1) else full
    return out, trips


def _pages(rng, sizes, wbuf, cut=0):
    items = [layout.make_item(b"w%06d" % i, rng.integers(0, 256, n, dtype=np.uint8).tobytes(), cas=i + 1)
             for i, n in enumerate(sizes)]
    buf, offs = layout.pack_wbufs(items, wbuf)
    return buf[:buf.size - cut] if cut else buf


def _check(buf, wbuf):
    for start in range(0, buf.size, wbuf):
        size = min(wbuf, buf.size - start)
        want = seq_walk(buf, start, size)
        for G in (1, 4):  # (the kernel's one guess per lane, and four)
            for adaptive in (True, False):  # (the kernel since round 6, and before)
                got, _ = wave_walk(buf, start, size, G, adaptive)
                assert got == want


@pytest.mark.parametrize("run", [1, 2, 63, 64, 65, 127, 128, 129, 255, 256, 257, 300])
def test_equal_runs(run):
    rng = np.random.default_rng(run)
    sizes = []
    while len(sizes) < 900:
        sizes += [int(rng.choice([0, 5, 100, 4096]))] * run
    for wbuf in (1 << 20, 4165 * 64 + 47, 4165 * 64 + 48, 4165 * 65):
        _check(_pages(rng, sizes, wbuf, cut=wbuf // 3), wbuf)


def test_corrupt_headers():
    """Flipped nbytes bits (huge or odd sizes), zeroed nkeys and random header
    bytes: the walk goes wherever the sequential walk goes."""
    rng = np.random.default_rng(7)
    wbuf = 1 << 20
    buf = _pages(rng, [4096] * 600 + [int(x) for x in rng.integers(0, 3000, 400)], wbuf)
    offs = seq_walk(buf, 0, min(wbuf, buf.size))
    for t in range(40):
        b = buf.copy()
        for o in rng.choice(offs, 3, replace=False):
            pos = int(o) + int(rng.choice([32, 33, 34, 35, 38, 39, 41]))
            b[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        if t % 4 == 0:
            b[int(offs[int(rng.integers(0, len(offs)))]) + 41] = 0
        _check(b, wbuf)


def test_round_trips():
    """Equal-sized items cost one round trip per 64 (plus two to learn the
    size: one guess after the first item, then 64 per trip); items of mixed
    sizes one round trip each, with one header read per trip."""
    rng = np.random.default_rng(3)
    wbuf = 4 << 20
    buf = _pages(rng, [4096] * 1007, wbuf)
    got, trips = wave_walk(buf, 0, wbuf)
    assert len(got) == 1007 and trips == 2 + -(-1005 // WAVE) + (1 if 1005 % WAVE == 0 else 0)
    got, trips = wave_walk(buf, 0, wbuf, adaptive=False)
    assert len(got) == 1007 and trips == 1 + -(-1006 // WAVE) + (1 if 1006 % WAVE == 0 else 0)
    sizes = [int(x) for x in np.exp(rng.uniform(np.log(512), np.log(65536), 300))]
    buf = _pages(rng, sizes, wbuf)
    want = seq_walk(buf, 0, wbuf)
    got, trips = wave_walk(buf, 0, wbuf)
    assert got == want and trips <= len(want) + 1


@pytest.mark.parametrize("wbuf", [48, 49, 61, 64, 100, 127])
def test_tiny_wbufs(wbuf):
    """wbufs that hold at most one image, and buffers cut inside a wbuf or
    shorter than a header."""
    rng = np.random.default_rng(wbuf)
    items = [layout.make_item(b"k", rng.integers(0, 256, int(rng.integers(0, 3)), dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(200)]
    items = [it for it in items if len(it) <= wbuf]
    if items:
        buf, _ = layout.pack_wbufs(items, wbuf)
    else:
        buf = np.zeros(3 * wbuf, np.uint8)
    for cut in (0, wbuf // 2, max(buf.size - 47, 0)):
        _check(buf[:buf.size - cut], wbuf)
