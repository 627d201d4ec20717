"""CPU restatement of k_count's wave-cooperative whole spans (round 4,
crc32c_kernels.hip whole_chunks / span_corr_arg's pieces case).

A span D = [p, E) of vlen = len + t <= kWholeMax bytes is all its thread's
(span_corr: z = M_t(f), f the register after D from ~c).  Its lane no longer
runs that chain alone while the other 63 lanes of the wave idle: the wave
cuts the pieces [ph, ceil16(E)) of all its whole spans (ph = floor16(p),
Ea = E + t) into 128-B chunks, every lane takes a chunk (r_c = raw of its
<= 8 pieces, the span's last piece cleared from E on, shifted past the rest
of the span: M_{Ea - end_c}(r_c)), and the chunks of one span are XORed into
R = raw([ph, Ea)) as the pieces lie with the tail F_t = [E, Ea) cleared, as
the span kernel clears it (round 5).  Then
    z = R ^ Z,  Z = M_{len+t}(~c ^ raw(F_h))
(F_h: the kh foreign bytes before p, moved to the top of a zero piece) --
the identity the span kernel's units rest on.  The owner of chunk q is the
first lane whose inclusive chunk count exceeds q.
"""
import numpy as np
import pytest

from tests import oracle
from tests.span_model import M32, WHOLE_MAX, mulmodp, span_head, tail_pad, xpow8

CHUNK = 128


def raw(data):
    return ~oracle.crc32c(M32, bytes(data)) & M32


def reg(r, data):
    return ~oracle.crc32c(~r & M32, bytes(data)) & M32


def zeros(v, n):
    return oracle.lib().oracle_shift_zeros(v & M32, n)


def is_whole(p, length):
    g1o, drop = span_head(p, length)
    return length > 0 and drop and g1o == length + tail_pad(p, length)


def chunks_R(buf, ph, e, ea, chunk=CHUNK):
    """R as the wave forms it from chunk-byte chunks (kWholeChunk) over the
    pieces [ph, ceil16(e)), the last one cleared from e on."""
    e16 = (e + 15) & ~15
    R = 0
    for c0 in range(ph, e16, chunk):
        np_ = min(chunk // 16, (e16 - c0) // 16)
        r = 0
        for k in range(np_):
            piece = bytearray(buf[c0 + 16 * k:c0 + 16 * k + 16])
            if c0 + 16 * k + 16 > e:
                piece[e - (c0 + 16 * k):] = bytes(c0 + 16 * k + 16 - e)
            r = reg(r, piece)
        after = ea - (c0 + 16 * np_)
        R ^= mulmodp(r, xpow8(after)) if after else r
    return R


def z_pieces(buf, p, length, c):
    """span_corr's pieces-as-they-lie correction (its non-drop branch)."""
    kh = p & 15
    t = tail_pad(p, length)
    y = ~c & M32
    if kh:
        y ^= raw(bytes(16 - kh) + bytes(buf[p - kh:p]))
    return mulmodp(y, xpow8(length + t))


def owners(nch):
    """(owner lane, chunk index) of every chunk q, by the kernel's search."""
    inc = np.cumsum(nch)
    excl = inc - nch
    out = []
    for q in range(int(inc[-1]) if len(inc) else 0):
        s = 0
        for step in (32, 16, 8, 4, 2, 1):
            if inc[s + step - 1] <= q:
                s += step
        out.append((s, q - int(excl[s])))
    return out


@pytest.mark.parametrize("seed", range(6))
def test_whole_span_chunks_give_the_thread_chain(seed):
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, 1 << 15, dtype=np.uint8).tobytes()
    for _ in range(60):
        length = int(rng.integers(1, WHOLE_MAX + 1))
        p = int(rng.integers(16, len(buf) - length - 32))
        if not is_whole(p, length):
            continue
        c = int(rng.integers(0, 1 << 32))
        t = tail_pad(p, length)
        ph, e, ea = p - (p & 15), p + length, p + length + t
        R = chunks_R(buf, ph, e, ea)
        assert R == raw(bytes(buf[ph:e]) + bytes(t))
        for chunk in (32, 64, 256):  # (other chunk sizes: the same R)
            assert chunks_R(buf, ph, e, ea, chunk) == R
        f = reg(~c & M32, buf[p:p + length])
        assert R ^ z_pieces(buf, p, length, c) == zeros(f, t)  # = span_corr's M_t(f)
        assert ~f & M32 == oracle.crc32c(c, buf[p:p + length])


def test_whole_spans_are_at_most_17_chunks():
    for length in range(1, WHOLE_MAX + 1):
        for al in range(16):
            if is_whole(al, length):
                assert (length + tail_pad(al, length) + al + CHUNK - 1) // CHUNK <= 9


@pytest.mark.parametrize("seed", range(4))
def test_chunk_owner_search(seed):
    rng = np.random.default_rng(seed)
    nch = rng.integers(0, 18, 64) * (rng.random(64) < 0.3)
    got = owners(nch)
    want = [(s, k) for s in range(64) for k in range(int(nch[s]))]
    assert got == want
