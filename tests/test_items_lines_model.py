"""CPU restatement of K5's line-anchored form (round 4, crc32c_kernels.hip
k_items, MCRC_K5_LINES): the block of an image starts and ends on 128-B lines,
so no HBM line is read both by a block and by an image's per-lane prep.

For span D = [p, E) with initial CRC c:
* A = ceil128(p + 4), B = floor128(E): the image's block is the virtual
  4 KiB window [A, A + 4096) -- the whole lines [A, B) of D, zeros past B
  (the group's lanes whose pieces start at or past B read the zero line);
  the shape is fused when the window holds 31 or 32 of D's lines;
* the epoch lane takes the head [p, A) (4..131 bytes; bytes below p cleared,
  ~c XORed into [p, p + 4): r_h = the register from ~c over [p, A)) and the
  tail [B, Et), Et = ceil16(E), bytes from E on cleared (r_t = raw of
  [B, E) followed by pad = Et - E zero bytes);
* with R = raw of the window from the group's lanes,
    V = M_{Et-A}(r_h) ^ M_{Et-A-4096}(R) ^ r_t = M_pad(f),
  f the register after D from ~c (the second shift is negative when the
  window runs past B: through round 5 the kernel multiplied by x^(8e) from
  a table for e in [-128, 4352));
* crc32c(c, D) = ~M_{-pad}(V); a verify is good iff V == M_pad(~stored).
* Round 6: the epoch lane forms W = M_128(V) = M_d(M_4096(r_h) ^ R) ^
  M_128(r_t), d = Et - A - 3968 in [0, 272), with the table operators
  (M_2048 twice, the tree levels M_16..M_128 by the bits of d, byte shifts
  below 16) instead of two multiplies by x^(8e): a verify is good iff
  W == M_128(M_pad(~stored)), the CRC is ~M_{-pad-128}(W).
Checked against the oracle at every 128-B alignment of the fused lengths.
"""
import numpy as np
import pytest

from tests import oracle
from tests.span_model import M32, mulmodp, xpow8, xpow8_inv

LINE = 128
BLOCK = 4096


def reg(r, data):
    return ~oracle.crc32c(~r & M32, bytes(data)) & M32


def raw(data):
    return reg(0, data)


def zeros(v, n):
    return oracle.lib().oracle_shift_zeros(v & M32, n)


def xk(e):
    """x^(8e) for -128 <= e < 4352 (the round-5 kernel's table; V below)."""
    assert -128 <= e < 4352
    return xpow8(e) if e >= 0 else xpow8_inv(-e)


def lines_shape(p, length):
    """(A, B, fused): k_items' line-anchored shape test."""
    A = (p + 4 + LINE - 1) // LINE * LINE
    E = p + length
    B = E // LINE * LINE
    return A, B, B > A and BLOCK - LINE <= B - A <= BLOCK


def head_dword(v, pa, inj):
    if pa >= 4:
        return 0
    if pa >= 0:
        return ((v & ((M32 << (8 * pa)) & M32)) ^ (inj << (8 * pa))) & M32
    if pa > -4:
        return v ^ (inj >> (8 * -pa))
    return v


def chain(dwords):
    """The lane's slice-by-4 chain over a dword stream from register 0."""
    x = 0
    for k, d in enumerate(dwords):
        x = d if k == 0 else zeros(x, 4) ^ d
    return zeros(x, 4) if dwords else 0


def head_chain(buf, p, A, inj):
    ph = p - (p & 15)
    dw = []
    for a in range(ph, A, 4):
        v = int.from_bytes(bytes(buf[a:a + 4]), "little")
        dw.append(head_dword(v, p - a, inj))
    return chain(dw)


def tail_chain(buf, B, E):
    Et = (E + 15) // 16 * 16
    dw = []
    for a in range(B, Et, 4):
        b = bytearray(buf[a:a + 4])
        for i in range(4):
            if a + i >= E:
                b[i] = 0
        dw.append(int.from_bytes(bytes(b), "little"))
    return chain(dw)


def shift_ops(y, d):
    """M_d(y) for 0 <= d < 512 as finish_run composes it: the tree levels
    M_256 (M_128 twice), M_128, M_64, M_32, M_16 by the bits of d, then
    zeros_lds for d mod 16."""
    assert 0 <= d < 512
    for bit, n in ((256, 256), (128, 128), (64, 64), (32, 32), (16, 16)):
        if d & bit:
            y = zeros(y, n)
    return zeros(y, d & 15)


def kernel_lines(buf, p, length, crc_in=0):
    """(V, W, pad) as the line-anchored k_lines computes them (W = M_128(V),
    round 6's form)."""
    A, B, fused = lines_shape(p, length)
    assert fused
    E = p + length
    Et = (E + 15) // 16 * 16
    pad = Et - E
    inj = ~crc_in & M32
    r_h = head_chain(buf, p, A, inj)
    assert r_h == reg(inj, buf[p:A])
    r_t = tail_chain(buf, B, E)
    assert r_t == zeros(raw(buf[B:E]), pad)
    window = bytes(buf[A:B]) + bytes(A + BLOCK - B)
    R = raw(window)
    V = mulmodp(r_h, xk(Et - A)) ^ mulmodp(R, xk(Et - A - BLOCK)) ^ r_t
    d = Et - A - (BLOCK - LINE)
    W = shift_ops(zeros(zeros(r_h, 2048), 2048) ^ R, d) ^ zeros(r_t, 128)
    return V, W, pad


@pytest.mark.parametrize("al", range(0, 128, 5))
def test_line_anchored_V_is_M_pad_of_the_register(al):
    rng = np.random.default_rng(al)
    buf = rng.integers(0, 256, 3 * BLOCK, dtype=np.uint8).tobytes()
    p = 256 + al
    for length in (4100, 4133, 4165, 4190, 4226, 4227):
        A, B, fused = lines_shape(p, length)
        if not fused:
            continue
        D = buf[p:p + length]
        f = reg(M32, D)
        V, W, pad = kernel_lines(buf, p, length)
        assert V == zeros(f, pad) and W == zeros(V, 128)
        crc = oracle.crc32c(0, D)
        assert ~mulmodp(V, xpow8_inv(pad)) & M32 == crc
        assert ~mulmodp(mulmodp(W, xpow8_inv(128)), xpow8_inv(pad)) & M32 == crc
        # verify: good iff V == M_pad(~stored), i.e. W == M_128(M_pad(~stored))
        assert V == zeros(~crc & M32, pad) and V != zeros(~(crc ^ 1) & M32, pad)
        assert W == zeros(zeros(~crc & M32, pad), 128) and W != zeros(zeros(~(crc ^ 1) & M32, pad), 128)
        c = int(rng.integers(0, 1 << 32))
        Vc, Wc, _ = kernel_lines(buf, p, length, crc_in=c)
        assert ~mulmodp(Vc, xpow8_inv(pad)) & M32 == oracle.crc32c(c, D)
        assert ~mulmodp(mulmodp(Wc, xpow8_inv(128)), xpow8_inv(pad)) & M32 == oracle.crc32c(c, D)


def test_line_anchored_shapes():
    """Every 128-B alignment of a 4133-B span (configs 2r and 5) is fused, and
    so is every length 4100..4227; lengths whose interior holds 33 lines or
    fewer than 31 are not; the head is 4..131 bytes, the exponents stay in
    the table's range."""
    for L in range(4100, 4228):
        for al in range(128):
            A, B, fused = lines_shape(al, L)
            assert fused, (L, al)
            E = al + L
            Et = (E + 15) // 16 * 16
            assert 4 <= A - al <= 131 and -128 <= Et - A - BLOCK and Et - A < 4352
            assert 0 <= Et - A - (BLOCK - LINE) < 272  # (d of finish_run's shift)
    assert not any(lines_shape(al, 4354)[2] and lines_shape(al, 4354)[1] - lines_shape(al, 4354)[0] > BLOCK
                   for al in range(128))
    assert not any(lines_shape(al, L)[2] for L in (3800, 3900, 4500) for al in range(128))


def lines_runs(n, W, w, nsr):
    """The images [(start, steps), ...] of wave w's runs (k_lines, round
    robin: run k of wave w starts at image (k W + w) 2 nsr)."""
    runs, k = [], 0
    while True:
        start = (k * W + w) * 2 * nsr
        if start >= n:
            return runs
        runs.append((start, min(nsr, (n - start + 1) // 2)))
        k += 1


@pytest.mark.parametrize("n", [1, 2, 63, 4096, 4097, 65535, 1 << 20, 4833600])
@pytest.mark.parametrize("grid", [1, 7, 256, 1024])
def test_line_runs_cover_every_image_once(n, grid):
    """Every image is taken by exactly one lane of one step of one run and
    runs hold at most 2 nsr <= 64 images (one per lane); nsr as launch_k5
    (crc32c_shim.hip) sets it."""
    W = grid * 16
    nsr = min(32, max(1, (n + 2 * W - 1) // (2 * W)))
    seen = np.zeros(n, dtype=np.int32)
    for w in range(W):
        if w * 2 * nsr >= n:
            break
        for start, steps in lines_runs(n, W, w, nsr):
            assert 1 <= steps <= nsr
            lanes = np.arange(64)
            items = start + lanes[(lanes < 2 * steps) & (start + lanes < n)]
            seen[items] += 1
    assert (seen == 1).all()
