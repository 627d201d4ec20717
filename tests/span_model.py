"""Integer restatement of the span kernels' work-unit geometry and of the
per-span correction (memcached_amd/csrc/crc32c_kernels.hip: nseg_of,
span_head, span_units, make_unit, load_block, span_corr).  Test
infrastructure: the CPU tests check the addressing and the algebra with it,
without a GPU."""
SEG = 128 * 1024  # kSegBytes
BLOCK = 4096
WHOLE = 0xFFFFFFFF
FRAG_MAX = 128    # kFragMax: a head fragment [p, G1) of at most this is the thread's
WHOLE_MAX = 512   # kWholeMax: so is a whole span of vlen at most this
POLY = 0x82F63B78
M32 = 0xFFFFFFFF


GRID = 128  # kGridAlign: the planned path's grid is anchored at E rounded up to a 128-B line


def tail_pad(p, length):
    """t = Ea - E, Ea = E rounded up to a 128-B line (grid_pad; round 5,
    it was 16 before)."""
    return (-(p + length)) & (GRID - 1)


def nseg_of(vlen):
    return 1 if vlen <= SEG + 16 else (vlen - 16 + SEG - 1) // SEG


def span_head(p, length):
    """(G1 - p, drop): G1 = the first point of the span's 4 KiB grid (anchored
    at Ea) after ph; drop = the head fragment [p, G1) is the span thread's."""
    kh = p & 15
    x = length + tail_pad(p, length) + kh
    g1o = x - BLOCK * ((x - 1) // BLOCK) - kh if length else 0
    return g1o, frag_drop(length, g1o, length + tail_pad(p, length))


def frag_drop(length, g1o, vlen):
    return length != 0 and (g1o <= FRAG_MAX or vlen <= WHOLE_MAX)


def span_units(p, length):
    if length == 0:
        return 0
    vlen = length + tail_pad(p, length)
    ns = nseg_of(vlen)
    g1o, drop = span_head(p, length)
    return ns - (1 if drop and g1o == vlen - (ns - 1) * SEG else 0)


def first_seg(p, length, nunit):
    return nseg_of(length + tail_pad(p, length)) - nunit if nunit else 0


def make_unit(base, off, length, seg):
    """(p, eo = e - p, niters, single, segk) of one work unit."""
    p0 = base + off
    vlen = length + tail_pad(p0, length)
    nseg = 1 if seg == WHOLE else nseg_of(vlen)
    single = nseg == 1
    head = single or seg == 0
    eo0 = vlen - (0 if single else (nseg - 1 - seg) * SEG)
    po = 0 if head else eo0 - SEG
    if head:
        g1o, drop = span_head(p0, length)
        if drop:
            po = g1o
    eo = eo0 - po
    niters = (eo + ((p0 + po) & 15) + BLOCK - 1) // BLOCK if length else 0
    return p0 + po, eo, niters, single, 0 if single else nseg - 1 - seg


def units_of(base, off, length):
    """The work units k_expand writes for a span."""
    nu = span_units(base + off, length)
    s0 = first_seg(base + off, length, nu)
    return [make_unit(base, off, length, s0 + s) for s in range(nu)]


def real_pieces(p, eo, niters, k):
    """Addresses of the pieces load_block reads from memory for block k (K1's
    lane layout: lane li's piece j at G + 512 j + 16 li)."""
    grel = eo - BLOCK * (niters - k)
    out = []
    for li in range(32):
        lrel = grel + 16 * li
        e0 = lrel + 16 + (p & 15) if niters else -BLOCK - 16
        for j in range(8):
            if e0 + 512 * j > 0:
                out.append(p + lrel + 512 * j)
    return out


# --- GF(2) arithmetic (crc32c.c:58-137's algebra, reflected basis) ---------

def mulmodp(a, b):
    prod = 0
    for i in range(31, -1, -1):
        if (a >> i) & 1:
            prod ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return prod


def xpow8(n):
    r, sq = 0x80000000, 0x00800000
    while n:
        if n & 1:
            r = mulmodp(r, sq)
        n >>= 1
        if n:
            sq = mulmodp(sq, sq)
    return r


_INV = {}


def xpow8_inv(t):
    """x^(-8t): the y with y * x^(8t) = 1 (solved over GF(2))."""
    if t not in _INV:
        a = xpow8(t)
        basis = {}
        for i in range(32):
            v, comb = mulmodp(1 << i, a), 1 << i
            for bit in sorted(basis, reverse=True):
                if (v >> bit) & 1:
                    v ^= basis[bit][0]
                    comb ^= basis[bit][1]
            if v:
                basis[v.bit_length() - 1] = (v, comb)
        target, comb = 0x80000000, 0
        for bit in sorted(basis, reverse=True):
            if (target >> bit) & 1:
                target ^= basis[bit][0]
                comb ^= basis[bit][1]
        assert target == 0
        _INV[t] = comb
    return _INV[t]


def one_block(p, length):
    """(is one block or none, none, G1) -- k_blocks' test (crc32c_kernels.hip one_block)."""
    kh = p & 15
    vlen = length + tail_pad(p, length)
    x = vlen + kh
    g1o = x - BLOCK * ((x - 1) // BLOCK) - kh if length else 0
    drop = frag_drop(length, g1o, vlen)
    none = length == 0 or (drop and g1o == vlen)
    if not drop and x == BLOCK:  # the unit [ph, Ea) is itself one block
        return True, False, p - kh
    return none or (drop and vlen - g1o == BLOCK), none, p + g1o


# --- balanced plan (crc32c_kernels.hip span_blocks, unit_piece, put_unit) ---

SEG_BLOCKS = SEG // BLOCK
BALANCE_MIN_PER = 2  # kBalanceMinPer


def span_blocks(p, length):
    """4 KiB blocks of the span's work units (span_blocks)."""
    nu = span_units(p, length)
    if nu == 0:
        return 0
    vlen = length + tail_pad(p, length)
    ns = nseg_of(vlen)
    if nu < ns:
        return SEG_BLOCKS * nu
    g1o, drop = span_head(p, length)
    po = g1o if drop else 0
    eo = vlen - (ns - 1) * SEG - po
    return (eo + ((p + po) & 15) + BLOCK - 1) // BLOCK + SEG_BLOCKS * (ns - 1)


def unit_piece(unit, k0, k1):
    """Blocks [k0, k1) of unit (p, eo, niters, single, shift in blocks) as a
    record of their own; None for an empty one (unit_piece)."""
    p, eo, nb, single, shift = unit
    if k0 == 0 and k1 == nb:
        return unit
    if k0 == k1:
        return None
    delta = eo - BLOCK * (nb - k0) if k0 else 0
    return (p + delta, eo - BLOCK * (nb - k1) - delta, k1 - k0, False, shift + nb - k1)


def balanced_plan(spans, groups):
    """Records and group starts of a batch [(p, length), ...] for `groups`
    32-lane groups (k_expand + k_expand_big with a balanced plan).  Returns
    (records, starts, per): records[i] = (span, record) with record as in
    unit_piece, starts[g] = group g's first record (g = 1 .. groups - 1 with
    blocks; groups past the last have none)."""
    units = []  # (span, unit with its shift in blocks)
    for s, (p, length) in enumerate(spans):
        for up, eo, nb, single, segk in units_of(0, p, length):
            units.append((s, (up, eo, nb, single, SEG_BLOCKS * segk)))
    t = sum(u[2] for _, u in units)
    per = max(-(-t // groups), BALANCE_MIN_PER)  # (k_expand: at least kBalanceMinPer blocks per group)
    gm = -(-t // per)
    starts = {0: 0}
    records = []
    bs = 0
    for j, (s, u) in enumerate(units):
        nb = u[2]
        cuts = min(-(-bs // per) - 1, gm - 1) if bs and gm else 0
        assert len(records) == j + cuts  # the record index k_expand computes
        k0 = 0
        g = max(-(-bs // per), 1)
        while g < gm and g * per < bs + nb:
            kb = g * per - bs
            records.append((s, unit_piece(u, k0, kb)))
            starts[g] = len(records)
            k0 = kb
            g += 1
        records.append((s, unit_piece(u, k0, nb)))
        bs += nb
    return records, starts, per
