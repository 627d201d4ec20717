"""GPU parity: every kernel, through the C-ABI (libmcrc32c.so), against the
CPU oracle and the reference-generated golden vectors.  Bit-exact."""
import os

import numpy as np
import pytest

try:  # GPU processes load torch (and its HIP runtime) before libmcrc32c.so
    import torch as _torch  # noqa: F401
except ImportError:
    pass

from memcached_amd import _lib, layout
from memcached_amd import crc32c as mc

from . import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(autouse=True, params=["small", "planned"])
def span_path(request):
    """Every case runs twice: batches of at most 8192 spans through the
    single-launch k_small (the default) and through the planned path
    (count / scan / expand / span kernel / final) that larger batches take
    (crc32c_set_small_max(0))."""
    prev = _lib.lib.crc32c_set_small_max(0 if request.param == "planned" else 8192)
    yield request.param
    _lib.lib.crc32c_set_small_max(prev)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    assert mc.gpu_count() >= 1, "libmcrc32c.so sees no gfx950 device"
    return t


def _dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def test_fixed_4096_k1(torch):
    rng = np.random.default_rng(42)
    n = 4099  # not a multiple of the 32 spans per block step
    host = rng.integers(0, 256, n * 4096, dtype=np.uint8)
    want = oracle.batch(host, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096))
    d = _dev(torch, host)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = _lib.Spans(d.data_ptr(), host.size, None, 4096, None, 4096, None, out.data_ptr(), n)
    import ctypes
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
    assert _lib.lib.crc32c_last_kernel_ms() > 0
    np.testing.assert_array_equal(_u32(out), want)
    # with per-item initial CRCs
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dcin = _dev(torch, cin.view(np.int32))
    s.crc_in = dcin.data_ptr()
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
    want_in = oracle.batch(host, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096), cin)
    np.testing.assert_array_equal(_u32(out), want_in)


@pytest.mark.parametrize("n,stride", [(1, 4096), (2, 4096), (3, 8192), (33, 4096), (65, 12288), (8193, 4096),
                                      (41160, 4096), (57347, 4096)])
def test_k1_edges(torch, n, stride):
    """K1 at item counts that leave odd groups, partial steps and idle waves,
    and at strides other than the item length; with and without crc_in.
    On 256 CUs (4096 waves, 2 items per wave-step) 41160 items give waves of
    6 and 5 steps, 57347 items waves of 8 and 7: every mix of the 4-step,
    2-step and single-step reductions."""
    import ctypes
    rng = np.random.default_rng(n)
    host = rng.integers(0, 256, n * stride, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * stride
    d = _dev(torch, host)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dcin = _dev(torch, cin.view(np.int32))
    for c in (None, cin):
        s = _lib.Spans(d.data_ptr(), host.size, None, stride, None, 4096,
                       None if c is None else dcin.data_ptr(), out.data_ptr(), n)
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
        np.testing.assert_array_equal(_u32(out), oracle.batch(host, offs, np.full(n, 4096), c))


def test_golden_all_lengths_alignments(torch):
    g = np.load(os.path.join(GOLD, "spans.npz"))
    buf = g["buf"]
    L, A = g["crc0"].shape
    offs = np.tile(np.arange(A, dtype=np.uint64), L)
    lens = np.repeat(np.arange(L, dtype=np.uint32), A)
    d = _dev(torch, buf)
    out = mc.batch(d, offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), g["crc0"].reshape(-1))
    cin = g["cin"].reshape(-1)
    out = mc.batch(d, offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)),
                   crc_in=_dev(torch, cin.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), g["crcin"].reshape(-1))


def test_golden_host_path():
    g = np.load(os.path.join(GOLD, "spans.npz"))
    L, A = g["crc0"].shape
    offs = np.tile(np.arange(A, dtype=np.uint64), L)
    lens = np.repeat(np.arange(L, dtype=np.uint32), A)
    # caller order (offsets not sorted): the library stages in offset order and scatters back
    out = mc.batch(g["buf"], offsets=offs, lens=lens, crc_in=g["cin"].reshape(-1))
    np.testing.assert_array_equal(out, g["crcin"].reshape(-1))
    order = np.argsort(offs, kind="stable")
    out = mc.batch(g["buf"], offsets=offs[order], lens=lens[order], crc_in=g["cin"].reshape(-1)[order])
    np.testing.assert_array_equal(out, g["crcin"].reshape(-1)[order])


def test_16b_aligned_spans(torch):
    """Spans whose starts and lengths are multiples of 16 (no head or tail
    fragment: the span kernel's pieces are exactly the span)."""
    rng = np.random.default_rng(5)
    n = 3000
    lens = (rng.integers(0, 700, n) * 16).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 16 * rng.integers(0, 3, n - 1))]).astype(np.uint64)
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    want = oracle.batch(host, offs, lens)
    d = _dev(torch, host)
    out = mc.batch(d, offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


def test_variable_unaligned_up_to_1mib(torch):
    rng = np.random.default_rng(7)
    classes = np.array([int(64 * 1.25 ** k) for k in range(44) if 64 * 1.25 ** k <= 1 << 20])
    p = 1.0 / np.arange(1, classes.size + 1)
    n = 2500
    cls = rng.choice(classes.size, n, p=p / p.sum())
    lens = (classes[cls] * rng.uniform(0.9, 1.1, n)).astype(np.uint32) + rng.integers(0, 16, n).astype(np.uint32)
    lens[:5] = [0, 1, 2, 3, (1 << 20) + 37]
    offs = np.concatenate([[3], 3 + np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 5), dtype=np.uint8)
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(host, offs, lens, cin)
    d = _dev(torch, host)
    out = mc.batch(d, offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)),
                   crc_in=_dev(torch, cin.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)
    # the same batch through the host staging path and the multi-GPU splitter
    np.testing.assert_array_equal(mc.batch(host, offsets=offs, lens=lens, crc_in=cin), want)
    np.testing.assert_array_equal(mc.batch_multi(host, offsets=offs, lens=lens, crc_in=cin), want)


@pytest.mark.parametrize("aligned", [False, True])
def test_long_spans_cross_segments(torch, aligned):
    """Spans of several 64 KiB work units: segment split + combine pass
    (aligned: every start and length a multiple of 16, the same kernels)."""
    rng = np.random.default_rng(31 + aligned)
    lens = rng.integers(0, 5 << 20, 60).astype(np.uint32)
    lens[:6] = [65536, 65537, 65535, 131072, 131073, (3 << 20) + 5]
    if aligned:
        lens = (lens // 16 * 16).astype(np.uint32)
    pad = 16 if aligned else 7
    offs = np.concatenate([[pad], pad + np.cumsum(lens[:-1].astype(np.uint64) + pad)]).astype(np.uint64)
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    cin = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(host, offs, lens, cin)
    d = _dev(torch, host)
    out = mc.batch(d, offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)),
                   crc_in=_dev(torch, cin.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


def test_very_long_spans(torch):
    """Spans of more than 256 segments (16 MiB): the segment shift takes the
    second factor of the shift table (x^(8 * 64Ki * 256 j)); k_expand_big
    places their units.  Up to 300 MiB, unaligned, with nested spans."""
    rng = np.random.default_rng(35)
    size = (300 << 20) + 4096
    host = rng.integers(0, 256, size, dtype=np.uint8)
    offs = np.array([3, 5, (1 << 20) + 1, 7 << 20, 123, 40 << 20, 9], dtype=np.uint64)
    lens = np.array([(17 << 20) + 5, (33 << 20) + 1, (16 << 20) + 16, (64 << 20) + 3, 4133, (256 << 20) - 77,
                     (300 << 20) + 11], dtype=np.uint32)
    cin = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(host, offs, lens, cin)
    out = mc.batch(_dev(torch, host), offsets=_dev(torch, offs.view(np.int64)),
                   lens=_dev(torch, lens.view(np.int32)), crc_in=_dev(torch, cin.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


MAX_SPAN = _lib.CRC32C_MAX_SPAN


def test_maximum_length_spans(torch):
    """Spans at the length limit (2 GiB - 64 KiB) and just under it, past
    2^31 - 2^20, overlapping so that the planner processes some as one unit
    (the second span pass), next to a short and an empty span, in a buffer
    past 2 GiB; a span one byte over the limit is not read: out 0 and
    CRC32C_ERANGE, the others still exact."""
    import ctypes
    rng = np.random.default_rng(41)
    size = (1 << 31) + 8192
    host = np.frombuffer(rng.bytes(size), dtype=np.uint8)
    offs = np.array([1, 7, (1 << 20) + 5, (1 << 31) + 100, 3, 2], dtype=np.uint64)
    lens = np.array([MAX_SPAN, MAX_SPAN - 1, MAX_SPAN - (1 << 20) - 11, 4133, 0, MAX_SPAN + 1], dtype=np.uint32)
    cin = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(host, offs[:-1], lens[:-1], cin[:-1])
    d = _dev(torch, host)
    d_offs, d_lens, d_cin = (_dev(torch, offs.view(np.int64)), _dev(torch, lens.view(np.int32)),
                             _dev(torch, cin.view(np.int32)))
    out = torch.empty(lens.size, dtype=torch.int32, device="cuda")
    sp = _lib.Spans(d.data_ptr(), size, d_offs.data_ptr(), 0, d_lens.data_ptr(), 0, d_cin.data_ptr(),
                    out.data_ptr(), lens.size)
    assert _lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_ERANGE
    got = _u32(out)
    np.testing.assert_array_equal(got[:-1], want)
    assert got[-1] == 0
    # without the oversize span the batch is clean
    sp.n = lens.size - 1
    assert _lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_OK
    np.testing.assert_array_equal(_u32(out)[:-1], want)
    # a fixed-length batch over the limit is rejected before any launch
    big = _lib.Spans(d.data_ptr(), size, None, 0, None, MAX_SPAN + 1, None, out.data_ptr(), 1)
    assert _lib.lib.crc32c_batch(ctypes.byref(big), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_EINVAL


def test_overlapping_long_spans_whole_pass(torch):
    """Overlapping spans whose units exceed the planner's capacity are processed
    whole by the second pass; results stay exact."""
    rng = np.random.default_rng(33)
    host = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 300
    offs = rng.integers(0, 200000, n).astype(np.uint64)
    lens = rng.integers(70000, (1 << 20) - 200000, n).astype(np.uint32)
    want = oracle.batch(host, offs, lens)
    out = mc.batch(_dev(torch, host), offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


def test_verify_long_items(torch):
    """Page verify of items whose spans exceed one 64 KiB unit."""
    rng = np.random.default_rng(35)
    items = [layout.make_item(b"big%05d" % i, rng.integers(0, 256, int(rng.integers(60000, 300000)),
                                                           dtype=np.uint8).tobytes(), cas=i) for i in range(40)]
    buf, offs = layout.pack_wbufs(items, 1 << 20)
    soffs, slens = layout.spans_of(buf, offs)
    layout.store_crcs(buf, offs, oracle.batch(buf, soffs, slens))
    ok, nbad = mc.verify_items(_dev(torch, buf), _dev(torch, offs.view(np.int64)))
    assert nbad == 0 and ok.cpu().numpy().all()
    buf[int(offs[5]) + 70000] ^= 4
    ok, nbad = mc.verify_items(buf, offs)
    assert nbad == 1 and ok[5] == 0


def test_verify_region_bound(torch):
    """A flipped high bit of nbytes makes a header claim a span past its wbuf:
    with region_bytes = wbuf size it is reported bad without being read; the
    neighbours are unaffected; without a region it is bad through its CRC."""
    rng = np.random.default_rng(36)
    items = [layout.make_item(b"rb%05d" % i, rng.integers(0, 256, 3000 + 37 * i, dtype=np.uint8).tobytes(), cas=i)
             for i in range(300)]
    wbuf = 1 << 20
    buf, offs = layout.pack_wbufs(items, wbuf)
    soffs, slens = layout.spans_of(buf, offs)
    layout.store_crcs(buf, offs, oracle.batch(buf, soffs, slens))
    buf[int(offs[7]) + 32 + 2] ^= 0x08  # nbytes += 512 KiB: crosses the 1 MiB wbuf
    for region in (wbuf, 0):
        ok, nbad = mc.verify_items(_dev(torch, buf), _dev(torch, offs.view(np.int64)), region_bytes=region)
        ok = ok.cpu().numpy()
        assert nbad == 1 and ok[7] == 0 and ok.sum() == offs.size - 1
    ok, nbad = mc.verify_items(buf, offs, region_bytes=wbuf)
    assert nbad == 1 and ok[7] == 0


def test_stamp_items(torch):
    """Write path: the spill CRC of every image of a wbuf written into exptime
    (storage.c:567), device and host, equals the oracle's; the stamped page
    then verifies clean; a header crossing its wbuf is left unstamped."""
    rng = np.random.default_rng(37)
    items = [layout.make_item(b"st%06d" % i, rng.integers(0, 256, int(rng.integers(0, 9000)), dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(900)]
    wbuf = 1 << 20
    buf, offs = layout.pack_wbufs(items, wbuf)
    soffs, slens = layout.spans_of(buf, offs)
    want = buf.copy()
    layout.store_crcs(want, offs, oracle.batch(buf, soffs, slens))
    d = _dev(torch, buf)
    ok, nbad = mc.stamp_items(d, _dev(torch, offs.view(np.int64)), region_bytes=wbuf)
    assert nbad == 0 and ok.cpu().numpy().all()
    np.testing.assert_array_equal(d.cpu().numpy(), want)
    h = buf.copy()
    ok, nbad = mc.stamp_items(h, offs, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    np.testing.assert_array_equal(h, want)
    ok, nbad = mc.verify_items(h, offs, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    # async device stamp on the default stream, fenced by a synchronize
    d = _dev(torch, buf)
    import ctypes
    doffs = _dev(torch, offs.view(np.int64))
    _lib.check(_lib.lib.crc32c_stamp_items(d.data_ptr(), d.numel(), wbuf, doffs.data_ptr(), offs.size, None, None,
                                           _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC,
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy(), want)
    # long images (> 64 KiB: several work units, stamped by the combine pass)
    big = [layout.make_item(b"lg%05d" % i, rng.integers(0, 256, int(rng.integers(65000, 400000)),
                                                        dtype=np.uint8).tobytes(), cas=i + 1) for i in range(30)]
    bbuf, boffs = layout.pack_wbufs(big, 1 << 20)
    bso, bsl = layout.spans_of(bbuf, boffs)
    bwant = bbuf.copy()
    layout.store_crcs(bwant, boffs, oracle.batch(bbuf, bso, bsl))
    bd = _dev(torch, bbuf)
    ok, nbad = mc.stamp_items(bd, _dev(torch, boffs.view(np.int64)), region_bytes=1 << 20)
    assert nbad == 0
    np.testing.assert_array_equal(bd.cpu().numpy(), bwant)
    ok, nbad = mc.stamp_items(bbuf, boffs, region_bytes=1 << 20)
    np.testing.assert_array_equal(bbuf, bwant)
    # malformed: nbytes claims a span past the wbuf -> not stamped, counted
    bad = buf.copy()
    bad[int(offs[11]) + 32 + 2] ^= 0x10
    ok, nbad = mc.stamp_items(bad, offs, region_bytes=wbuf)
    assert nbad == 1 and ok[11] == 0 and ok.sum() == offs.size - 1
    assert bytes(bad[int(offs[11]) + 28:int(offs[11]) + 32]) == b"\0\0\0\0"


def test_item_headers_at_every_alignment(torch):
    """Item images starting at every offset mod 16, so the header fields the
    kernels parse from two 16-B pieces (bytes 28..43, funnel-shifted by
    (off + 28) & 15: parse_hdr) sit at every alignment, with key
    lengths, value sizes, CAS and client flags varied so that the field bytes
    differ from image to image: stamp, verify (device and host) and the
    device page walk agree with the oracle, and one damaged image per
    alignment is reported exactly."""
    rng = np.random.default_rng(53)
    items = []
    for i in range(2048):
        nkey = 1 + (i * 37) % 250
        cas = None if i % 3 == 0 else i + 1
        cfl = (i * 2654435761) & 0xFFFFFFFF if i % 5 == 0 else 0
        key = (b"%06d" % i + b"k" * 250)[:nkey]
        vlen = int(rng.integers(0, 20000))
        # ITEM_ntotal = 1 (mod 16): consecutive images step through every residue
        vlen += (1 - len(layout.make_item(key, bytes(vlen), cas=cas, client_flags=cfl))) % 16
        items.append(layout.make_item(key, rng.integers(0, 256, vlen, dtype=np.uint8).tobytes(), cas=cas,
                                      client_flags=cfl))
    wbuf = 1 << 20
    buf, offs = layout.pack_wbufs(items, wbuf)
    assert {int(o) % 16 for o in offs} == set(range(16))
    soffs, slens = layout.spans_of(buf, offs)
    want = buf.copy()
    layout.store_crcs(want, offs, oracle.batch(buf, soffs, slens))
    d = _dev(torch, buf)
    ok, nbad = mc.stamp_items(d, _dev(torch, offs.view(np.int64)), region_bytes=wbuf)
    assert nbad == 0 and ok.cpu().numpy().all()
    np.testing.assert_array_equal(d.cpu().numpy(), want)
    # one damaged image per start residue (a value byte flipped)
    victims = [min(i for i in range(16 * r + 16, offs.size) if int(offs[i]) % 16 == r) for r in range(16)]
    bad = want.copy()
    for v in victims:
        o = int(offs[v])
        bad[o + int(rng.integers(48, layout.ntotal_of(bad, o)))] ^= 0x20
    for dev in (True, False):
        ok, nbad = mc.verify_items(_dev(torch, bad) if dev else bad, _dev(torch, offs.view(np.int64)) if dev else offs,
                                   region_bytes=wbuf)
        ok = ok.cpu().numpy() if dev else ok
        assert nbad == len(victims) and sorted(np.flatnonzero(ok == 0).tolist()) == sorted(victims)
    np.testing.assert_array_equal(_walk(bad, wbuf), offs)
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, bad), wbuf)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), offs)
    assert nbad == len(victims) and sorted(np.flatnonzero(got_ok.cpu().numpy() == 0).tolist()) == sorted(victims)


def _walk(buf, wbuf):
    """storage_compact_readback's walk (storage.c:950-1070), one read per wbuf."""
    offs = []
    for start in range(0, buf.size, wbuf):
        size, off = min(wbuf, buf.size - start), 0
        while off + 48 <= size and buf[start + off + 41] != 0:
            offs.append(start + off)
            off += layout.ntotal_of(buf, start + off) & 0xffffffff  # (unsigned int ntotal, storage.c:954)
    return np.asarray(offs, np.uint64)


def test_verify_pages_device_walk(torch):
    """Pages walked on the device: same items as the reference walk, every
    stored CRC checked, corrupted items (and a zeroed nkey, which ends its
    wbuf's walk early) reported exactly."""
    rng = np.random.default_rng(38)
    items = [layout.make_item(b"pg%06d" % i, rng.integers(0, 256, int(rng.integers(0, 20000)), dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(1500)]
    wbuf = 1 << 20
    buf, offs = layout.pack_wbufs(items, wbuf)
    ok, nbad = mc.stamp_items(buf, offs, region_bytes=wbuf)
    assert nbad == 0
    np.testing.assert_array_equal(_walk(buf, wbuf), offs)
    for dev in (True, False):
        got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf) if dev else buf, wbuf)
        got_offs = got_offs.cpu().numpy().astype(np.uint64) if dev else got_offs
        got_ok = got_ok.cpu().numpy() if dev else got_ok
        np.testing.assert_array_equal(got_offs, offs)
        assert nbad == 0 and got_ok.all()
    victims = [3, 700, 1499]
    for v in victims:
        o = int(offs[v])
        buf[o + 32 + int(rng.integers(16, layout.ntotal_of(buf, o) - 32))] ^= 0x40
    buf[int(offs[900]) + 41] = 0  # nkey == 0: the walk of this wbuf ends here
    want = _walk(buf, wbuf)
    assert want.size < offs.size
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), wbuf)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), want)
    bad_offs = sorted(int(x) for x in got_offs.cpu().numpy()[got_ok.cpu().numpy() == 0])
    assert bad_offs == sorted(int(offs[v]) for v in victims if int(offs[v]) in set(want.tolist()))
    assert nbad == len(bad_offs)


def test_verify_pages_walk_stride_runs(torch):
    """The device walk fetches several headers per round trip at the last
    item's stride: runs of equal-sized items broken by other sizes, a header
    whose nbytes was flipped (the walk diverges from the packed offsets), a
    zeroed nkey mid-run, wbufs ending a few bytes after an item, a partial last
    wbuf, and more than 2048 equal items per wbuf (the overflow re-walk) -- all
    give exactly the sequential walk of storage.c:950-1070."""
    rng = np.random.default_rng(43)
    sizes = []
    while len(sizes) < 6000:
        run = int(rng.integers(1, 40))
        sizes += [int(rng.choice([0, 1, 7, 100, 4096, 4097]))] * run
    items = [layout.make_item(b"r%06d" % i, rng.integers(0, 256, n, dtype=np.uint8).tobytes(), cas=i + 1)
             for i, n in enumerate(sizes)]
    for wbuf in (1 << 20, 4165 * 9 + 47, 4165 * 9 + 48):
        buf, offs = layout.pack_wbufs(items, wbuf)
        buf = buf[:buf.size - wbuf // 3]  # partial last wbuf
        want = _walk(buf, wbuf)
        got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), wbuf)
        np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), want)
    buf, offs = layout.pack_wbufs(items, 1 << 20)
    ok, nbad = mc.stamp_items(buf, offs, region_bytes=1 << 20)
    assert nbad == 0
    buf[int(offs[1234]) + 33] ^= 0x01  # nbytes + 256: the walk leaves the packed offsets
    buf[int(offs[3000]) + 41] = 0      # nkey == 0 mid-run
    want = _walk(buf, 1 << 20)
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), 1 << 20)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), want)
    # > 2048 equal items per wbuf
    small = [layout.make_item(b"e%06d" % i, b"x" * 5, cas=i + 1) for i in range(12000)]
    buf, offs = layout.pack_wbufs(small, 256 << 10)
    assert np.bincount((offs // (256 << 10)).astype(np.int64)).max() > 2048
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), 256 << 10)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), offs)
    assert nbad == int((got_ok.cpu().numpy() == 0).sum())


def test_verify_pages_walk_wave_runs(torch):
    """The walk reads 64 guessed headers per round trip (one wave per wbuf):
    runs of equal items just under, at and over the wave width, wbufs that end
    inside or right after a run, and corrupt sizes mid-run walk exactly as
    storage.c:950-1070 (tests/test_walk_model.py restates the round trip)."""
    rng = np.random.default_rng(44)
    sizes = []
    for run in (63, 64, 65, 1, 128, 129, 127, 2, 300, 64, 64, 5):
        sizes += [int(rng.choice([0, 3, 100, 4096]))] * run
    items = [layout.make_item(b"v%06d" % i, rng.integers(0, 256, n, dtype=np.uint8).tobytes(), cas=i + 1)
             for i, n in enumerate(sizes)]
    for wbuf in (1 << 20, 4165 * 64 + 47, 4165 * 64 + 48, 4165 * 128):
        buf, offs = layout.pack_wbufs(items, wbuf)
        want = _walk(buf, wbuf)
        np.testing.assert_array_equal(want, offs)
        for flip in (None, 33, 35, 41):
            b = buf.copy()
            if flip is not None:
                b[int(offs[int(rng.integers(0, offs.size))]) + flip] ^= np.uint8(0x80 if flip == 35 else 0x01)
            got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, b), wbuf)
            np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), _walk(b, wbuf))


def _walk_np(buf, wbuf):
    """_walk with every wbuf walked in lockstep (numpy over the wbufs): the
    same items in the same order, fast enough for hundreds of pages."""
    nw = -(-buf.size // wbuf)
    start = np.arange(nw, dtype=np.int64) * wbuf
    size = np.minimum(wbuf, buf.size - start)
    off = np.zeros(nw, np.int64)
    live = np.ones(nw, bool)
    ws, os_ = [], []
    while live.any():
        live &= off + 48 <= size
        at = start + np.where(live, off, 0)
        live &= buf[at + 41] != 0
        ws.append(np.nonzero(live)[0])
        os_.append(at[live])
        nbytes = (buf[at + 32].astype(np.int64) | buf[at + 33].astype(np.int64) << 8 |
                  buf[at + 34].astype(np.int64) << 16 | buf[at + 35].astype(np.int64) << 24)
        flags = buf[at + 38].astype(np.int64) | buf[at + 39].astype(np.int64) << 8
        nt = (49 + buf[at + 41].astype(np.int64) + nbytes + np.where(flags & 256, 4, 0) +
              np.where(flags & 2, 8, 0)) & 0xffffffff  # (unsigned int ntotal, storage.c:954)
        off = np.where(live, off + nt, off)
    w, o = np.concatenate(ws), np.concatenate(os_)
    return o[np.lexsort((o, w))].astype(np.uint64)


@pytest.mark.parametrize("pages", [4, 300])
def test_verify_pages_bench_layout(torch, span_path, pages):
    """The bench's config-5 pages (1007 packed 4165-B images per 4 MiB wbuf,
    1 % single-bit flips) plus flipped header bits (nbytes, it_flags, nkey) in
    40 images: the planned device walk + verify gives the sequential walk's
    items and (4 pages) the oracle's verdicts, leaves the pages untouched, and
    gives the same answer when repeated.  (300 pages, 4800 walking waves: a
    walk whose state went wrong under load did so only on large page sets --
    DESIGN.md section 3.)"""
    import argparse
    import bench
    if span_path == "small" and pages > 4:
        pytest.skip("the planned path only (pages >> the small-batch bound)")
    bench.workload_config5(argparse.Namespace(pages=pages), 0, 1)
    data = bench._KEEP[-2]
    rng = np.random.default_rng(45)
    items = rng.choice(pages * 16 * 1007, 40, replace=False)
    pos = [int(i // 1007) * (4 << 20) + int(i % 1007) * 4165 + int(rng.choice([32, 33, 34, 35, 38, 39, 41]))
           for i in items]
    flip = torch.tensor([1 << int(rng.integers(0, 8)) for _ in pos], dtype=torch.uint8, device="cuda")
    data[torch.tensor(pos, device="cuda")] ^= flip
    buf = data.cpu().numpy()
    want = _walk_np(buf, 4 << 20)
    if pages == 4:
        np.testing.assert_array_equal(want, _walk(buf, 4 << 20))
    keep = data.clone()
    for rep in range(2):
        got_offs, got_ok, nbad = mc.verify_pages(data, 4 << 20)
        np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), want)
    assert torch.equal(data, keep)
    del data, keep
    bench._KEEP.clear()
    if pages > 4:
        # every verdict of the 4.8 M items against the oracle (vectorised
        # headers, the spans' CRCs in eight threads)
        o = want.astype(np.int64)
        u32 = lambda at: (buf[at].astype(np.uint64) | buf[at + 1].astype(np.uint64) << 8 |
                          buf[at + 2].astype(np.uint64) << 16 | buf[at + 3].astype(np.uint64) << 24)
        nbytes, flags, nkey = u32(o + 32), buf[o + 38].astype(np.uint64) | buf[o + 39].astype(np.uint64) << 8, \
            buf[o + 41].astype(np.uint64)
        nt = 49 + nkey + nbytes + np.where(flags & 256, 4, 0) + np.where(flags & 2, 8, 0)
        wb = 4 << 20
        sane = (nkey != 0) & (nbytes < 1 << 31) & (o + nt <= buf.size) & (o // wb == (o + nt - 1) // wb)
        idx = np.flatnonzero(sane)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(8) as ex:
            crcs = np.concatenate(list(ex.map(
                lambda ix: oracle.batch(buf, (o[ix] + 32).astype(np.uint64), (nt[ix] - 32).astype(np.uint64)),
                np.array_split(idx, 8))))
        good = np.zeros(o.size, bool)
        good[idx] = crcs == u32(o[idx] + 28).astype(np.uint32)
        np.testing.assert_array_equal(got_ok.cpu().numpy().astype(bool), good)
        assert nbad == o.size - int(good.sum())
        return
    # the verdicts: the stored CRC of every item whose span is sane
    spans_ok = []
    for o in want:
        o = int(o)
        nt = layout.ntotal_of(buf, o) & 0xffffffff
        sane = buf[o + 41] != 0 and o + nt <= buf.size and o // (4 << 20) == (o + nt - 1) // (4 << 20)
        spans_ok.append(bool(sane) and oracle.crc32c(0, buf[o + 32:o + nt]) ==
                        int(buf[o + 28:o + 32].view(np.uint32)[0]))
    np.testing.assert_array_equal(got_ok.cpu().numpy().astype(bool), np.array(spans_ok))
    assert nbad == len(spans_ok) - int(np.sum(spans_ok))


def test_config3_full_size(torch, span_path):
    """BASELINE config 3 at full size through the bench's own generator (1 Mi
    Zipf spans of 64 B - 1 MiB at odd offsets, 28.5 GB): two runs agree on
    every span, and every span matches the oracle (run over the host copy in
    eight threads)."""
    import argparse
    import ctypes
    import bench
    if span_path == "small":
        pytest.skip("a planned batch (1 Mi spans)")
    spans, nbytes, _ = bench.workload_config3(argparse.Namespace(items=1 << 20), 0, 1)
    data, d_offs, d_lens, out = bench._KEEP[-4:]
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(spans), _lib.CRC32C_DEVICE, None))
    torch.cuda.synchronize()
    first = out.clone()
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(spans), _lib.CRC32C_DEVICE, None))
    torch.cuda.synchronize()
    assert torch.equal(first, out)
    offs, lens = d_offs.cpu().numpy().view(np.uint64), d_lens.cpu().numpy().view(np.uint32)
    host = data.cpu().numpy()
    from concurrent.futures import ThreadPoolExecutor
    parts = np.array_split(np.arange(lens.size), 8)
    with ThreadPoolExecutor(8) as ex:  # (the oracle's C call releases the GIL)
        want = np.concatenate(list(ex.map(lambda ix: oracle.batch(host, offs[ix], lens[ix].astype(np.uint64)), parts)))
    got = _u32(out)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:10], lens[bad[:10]])
    del data, d_offs, d_lens, out, first, host
    bench._KEEP.clear()


def test_planned_rounds_past_16_gib(torch, span_path):
    """The balanced plan's rounds (crc32c_shim.hip plan_rounds: one per 8 GiB
    of the batch's buffer, k_spans restarting every group's pipeline per
    round) on a 17 GiB device buffer: 3 rounds, each cutting its third of the
    plan's blocks (span order) into one share per span-kernel group.  Spans
    sorted by offset over the whole buffer, some straddling the 8 and 16 GiB
    marks, several MiB long ones among them: MODE 0 CRCs with and without
    crc_in against the oracle.  Then 1 MiB wbufs of item images placed on
    both sides of those marks and elsewhere: the device stamp (MODE 2) equals
    the oracle's, the stamped images verify clean (MODE 1), and damaged ones
    are reported exactly."""
    if span_path == "small":
        pytest.skip("a planned batch (the small path has no rounds)")
    GiB, MiB = 1 << 30, 1 << 20
    size = 17 * GiB
    if torch.cuda.mem_get_info()[0] < size + 8 * GiB:
        pytest.skip("needs about 25 GiB of free device memory")
    rng = np.random.default_rng(1717)
    data = torch.empty(size, dtype=torch.uint8, device="cuda")
    gen = torch.Generator(device="cuda")
    gen.manual_seed(17)
    for c in range(0, size, GiB):
        data[c:c + GiB] = torch.randint(0, 256, (GiB,), dtype=torch.uint8, device="cuda", generator=gen)
    # spans: log-uniform 1 B - 1 MiB over the buffer, 100 across each mark, 12 of 2-6 MiB
    n = 6000
    lens = np.exp(rng.uniform(0, np.log(MiB), n)).astype(np.uint64)
    lens[:12] = rng.integers(2 * MiB, 6 * MiB, 12)
    offs = rng.integers(0, size - 8 * MiB, n).astype(np.uint64)
    for k, mark in enumerate((8 * GiB, 16 * GiB)):
        ix = np.arange(100 + 100 * k, 200 + 100 * k)
        lens[ix] = np.maximum(lens[ix], 4096)
        offs[ix] = mark - 1 - rng.integers(0, 2 ** 40, ix.size).astype(np.uint64) % (lens[ix] - 1)
    order = np.argsort(offs, kind="stable")
    offs, lens = offs[order], lens[order]
    assert ((offs < 8 * GiB) & (offs + lens > 8 * GiB)).sum() >= 90
    assert ((offs < 16 * GiB) & (offs + lens > 16 * GiB)).sum() >= 90
    # the oracle over the spans' bytes, gathered on the device and copied once
    cat = torch.cat([data[int(o):int(o + l)] for o, l in zip(offs, lens)]).cpu().numpy()
    coffs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    cin = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    d_offs, d_lens = _dev(torch, offs.view(np.int64)), _dev(torch, lens.astype(np.uint32).view(np.int32))
    for c in (None, cin):
        got = mc.batch(data, offsets=d_offs, lens=d_lens, crc_in=None if c is None else _dev(torch, c.view(np.int32)))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_u32(got), oracle.batch(cat, coffs, lens, c))
    del cat
    # item images: 1 MiB wbufs at MiB-aligned places around both marks and spread over the buffer
    items = [layout.make_item(b"rd%06d" % i, rng.integers(0, 256, int(np.exp(rng.uniform(np.log(10), np.log(300000)))),
                                                          dtype=np.uint8).tobytes(), cas=i + 1) for i in range(2500)]
    hb, loc = layout.pack_wbufs(items, MiB)
    nw = hb.size // MiB
    near = [8 * GiB + (j - 12) * MiB for j in range(24)] + [16 * GiB + (j - 12) * MiB for j in range(24)]
    spread = sorted(set(int(x) * MiB for x in rng.integers(0, size // MiB - 1, 4 * nw)) - set(near))
    pos = np.asarray((near + spread[:max(0, nw - len(near))])[:nw], np.uint64)
    assert pos.size == nw
    for j in range(nw):
        data[int(pos[j]):int(pos[j]) + MiB] = torch.from_numpy(hb[j * MiB:(j + 1) * MiB]).cuda()
    ioffs = pos[(loc // MiB).astype(np.int64)] + loc % MiB
    want = hb.copy()
    so, sl = layout.spans_of(hb, loc)
    layout.store_crcs(want, loc, oracle.batch(hb, so, sl))
    d_ioffs = _dev(torch, ioffs.view(np.int64))
    ok, nbad = mc.stamp_items(data, d_ioffs, region_bytes=MiB)
    assert nbad == 0 and ok.cpu().numpy().all()
    back = torch.cat([data[int(p):int(p) + MiB] for p in pos]).cpu().numpy()
    np.testing.assert_array_equal(back, want)
    ok, nbad = mc.verify_items(data, d_ioffs, region_bytes=MiB)
    assert nbad == 0 and ok.cpu().numpy().all()
    victims = sorted({int(np.argmax(ioffs > 8 * GiB)), int(np.argmax(ioffs > 16 * GiB)) - 1, loc.size - 1})
    for v in victims:
        o = int(ioffs[v])
        data[o + 60] ^= 0x04
    ok, nbad = mc.verify_items(data, d_ioffs, region_bytes=MiB)
    assert nbad == len(victims) and np.flatnonzero(ok.cpu().numpy() == 0).tolist() == victims
    del data


@pytest.mark.parametrize("wbuf", [61, 64, 100, 127, 4099])
def test_verify_pages_tiny_wbufs(torch, wbuf):
    """wbufs barely larger than one image (one item each, 48-B tail rule at
    the edge), a buffer that ends inside a wbuf, and buffers shorter than a
    header: the device walk and verify give the sequential walk's items."""
    rng = np.random.default_rng(wbuf)
    items = [layout.make_item(b"k", rng.integers(0, 256, int(rng.integers(0, 3)), dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(3000)]
    items = [it for it in items if len(it) <= wbuf]
    buf, offs = layout.pack_wbufs(items, wbuf)
    ok, nbad = mc.stamp_items(buf, offs, region_bytes=wbuf)
    assert nbad == 0
    for cut in (0, wbuf // 2, buf.size - 47, buf.size - 1):
        b = buf[:buf.size - cut] if cut < buf.size else buf[:1]
        want = _walk(b, wbuf)
        got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, b), wbuf)
        np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), want)
        assert nbad == int((got_ok.cpu().numpy() == 0).sum())


@pytest.mark.parametrize("wbuf", [8 << 10, 16 << 10])
def test_verify_pages_k5_small_wbufs_walked_twice(torch, wbuf):
    """K5-shaped images (4165 B) in wbufs of one to three images, 4200 of
    them: 8 KiB wbufs keep no walk slots (the emit pass walks every wbuf
    again), 16 KiB wbufs keep 8 each; both give the sequential walk's items
    and the oracle's verdicts, with 1 % of the images corrupted."""
    rng = np.random.default_rng(wbuf)
    items = [layout.make_item(b"key%07d" % i, rng.integers(0, 256, 4096, dtype=np.uint8).tobytes(), cas=i + 1)
             for i in range(4200)]
    buf, offs = layout.pack_wbufs(items, wbuf)
    ok, nbad = mc.stamp_items(buf, offs, region_bytes=wbuf)
    assert nbad == 0
    bad = rng.choice(offs.size, 42, replace=False)
    for i in bad:
        buf[int(offs[i]) + 100 + int(rng.integers(0, 3000))] ^= 1 << int(rng.integers(0, 8))
    want = _walk(buf, wbuf)
    np.testing.assert_array_equal(want, offs)
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), wbuf)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), want)
    expect = np.ones(offs.size, bool)
    expect[bad] = False
    np.testing.assert_array_equal(got_ok.cpu().numpy().astype(bool), expect)
    assert nbad == bad.size


def test_verify_pages_slot_boundary(torch):
    """64 KiB wbufs keep 32 walk slots: wbufs of 31, 32 and 33 items (and an
    empty one and one of a single item), verified as a planned batch (fewer
    than 4096 items: the emit pass copies the slots of the wbufs that fit
    and walks the 33-item wbuf again, k_count reads every header): the
    sequential walk's offsets and the oracle's verdicts, with damaged items
    on both sides of the boundary."""
    rng = np.random.default_rng(57)
    wbuf = 64 << 10
    parts, offs = [], []
    for w, n in enumerate([31, 32, 33, 0, 1, 32, 33]):
        items = [layout.make_item(b"s%02d%05d" % (w, i), rng.integers(0, 256, 1800, dtype=np.uint8).tobytes(),
                                  cas=w * 100 + i + 1) for i in range(n)]
        b, o = layout.pack_wbufs(items, wbuf) if items else (np.zeros(wbuf, np.uint8), np.zeros(0, np.uint64))
        assert b.size == wbuf  # (one wbuf each)
        parts.append(b)
        offs.append(o + np.uint64(w * wbuf))
    buf, offs = np.concatenate(parts), np.concatenate(offs)
    ok, nbad = mc.stamp_items(buf, offs, region_bytes=wbuf)
    assert nbad == 0
    first = np.searchsorted(offs, np.arange(7, dtype=np.uint64) * wbuf)  # each wbuf's first item
    # the last item of the 31-item wbuf, the first and last (32nd) of the 32-item
    # one, the first, 32nd and 33rd of the 33-item one, the single item, the last
    # item of the pages
    victims = [int(first[1]) - 1, int(first[1]), int(first[2]) - 1, int(first[2]), int(first[2]) + 31,
               int(first[3]) - 1, int(first[4]), offs.size - 1]
    for v in victims:
        buf[int(offs[v]) + 200] ^= 0x10
    np.testing.assert_array_equal(_walk(buf, wbuf), offs)
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), wbuf)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), offs)
    expect = np.ones(offs.size, np.uint8)
    expect[victims] = 0
    np.testing.assert_array_equal(got_ok.cpu().numpy(), expect)
    assert nbad == len(victims)


def test_chained_iovs(torch):
    """Chunked items (storage.c:163-170): the CRC chained over an item's iovs
    (header from +32, then each chunk) equals crc32c(0, concatenation)."""
    rng = np.random.default_rng(39)
    buf = rng.integers(0, 256, 6 << 20, dtype=np.uint8)
    nch = 120
    counts = rng.integers(1, 12, nch)
    counts[:3] = [1, 2, 40]
    n = int(counts.sum())
    lens = rng.integers(0, 600000, n).astype(np.uint32)
    lens[:5] = [0, 3, 17, 524288, 1]
    offs = rng.integers(0, buf.size - 600000, n).astype(np.uint64)
    first = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    want = np.empty(nch, np.uint32)
    for c in range(nch):
        parts = [buf[int(o):int(o) + int(l)] for o, l in zip(offs[first[c]:first[c + 1]], lens[first[c]:first[c + 1]])]
        cat = np.concatenate(parts) if parts else np.empty(0, np.uint8)
        want[c] = oracle.batch(cat, np.zeros(1, np.uint64), np.array([cat.size]))[0]
    got = mc.batch_chains(_dev(torch, buf), _dev(torch, offs.view(np.int64)), _dev(torch, lens.view(np.int32)),
                          _dev(torch, first.view(np.int64)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(got), want)
    # host path, iovs in chain order (not memory order), several pipeline slots
    np.testing.assert_array_equal(mc.batch_chains(buf, offs, lens, first), want)
    # and over sorted iovs
    offs_s = np.sort(offs)
    want_s = np.empty(nch, np.uint32)
    for c in range(nch):
        sl = slice(int(first[c]), int(first[c + 1]))
        cat = np.concatenate([buf[int(o):int(o) + int(l)] for o, l in zip(offs_s[sl], lens[sl])])
        want_s[c] = oracle.batch(cat, np.zeros(1, np.uint64), np.array([cat.size]))[0]
    np.testing.assert_array_equal(mc.batch_chains(buf, offs_s, lens, first), want_s)


def test_pinned_host_alloc():
    """crc32c_host_alloc buffers (pinned wbufs) take the host path with no
    staging copy and give the same CRCs."""
    import ctypes
    nbytes = 3 << 20
    p = _lib.lib.crc32c_host_alloc(nbytes)
    assert p
    try:
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        arr[:] = np.random.default_rng(40).integers(0, 256, nbytes, dtype=np.uint8)
        offs = np.arange(0, nbytes - 5000, 4165, dtype=np.uint64) + 32
        lens = np.full(offs.size, 4133, np.uint32)
        np.testing.assert_array_equal(mc.batch(arr, offsets=offs, lens=lens), oracle.batch(arr, offs, lens))
    finally:
        _lib.lib.crc32c_host_free(p)


def test_verify_pages_many_small_items(torch):
    """More items per wbuf than the walk keeps per pass (2048): the overflow
    re-walk places the rest."""
    rng = np.random.default_rng(41)
    items = [layout.make_item(b"s%05d" % i, rng.integers(0, 256, int(rng.integers(0, 24)), dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(9000)]
    wbuf = 256 << 10
    buf, offs = layout.pack_wbufs(items, wbuf)
    assert np.bincount((offs // wbuf).astype(np.int64)).max() > 2048
    ok, nbad = mc.stamp_items(buf, offs, region_bytes=wbuf)
    assert nbad == 0
    buf[int(offs[5000]) + 40] ^= 1  # nkey byte is 41: flip a header byte inside the span instead
    got_offs, got_ok, nbad = mc.verify_pages(_dev(torch, buf), wbuf)
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), offs)
    assert nbad == 1 and got_ok.cpu().numpy()[5000] == 0


def test_concurrent_streams_share_plan_buffers(torch):
    """Two host threads enqueue planned (multi-segment) batches on two streams
    at once: the plan buffers are handed over in stream order, results exact."""
    import threading
    rng = np.random.default_rng(42)
    jobs = []
    for t in range(2):
        lens = rng.integers(0, 400000, 300).astype(np.uint32)
        offs = np.concatenate([[5], 5 + np.cumsum(lens[:-1].astype(np.uint64) + 3)]).astype(np.uint64)
        host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 16), dtype=np.uint8)
        jobs.append((host, offs, lens, oracle.batch(host, offs, lens)))
    errors = []

    def worker(t):
        try:
            host, offs, lens, want = jobs[t]
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                d = _dev(torch, host)
                do, dl = _dev(torch, offs.view(np.int64)), _dev(torch, lens.view(np.int32))
                for _ in range(10):
                    out = mc.batch(d, offsets=do, lens=dl, asynchronous=True)
                st.synchronize()
                got = _u32(out)
            if not np.array_equal(got, want):
                errors.append(f"thread {t}: {int((got != want).sum())} mismatches")
        except Exception as e:  # noqa: BLE001
            errors.append(f"thread {t}: {e!r}")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


def test_realistic_item_spans_4133(torch):
    """config-1/config-5 geometry: 4133-byte spans at +32 of 4165-byte images."""
    items = [layout.make_item(b"key%07d" % i, np.random.default_rng(i).integers(0, 256, 4096, dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(700)]
    buf, offs = layout.pack_wbufs(items, 1 << 20)
    soffs, slens = layout.spans_of(buf, offs)
    assert (slens == 4133).all()
    want = oracle.batch(buf, soffs, slens)
    d = _dev(torch, buf)
    out = mc.batch(d, offsets=_dev(torch, soffs.view(np.int64)), lens=_dev(torch, slens.astype(np.uint32).view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


def test_offsets_with_fixed_length(torch):
    """offsets[] given, lens[] absent: every span is `len` bytes (config 5 shape)."""
    import ctypes
    rng = np.random.default_rng(21)
    n, L = 1500, 4133
    offs = (np.arange(n, dtype=np.uint64) * 4165 + 32).astype(np.uint64)
    host = rng.integers(0, 256, n * 4165 + 64, dtype=np.uint8)
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d, doffs = _dev(torch, host), _dev(torch, offs.view(np.int64))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for crc_in in (None, _dev(torch, cin.view(np.int32))):
        s = _lib.Spans(d.data_ptr(), host.size, doffs.data_ptr(), 0, None, L,
                       None if crc_in is None else crc_in.data_ptr(), out.data_ptr(), n)
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
        want = oracle.batch(host, offs, np.full(n, L), None if crc_in is None else cin)
        np.testing.assert_array_equal(_u32(out), want)
    # and the host path with the same descriptor shape
    outh = np.empty(n, np.uint32)
    s = _lib.Spans(host.ctypes.data, host.size, offs.ctypes.data, 0, None, L, None, outh.ctypes.data, n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), 0, None))
    np.testing.assert_array_equal(outh, oracle.batch(host, offs, np.full(n, L)))


@pytest.mark.parametrize("L", [1, 15, 100, 896, 897, 898, 1008, 1009, 1010, 1024, 1040, 4080, 4097, 4200, 4209, 4224,
                               4225, 4240, 5104, 5125, 8195, 65536, 65552])
def test_fixed_length_head_fragment_thresholds(torch, L):
    """offsets[] with one shared length (one unit per span, no plan) at the
    lengths where the head fragment moves between the span kernel and the
    span's thread (kFragMax = 128; whole spans up to kWholeMax = 1024) or the
    span skips the kernel entirely."""
    import ctypes
    rng = np.random.default_rng(L)
    n = 700
    size = n * (L + 40) + 64
    host = rng.integers(0, 256, size, dtype=np.uint8)
    offs = np.sort(rng.integers(0, size - L, n)).astype(np.uint64)
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d, doffs, dcin = _dev(torch, host), _dev(torch, offs.view(np.int64)), _dev(torch, cin.view(np.int32))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = _lib.Spans(d.data_ptr(), host.size, doffs.data_ptr(), 0, None, L, dcin.data_ptr(), out.data_ptr(), n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
    np.testing.assert_array_equal(_u32(out), oracle.batch(host, offs, np.full(n, L), cin))


@pytest.mark.parametrize("name", ["cfg1", "varied"])
def test_verify_golden_items(torch, name):
    g = np.load(os.path.join(GOLD, "items.npz"))
    buf, offs = g[f"{name}_buf"].copy(), g[f"{name}_offsets"]
    ok, nbad = mc.verify_items(_dev(torch, buf), _dev(torch, offs.view(np.int64)))
    assert nbad == 0 and ok.cpu().numpy().all()
    ok, nbad = mc.verify_items(buf, offs)  # host path
    assert nbad == 0 and ok.all()
    # flip one bit in 3 items: exactly those fail (the reference has no such test)
    rng = np.random.default_rng(11)
    victims = rng.choice(offs.size, 3, replace=False)
    for v in victims:
        o = int(offs[v])
        buf[o + 32 + int(rng.integers(0, layout.ntotal_of(buf, o) - 32))] ^= 1 << int(rng.integers(0, 8))
    ok, nbad = mc.verify_items(buf, offs)
    assert nbad == 3
    assert sorted(np.flatnonzero(ok == 0).tolist()) == sorted(victims.tolist())


def test_empty_batch_and_zero_lengths(torch):
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    out = mc.batch(d, offsets=torch.zeros(0, dtype=torch.int64, device="cuda"),
                   lens=torch.zeros(0, dtype=torch.int32, device="cuda"))
    assert out.numel() == 0
    cin = np.array([0, 1, 0xFFFFFFFF, 0x12345678], np.uint32)
    out = mc.batch(d, offsets=torch.tensor([0, 5, 17, 63], device="cuda"),
                   lens=torch.zeros(4, dtype=torch.int32, device="cuda"),
                   crc_in=_dev(torch, cin.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), cin)  # crc32c(c, "", 0) == c


def test_full_size_config2(torch):
    """BASELINE config 2 at full size: 1 M x 4 KiB, every CRC checked."""
    n, L = 1 << 20, 4096
    g = torch.Generator(device="cuda").manual_seed(42)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    import ctypes
    s = _lib.Spans(d.data_ptr(), n * L, None, L, None, L, None, out.data_ptr(), n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
    host = d.cpu().numpy()
    want = oracle.batch(host, np.arange(n, dtype=np.uint64) * L, np.full(n, L))
    np.testing.assert_array_equal(_u32(out), want)


def test_async_submit_wait():
    import ctypes
    rng = np.random.default_rng(9)
    host = rng.integers(0, 256, 1 << 22, dtype=np.uint8)
    offs = np.arange(0, host.size - 5000, 5000, dtype=np.uint64) + 1
    lens = np.full(offs.size, 4999, np.uint32)
    out = np.empty(offs.size, np.uint32)
    s = _lib.Spans(host.ctypes.data, host.size, offs.ctypes.data, 0, lens.ctypes.data, 0, None, out.ctypes.data,
                   offs.size)
    job = ctypes.c_void_p()
    _lib.check(_lib.lib.crc32c_batch_submit(ctypes.byref(s), 0, ctypes.byref(job)))
    _lib.check(_lib.lib.crc32c_batch_wait(job))
    np.testing.assert_array_equal(out, oracle.batch(host, offs, lens))


def _mixed_page(rng, n_items, wbuf, max_value):
    items = [layout.make_item(b"m%06d" % i, rng.integers(0, 256, int(rng.integers(0, max_value)),
                                                         dtype=np.uint8).tobytes(), cas=i + 1)
             for i in range(n_items)]
    buf, offs = layout.pack_wbufs(items, wbuf)
    soffs, slens = layout.spans_of(buf, offs)
    layout.store_crcs(buf, offs, oracle.batch(buf, soffs, slens))
    return buf, offs


def test_verify_4165_items_with_corrupt_lengths(torch):
    """The config-5 shape: packed 4165-B images (one 4 KiB block each after
    the head fragment, k_blocks), a few with a flipped bit in nbytes (their
    spans leave the one-block shape, or the wbuf: the span kernel, or not
    sane) and a few with a flipped data bit.  Exactly the corrupted images
    fail, through both kernels in one call; a stamp then repairs the data
    flips in place."""
    rng = np.random.default_rng(4165)
    n = 3000
    items = [layout.make_item(b"key%07d" % i, rng.integers(0, 256, 4096, dtype=np.uint8).tobytes(), cas=i + 1)
             for i in range(n)]
    assert len(items[0]) == 4165
    buf, offs = layout.pack_wbufs(items, 1 << 20)
    soffs, slens = layout.spans_of(buf, offs)
    layout.store_crcs(buf, offs, oracle.batch(buf, soffs, slens))
    victims = rng.choice(n, 60, replace=False)
    hdr, data = victims[:30], victims[30:]
    for v in hdr:  # nbytes (bytes 32..35): a length bit
        buf[int(offs[v]) + 32 + int(rng.integers(0, 2))] ^= 1 << int(rng.integers(0, 8))
    for v in data:
        buf[int(soffs[v] + rng.integers(16, slens[v]))] ^= 1 << int(rng.integers(0, 8))
    ok, nbad = mc.verify_items(_dev(torch, buf), _dev(torch, offs.view(np.int64)), region_bytes=1 << 20)
    want = np.ones(n, np.uint8)
    want[victims] = 0
    assert nbad == victims.size
    np.testing.assert_array_equal(ok.cpu().numpy(), want)


@pytest.mark.parametrize("max_value", [24, 700, 9000])
def test_page_stream_tiny_to_large_items(torch, max_value):
    """Item images from ~52 B (more than 32 spans per 4 KiB block) to ~9 KB,
    verified and stamped through the page stream; flipped bits found exactly."""
    rng = np.random.default_rng(max_value)
    buf, offs = _mixed_page(rng, 3000, 1 << 20, max_value)
    d = _dev(torch, buf)
    ok, nbad = mc.verify_items(d, _dev(torch, offs.view(np.int64)), region_bytes=1 << 20)
    assert nbad == 0 and ok.cpu().numpy().all()
    victims = rng.choice(offs.size, 40, replace=False)
    soffs, slens = layout.spans_of(buf, offs)
    for v in victims:  # (past the header fields, so every span keeps its length)
        buf[int(soffs[v] + rng.integers(16, slens[v]))] ^= 1 << int(rng.integers(0, 8))
    ok, nbad = mc.verify_items(_dev(torch, buf), _dev(torch, offs.view(np.int64)), region_bytes=1 << 20)
    want = np.ones(offs.size, np.uint8)
    want[victims] = 0
    assert nbad == victims.size
    np.testing.assert_array_equal(ok.cpu().numpy(), want)
    # stamp restores every CRC in place; the stamped buffer then verifies clean
    d = _dev(torch, buf)
    ok, nbad = mc.stamp_items(d, _dev(torch, offs.view(np.int64)), region_bytes=1 << 20)
    assert nbad == 0 and ok.cpu().numpy().all()
    stamped = d.cpu().numpy()
    want_crc = oracle.batch(stamped, soffs, slens)
    got_crc = np.array([int.from_bytes(stamped[int(o) + 28:int(o) + 32].tobytes(), "little") for o in offs],
                       np.uint32)
    np.testing.assert_array_equal(got_crc, want_crc)


def test_page_stream_unsorted_offsets_bad_headers_and_tail(torch):
    """Shuffled offsets, duplicated items, malformed headers and a buffer that
    ends inside a 4 KiB block: the spans that cannot join the stream go
    through the per-span kernel, the results are the oracle's."""
    rng = np.random.default_rng(77)
    buf, offs = _mixed_page(rng, 700, 1 << 20, 3000)
    soffs, slens = layout.spans_of(buf, offs)
    end = int(soffs[-1] + slens[-1])
    buf = buf[: end + 5].copy()  # not a multiple of 4096: the last items are past the whole blocks
    bad_hdr = rng.choice(offs.size, 7, replace=False)
    for v in bad_hdr:
        buf[int(offs[v]) + layout.NKEY_OFF] = 0  # nkey 0: malformed
    flipped = np.setdiff1d(rng.choice(offs.size, 11, replace=False), bad_hdr)
    for v in flipped:
        buf[int(soffs[v] + slens[v] // 2)] ^= 0x10
    order = rng.permutation(offs.size)
    q = np.concatenate([offs[order], offs[order[:25]]])  # and 25 items listed twice
    want = np.ones(offs.size, np.uint8)
    want[bad_hdr] = 0
    want[flipped] = 0
    want_q = want[np.concatenate([order, order[:25]])]
    ok, nbad = mc.verify_items(_dev(torch, buf), _dev(torch, q.view(np.int64)))
    np.testing.assert_array_equal(ok.cpu().numpy(), want_q)
    assert nbad == int((want_q == 0).sum())


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_spans(torch, seed):
    """Seeded fuzz of crc32c_batch: random (possibly overlapping) offsets, a
    mix of tiny, ~4 KiB, multi-block and multi-segment lengths, random crc_in
    or none, random base misalignment; compared with the oracle."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 1500))
    kind = rng.integers(0, 4, n)
    lens = np.where(kind == 0, rng.integers(0, 64, n),
                    np.where(kind == 1, rng.integers(4000, 4300, n),
                             np.where(kind == 2, rng.integers(0, 20000, n), rng.integers(60000, 300000, n))))
    lens = lens.astype(np.uint32)
    size = int(lens.max()) + int(rng.integers(1, 1 << 20))
    host = rng.integers(0, 256, size + 64, dtype=np.uint8)
    offs = np.array([rng.integers(0, size - int(l) + 1) for l in lens], dtype=np.uint64)
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if seed % 2 else None
    want = oracle.batch(host, offs, lens, cin)
    d = _dev(torch, host)
    out = mc.batch(d, offsets=_dev(torch, offs.view(np.int64)), lens=_dev(torch, lens.view(np.int32)),
                   crc_in=None if cin is None else _dev(torch, cin.view(np.int32)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u32(out), want)


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_k1_fixed(torch, seed):
    """Seeded fuzz of the K1 path: 4 KiB items at random 16-B-multiple strides
    and random counts (every mix of 4/2/1-step reductions), with and without
    crc_in."""
    import ctypes
    rng = np.random.default_rng(2000 + seed)
    n = int(rng.integers(1, 40000))
    stride = 4096 + 16 * int(rng.integers(0, 64))
    host = rng.integers(0, 256, n * stride, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * stride
    d = _dev(torch, host)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dcin = _dev(torch, cin.view(np.int32))
    for c in (None, cin):
        s = _lib.Spans(d.data_ptr(), host.size, None, stride, None, 4096,
                       None if c is None else dcin.data_ptr(), out.data_ptr(), n)
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None))
        np.testing.assert_array_equal(_u32(out), oracle.batch(host, offs, np.full(n, 4096), c))


def test_device_spans_outside_buffer_not_read(torch):
    """Spans past base_bytes are skipped (out = 0) and reported as ERANGE; the
    rest of the batch is exact.  Both the one-unit-per-span path (fixed
    length) and the planned path (per-span lengths)."""
    import ctypes
    rng = np.random.default_rng(77)
    host = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    d = _dev(torch, host)
    n = 500
    offs = rng.integers(0, host.size - 5000, n).astype(np.uint64)
    bad = np.array([3, 77, 499])
    offs[bad] = [host.size - 10, host.size + 4096, 1 << 62]
    for lens in (np.full(n, 4133, np.uint32), rng.integers(0, 5000, n).astype(np.uint32)):
        lens[bad[0]] = max(int(lens[bad[0]]), 11)  # ends past the buffer
        good = np.ones(n, bool)
        good[bad] = False
        want = np.zeros(n, np.uint32)
        want[good] = oracle.batch(host, offs[good], lens[good])
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        dl = _dev(torch, lens.view(np.int32))
        s = _lib.Spans(d.data_ptr(), host.size, _dev(torch, offs.view(np.int64)).data_ptr(), 0,
                       dl.data_ptr() if lens.min() != lens.max() else None, int(lens[0]), None, out.data_ptr(), n)
        rc = _lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None)
        assert rc == _lib.CRC32C_ERANGE
        np.testing.assert_array_equal(_u32(out), want)
        # a batch without such spans reports OK again (the counter is per call)
        s.n = 3
        assert _lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_OK


def test_fixed_stride_overrun_rejected(torch):
    import ctypes
    d = torch.zeros(10 * 4096, dtype=torch.uint8, device="cuda")
    out = torch.zeros(11, dtype=torch.int32, device="cuda")
    s = _lib.Spans(d.data_ptr(), d.numel(), None, 4096, None, 4096, None, out.data_ptr(), 11)
    assert _lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_EINVAL
    s.n = 10
    assert _lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_OK
    # base_bytes larger than the allocation holding base
    s.base_bytes = 1 << 40
    assert _lib.lib.crc32c_batch(ctypes.byref(s), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_EINVAL


def test_python_device_descriptor_checks(torch):
    d = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(TypeError):
        mc.batch(d, offsets=torch.zeros(4, dtype=torch.int32, device="cuda"), length=16)
    with pytest.raises(TypeError):
        mc.batch(d, offsets=torch.zeros(4, dtype=torch.int64, device="cuda"),
                 lens=torch.zeros(4, dtype=torch.int64, device="cuda"))
    with pytest.raises(ValueError):
        mc.batch(d, offsets=torch.zeros(4, dtype=torch.int64, device="cuda"),
                 lens=torch.zeros(4, dtype=torch.int32, device="cuda"),
                 out=torch.zeros(3, dtype=torch.int32, device="cuda"))
    with pytest.raises(TypeError):
        mc.verify_items(d, torch.zeros(4, dtype=torch.int32, device="cuda"))


def test_verify_pages_count_only_query(torch):
    """cap == 0 counts the walk's items and verifies nothing; a cap below the
    count still verifies every item."""
    import ctypes
    rng = np.random.default_rng(43)
    items = [layout.make_item(b"q%05d" % i, rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes(),
                              cas=i + 1) for i in range(700)]
    wbuf = 128 << 10
    buf, offs = layout.pack_wbufs(items, wbuf)
    mc.stamp_items(buf, offs, region_bytes=wbuf)
    buf[int(offs[10]) + 60] ^= 4
    d = _dev(torch, buf)
    nitems, nbad = ctypes.c_uint64(0), ctypes.c_uint64(7)
    _lib.check(_lib.lib.crc32c_verify_pages(d.data_ptr(), buf.size, wbuf, None, None, 0, ctypes.byref(nitems),
                                            ctypes.byref(nbad), _lib.CRC32C_DEVICE, None))
    assert nitems.value == offs.size and nbad.value == 0
    got_offs, got_ok, nb = mc.verify_pages(d, wbuf)
    assert nb == 1 and got_ok.cpu().numpy()[10] == 0
    np.testing.assert_array_equal(got_offs.cpu().numpy().astype(np.uint64), offs)
    # host path: capacity bound from the header
    got_offs, got_ok, nb = mc.verify_pages(buf, wbuf)
    assert nb == 1 and got_offs.size == offs.size
    # a capacity below the item count: the first cap items and verdicts, the
    # full count, every item verified (device and host arrays)
    cap = offs.size // 2
    want_ok = np.ones(cap, np.uint8)
    want_ok[10] = 0
    d_offs = _dev(torch, np.full(cap + 5, -1, np.int64))
    d_ok = _dev(torch, np.full(cap + 5, 7, np.uint8))
    _lib.check(_lib.lib.crc32c_verify_pages(d.data_ptr(), buf.size, wbuf, d_offs.data_ptr(), d_ok.data_ptr(), cap,
                                            ctypes.byref(nitems), ctypes.byref(nbad), _lib.CRC32C_DEVICE, None))
    torch.cuda.synchronize()
    assert nitems.value == offs.size and nbad.value == 1
    np.testing.assert_array_equal(d_offs.cpu().numpy()[:cap].astype(np.uint64), offs[:cap])
    np.testing.assert_array_equal(d_ok.cpu().numpy()[:cap], want_ok)
    assert (d_offs.cpu().numpy()[cap:] == -1).all() and (d_ok.cpu().numpy()[cap:] == 7).all()
    h_offs, h_ok = np.zeros(cap, np.uint64), np.zeros(cap, np.uint8)
    _lib.check(_lib.lib.crc32c_verify_pages(buf.ctypes.data, buf.size, wbuf, h_offs.ctypes.data, h_ok.ctypes.data, cap,
                                            ctypes.byref(nitems), ctypes.byref(nbad), 0, None))
    assert nitems.value == offs.size and nbad.value == 1
    np.testing.assert_array_equal(h_offs, offs[:cap])
    np.testing.assert_array_equal(h_ok, want_ok)
