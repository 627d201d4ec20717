"""GPU parity, round 3: item images of LARGE_CLIENT_FLAGS builds, exact bad
counts across consecutive small calls, host item calls on page-locked and
pageable buffers (zero-copy and staged), the coalescing submit queue, the
multi-GPU split and two ranks sharing the batch path.  Bit-exact against the
CPU oracle."""
import ctypes
import os
import socket
import threading

import numpy as np
import pytest

try:  # GPU processes load torch (and its HIP runtime) before libmcrc32c.so
    import torch as _torch  # noqa: F401
except ImportError:
    pass

from memcached_amd import _lib, layout, shard
from memcached_amd import crc32c as mc

from . import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    assert mc.gpu_count() >= 1, "libmcrc32c.so sees no gfx950 device"
    return t


@pytest.fixture(params=["small", "planned"])
def span_path(request):
    prev = mc.set_small_max(0 if request.param == "planned" else 8192)
    yield request.param
    mc.set_small_max(prev)


def _pages(rng, n, wbuf, cfl, max_value=3000, flag_every=2):
    items = [layout.make_item(b"key%07d" % i, rng.integers(0, 256, int(rng.integers(0, max_value)),
                                                            dtype=np.uint8).tobytes(),
                              cas=i + 1 if i % 5 else None,
                              client_flags=(0x1_0000_0003 if cfl == 8 else 0x3) * (i % flag_every),
                              cflags_bytes=cfl) for i in range(n)]
    buf, offs = layout.pack_wbufs(items, wbuf)
    return buf, offs


def _crcs(buf, offs, cfl):
    return np.array([oracle.item_crc(buf, o, cfl) for o in offs], np.uint32)


def _stored(buf, offs):
    return buf[(offs[:, None].astype(np.int64) + np.arange(28, 32))].copy().view("<u4").reshape(-1)


@pytest.mark.parametrize("cfl", [4, 8])
def test_client_flags_width_items(torch, span_path, cfl):
    """Verify, stamp and the device page walk over images whose ITEM_CFLAGS
    suffix is 4 or 8 bytes (memcached.h:96-100, :149-152): exact with the
    matching width, and the wrong width breaks flagged items."""
    rng = np.random.default_rng(100 + cfl)
    wbuf = 128 * 1024
    buf, offs = _pages(rng, 400, wbuf, cfl)
    want = _crcs(buf, offs, cfl)
    layout.store_crcs(buf, offs, want)
    wide = cfl == 8
    d = torch.from_numpy(buf).cuda()
    doffs = torch.from_numpy(offs.view(np.int64)).cuda()
    ok, nbad = mc.verify_items(d, doffs, region_bytes=wbuf, cflags64=wide)
    assert nbad == 0 and bool(ok.all())
    ok_h, nbad_h = mc.verify_items(buf, offs, region_bytes=wbuf, cflags64=wide)
    assert nbad_h == 0 and ok_h.all()
    if wide:  # the 4-byte rule mis-sizes the flagged items (half of them)
        _, nbad_w = mc.verify_items(d, doffs, region_bytes=wbuf, cflags64=False)
        assert nbad_w >= (offs.size // 2) * 9 // 10
    # stamp: exptime zeroed, then written by the library = the oracle's spill CRC
    z = buf.copy()
    layout.store_crcs(z, offs, np.zeros(offs.size, np.uint32))
    dz = torch.from_numpy(z).cuda()
    ok, nbad = mc.stamp_items(dz, doffs, region_bytes=wbuf, cflags64=wide)
    torch.cuda.synchronize()
    assert nbad == 0 and bool(ok.all())
    np.testing.assert_array_equal(_stored(dz.cpu().numpy(), offs), want)
    zh = z.copy()
    ok, nbad = mc.stamp_items(zh, offs, region_bytes=wbuf, cflags64=wide)
    assert nbad == 0 and ok.all()
    np.testing.assert_array_equal(zh, buf)
    # the device walk finds every image at its offset
    w_offs, w_ok, w_bad = mc.verify_pages(d, wbuf, cflags64=wide)
    np.testing.assert_array_equal(w_offs.cpu().numpy().astype(np.uint64), offs)
    assert w_bad == 0 and bool(w_ok.all())


@pytest.mark.parametrize("where", ["device", "host"])
def test_small_verify_bad_counts_exact_across_calls(torch, where):
    """k_small hands its bad count to the host through its last workgroup:
    calls with thousands of bad items spread over every workgroup, alternated
    with clean calls, must each report exactly their own count (an
    add still in flight when the last workgroup read the counter was lost in
    its call and counted in the next)."""
    rng = np.random.default_rng(7)
    wbuf = 4 << 20
    buf, offs = _pages(rng, 2000, wbuf, 4, max_value=1500, flag_every=3)
    layout.store_crcs(buf, offs, _crcs(buf, offs, 4))
    bad = buf.copy()
    victims = np.sort(rng.choice(offs.size, 1500, replace=False))
    for v in victims:
        bad[int(offs[v]) + 40] ^= 0x01  # pad byte 40 lies in the span: a CRC mismatch
    assert buf.size <= 8 << 20  # the single-launch path
    mk = (lambda a: torch.from_numpy(a).cuda()) if where == "device" else (lambda a: a)
    clean_b, bad_b = mk(buf), mk(bad)
    o = torch.from_numpy(offs.view(np.int64)).cuda() if where == "device" else offs
    for rep in range(12):
        ok, nbad = mc.verify_items(bad_b, o, region_bytes=wbuf)
        assert nbad == victims.size, rep
        okn = ok.cpu().numpy() if where == "device" else ok
        np.testing.assert_array_equal(np.nonzero(okn == 0)[0], victims)
        ok, nbad = mc.verify_items(clean_b, o, region_bytes=wbuf)
        assert nbad == 0, rep


def test_host_item_calls_pinned_pageable_and_large(torch):
    """Host stamp / verify: page-locked buffers are read (and stamped) in place
    by the kernel, also through an interior pointer; pageable ones through a
    pinned copy; buffers past 8 MiB through the staged planned path."""
    rng = np.random.default_rng(11)
    wbuf = 1 << 20
    buf, offs = _pages(rng, 900, wbuf, 4, max_value=2500)
    want = _crcs(buf, offs, 4)
    z = buf.copy()
    layout.store_crcs(z, offs, np.zeros(offs.size, np.uint32))
    ref = z.copy()
    layout.store_crcs(ref, offs, want)
    # pageable
    zh = z.copy()
    ok, nbad = mc.stamp_items(zh, offs, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    np.testing.assert_array_equal(zh, ref)
    # page-locked, from the start and from an interior pointer (one wbuf in)
    pin = torch.from_numpy(z.copy()).pin_memory()
    pa = pin.numpy()
    ok, nbad = mc.stamp_items(pa, offs, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    np.testing.assert_array_equal(pa, ref)
    pin2 = torch.from_numpy(z.copy()).pin_memory()
    tail = pin2.numpy()[wbuf:]
    sel = offs >= wbuf
    ok, nbad = mc.stamp_items(tail, offs[sel] - wbuf, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    np.testing.assert_array_equal(pin2.numpy()[wbuf:], ref[wbuf:])
    assert (pin2.numpy()[:wbuf] == z[:wbuf]).all()
    ok, nbad = mc.verify_items(pa, offs, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    # large (> 8 MiB): staged into device scratch, planned kernels
    big_items = [layout.make_item(b"key%07d" % i, rng.integers(0, 256, 9000, dtype=np.uint8).tobytes())
                 for i in range(1100)]
    bb, bo = layout.pack_wbufs(big_items, wbuf)
    assert bb.size > 8 << 20
    bwant = _crcs(bb, bo, 4)
    ok, nbad = mc.stamp_items(bb, bo, region_bytes=wbuf)
    assert nbad == 0 and ok.all()
    np.testing.assert_array_equal(_stored(bb, bo), bwant)
    bb[int(bo[500]) + 100] ^= 4
    ok, nbad = mc.verify_items(bb, bo, region_bytes=wbuf)
    assert nbad == 1 and np.nonzero(ok == 0)[0].tolist() == [500]


def _submit(spans, flags=0):
    job = ctypes.c_void_p()
    _lib.check(_lib.lib.crc32c_batch_submit(ctypes.byref(spans), flags, ctypes.byref(job)), "submit")
    return job


def test_queue_mixed_jobs_from_threads(torch):
    """Jobs from 12 threads through crc32c_batch_submit / _wait: page-locked
    host jobs (coalesced into shared launches), pageable host jobs and device
    jobs (run alone by the dispatcher), chained with crc_in; every CRC exact."""
    rng = np.random.default_rng(21)
    size = 3 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    pin = torch.from_numpy(host).pin_memory()
    dev = torch.from_numpy(host).cuda()
    torch.cuda.synchronize()
    l0, s0, j0, q0 = mc.queue_stats()
    errors = []

    def worker(t):
        try:
            r = np.random.default_rng(1000 + t)
            for it in range(40):
                n = int(r.integers(1, 9))
                lens = r.integers(0, 70000, n).astype(np.uint32)
                offs = np.array([int(r.integers(0, size - int(x))) for x in lens], np.uint64)
                cin = r.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
                out = np.empty(n, np.uint32)
                kind = (t + it) % 3
                if kind == 2:  # device job: every array in device memory
                    do = torch.from_numpy(offs.view(np.int64)).cuda()
                    dl = torch.from_numpy(lens.view(np.int32)).cuda()
                    dc = torch.from_numpy(cin.view(np.int32)).cuda()
                    dout = torch.empty(n, dtype=torch.int32, device="cuda")
                    torch.cuda.synchronize()
                    sp = _lib.Spans(dev.data_ptr(), size, do.data_ptr(), 0, dl.data_ptr(), 0, dc.data_ptr(),
                                    dout.data_ptr(), n)
                    _lib.check(_lib.lib.crc32c_batch_wait(_submit(sp, _lib.CRC32C_DEVICE)), "wait")
                    out = dout.cpu().numpy().view(np.uint32)
                else:
                    base = pin.data_ptr() if kind == 0 else host.ctypes.data
                    sp = _lib.Spans(base, size, offs.ctypes.data, 0, lens.ctypes.data, 0, cin.ctypes.data,
                                    out.ctypes.data, n)
                    _lib.check(_lib.lib.crc32c_batch_wait(_submit(sp)), "wait")
                want = oracle.batch(host, offs, lens, cin)
                if not (out == want).all():
                    errors.append((t, it, kind))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    l1, s1, j1, q1 = mc.queue_stats()
    assert q1 - q0 == 2 * 160  # pageable + device jobs ran alone
    assert j1 - j0 == 160 and l1 - l0 <= 160  # page-locked jobs, packed into launches


def test_queue_rejects_out_of_range_host_spans(torch):
    buf = np.zeros(4096, np.uint8)
    offs = np.array([4000], np.uint64)
    lens = np.array([200], np.uint32)
    out = np.empty(1, np.uint32)
    sp = _lib.Spans(buf.ctypes.data, buf.size, offs.ctypes.data, 0, lens.ctypes.data, 0, None, out.ctypes.data, 1)
    job = ctypes.c_void_p()
    assert _lib.lib.crc32c_batch_submit(ctypes.byref(sp), 0, ctypes.byref(job)) == _lib.CRC32C_EINVAL


def test_batch_multi_matches_oracle(torch):
    """crc32c_batch_multi on every visible device (the byte-balanced split of
    crc32c_shard_cuts) over a Zipf-sized host batch."""
    rng = np.random.default_rng(33)
    lens = np.minimum(rng.zipf(1.3, 3000) * 64, 1 << 20).astype(np.uint32)
    offs = np.concatenate([[3], 3 + np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1] + 5), dtype=np.uint8)
    for ng in (1, 0):
        got = mc.batch_multi(buf, offsets=offs, lens=lens, ngpus=ng)
        np.testing.assert_array_equal(got, oracle.batch(buf, offs, lens))
    np.testing.assert_array_equal(mc.shard_cuts(lens, 8), shard.plan(lens, 8))


def test_batch_multi_config4_shape_every_device(torch):
    """BASELINE config 4's shape (equal 4 KiB items at stride 4096, one pinned
    host batch) split by crc32c_batch_multi over every visible device
    (torch.cuda.device_count(): the device != 0 paths run wherever the box has
    more than one), and over each device alone; every CRC against the oracle."""
    ng = torch.cuda.device_count()
    n = 32768 * max(ng, 2)
    host = torch.randint(0, 256, (n * 4096,), dtype=torch.uint8).pin_memory()
    buf = host.numpy()
    want = oracle.batch(buf, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096, np.uint64))
    out = np.empty(n, np.uint32)
    sp = _lib.Spans(host.data_ptr(), host.numel(), None, 4096, None, 4096, None, out.ctypes.data, n)
    _lib.check(_lib.lib.crc32c_batch_multi(ctypes.byref(sp), ng), "batch_multi")
    np.testing.assert_array_equal(out, want)
    cuts = mc.shard_cuts(np.full(n, 4096, np.uint32), ng)
    assert cuts[0] == 0 and cuts[-1] == n and all(int(cuts[g + 1] - cuts[g]) == n // ng for g in range(ng))
    for g in range(ng):  # each device alone, as the current device
        with torch.cuda.device(g):
            out[:] = 0
            _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), 0, None), f"device {g}")
            np.testing.assert_array_equal(out, want)


def test_eight_threads_concurrent_device_batches(torch):
    """Eight host threads each enqueue device batches on their own stream at
    once (thread t on device t % device_count: every device where the box has
    several), mixing K1 items, unaligned spans and async calls, many rounds:
    the per-call device lookup takes no process-wide lock after the first call
    (crc32c_shim.hip current_device) and no batch sees another's scratch.
    Every CRC against the oracle."""
    ng = torch.cuda.device_count()
    rng = np.random.default_rng(88)
    nthreads, rounds = 8, 12
    host = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    n1 = 512  # K1: 512 aligned 4 KiB items
    want1 = oracle.batch(host, np.arange(n1, dtype=np.uint64) * 4096, np.full(n1, 4096, np.uint64))
    lens = rng.integers(0, 20000, 400).astype(np.uint32)
    offs = rng.integers(0, host.size - 20000, 400).astype(np.uint64)
    want2 = oracle.batch(host, offs, lens)
    errors = []

    def worker(t):
        try:
            dev = t % ng
            with torch.cuda.device(dev):
                st = torch.cuda.Stream(device=dev)
                d = torch.from_numpy(host).to(f"cuda:{dev}")
                d_offs = torch.from_numpy(offs.view(np.int64)).to(f"cuda:{dev}")
                d_lens = torch.from_numpy(lens.view(np.int32)).to(f"cuda:{dev}")
                torch.cuda.synchronize(dev)
                for r in range(rounds):
                    with torch.cuda.stream(st):
                        out1 = torch.empty(n1, dtype=torch.int32, device=f"cuda:{dev}")
                        sp = _lib.Spans(d.data_ptr(), n1 * 4096, None, 4096, None, 4096, None, out1.data_ptr(), n1)
                        flags = _lib.CRC32C_DEVICE | (_lib.CRC32C_ASYNC if r % 2 else 0)
                        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), flags, ctypes.c_void_p(st.cuda_stream)))
                        out2 = mc.batch(d, offsets=d_offs, lens=d_lens, stream=st.cuda_stream,
                                        asynchronous=bool(r % 3 == 1))
                    st.synchronize()
                    if not (out1.cpu().numpy().view(np.uint32) == want1).all():
                        errors.append((t, r, "K1"))
                    if not (out2.cpu().numpy().view(np.uint32) == want2).all():
                        errors.append((t, r, "spans"))
        except Exception as e:  # noqa: BLE001  (reported by the main thread)
            errors.append((t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:8]


def test_bench_headline_over_every_device_in_one_process(torch):
    """bench.py --gpus N without a launcher (the driver's way of starting it):
    headline_devices runs K1 on every visible device from one process and
    prints the bench line with n_gpus = N (small batches here)."""
    import argparse
    import bench
    ng = torch.cuda.device_count()
    args = argparse.Namespace(gpus=ng, steps=3, warmup=1, settle_ms=0.0, items=1 << 14, fill="splitmix",
                              no_cpu_baseline=True, events="region")
    res = bench.headline_devices(args)
    assert res["n_gpus"] == ng and res["value"] > 0 and len(res["kernel_ms_per_device"]) == ng
    assert res["roofline"]["frac"] > 0 and res["scaling"] == "weak"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from memcached_amd import crc32c as mcl
    from memcached_amd import shard as sh
    torch.cuda.set_device(rank % torch.cuda.device_count())  # (one device per rank where there are several)
    rng = np.random.default_rng(77)  # the same batch on every rank
    lens = np.minimum(rng.zipf(1.2, 5000) * 32, 1 << 20).astype(np.uint32)
    offs = np.concatenate([[1], 1 + np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1] + 1), dtype=np.uint8)
    c = sh.plan(lens, world)
    lo, hi = int(c[rank]), int(c[rank + 1])
    d = torch.from_numpy(buf).cuda()  # each rank: its own copy, its own shard's spans
    out = mcl.batch(d, offsets=torch.from_numpy(offs[lo:hi].view(np.int64)).cuda(),
                    lens=torch.from_numpy(lens[lo:hi].view(np.int32)).cuda())
    torch.cuda.synchronize()
    mine = out.cpu().numpy().view(np.uint32).tolist()
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, lo, mine))
    dist.destroy_process_group()
    if rank == 0:
        full = [x for _, _, part in sorted(gathered) for x in part]
        q.put(full == [int(x) for x in oracle.batch(buf, offs, lens)])


def test_two_ranks_device_batch_path(torch):
    """Two processes (gloo for the exchange of results only), each checksumming
    its shard of shard.plan through the device batch path on the GPU."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


# ---------------------------------------------------------------------------
# One-block spans; K5 (k_items): one-block item images end to end
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("length", [4100, 4133, 4171, 4209])
def test_k5_fixed_length_spans(torch, length):
    """Batches of equal spans of 4100..4209 bytes (one block after a head
    fragment at every alignment: k_blocks + k_final): by stride and by
    offsets at every alignment, with and without initial CRCs, and a span
    outside the buffer (ERANGE, not read)."""
    rng = np.random.default_rng(length)
    n = 9000  # past the single-launch path's 8192
    stride = length + 29
    buf = rng.integers(0, 256, n * stride + 64, dtype=np.uint8)
    d = torch.from_numpy(buf).cuda()
    offs = (np.arange(n, dtype=np.uint64) * stride + 7).astype(np.uint64)
    want = oracle.batch(buf, offs, np.full(n, length, np.uint64))
    # by stride (base + 7: every alignment occurs)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = _lib.Spans(d.data_ptr() + 7, buf.size - 7, None, stride, None, length, None, out.data_ptr(), n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, None))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    # by offsets, shuffled, with crc_in
    perm = rng.permutation(n)
    cin = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    got = mc.batch(d, offsets=torch.from_numpy(offs[perm].view(np.int64)).cuda(), length=length,
                   crc_in=torch.from_numpy(cin.view(np.int32)).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32),
                                  oracle.batch(buf, offs[perm], np.full(n, length, np.uint64), cin))
    # one span past the end: out 0, CRC32C_ERANGE, the others exact
    bad = offs.copy()
    bad[123] = buf.size - length + 1
    out2 = torch.empty(n, dtype=torch.int32, device="cuda")
    o2 = torch.from_numpy(bad.view(np.int64)).cuda()
    sp2 = _lib.Spans(d.data_ptr(), buf.size, o2.data_ptr(), 0, None, length, None, out2.data_ptr(), n)
    assert _lib.lib.crc32c_batch(ctypes.byref(sp2), _lib.CRC32C_DEVICE, None) == _lib.CRC32C_ERANGE
    g2 = out2.cpu().numpy().view(np.uint32)
    assert g2[123] == 0
    np.testing.assert_array_equal(np.delete(g2, 123), np.delete(want, 123))


@pytest.mark.parametrize("n", [300001, 262144 * 2 + 8192 * 3 + 5])
def test_k5_spans_full_epochs(torch, n):
    """K5 MODE 0 over enough equal spans that every wave runs whole 32-step
    epochs plus a partial one (quad, pair and single tails): every CRC goes
    from the lanes that finish four images per quad back to the images' epoch
    lanes, which store it (no k_fix pass).  The config 2 variant's shape
    (4133-B spans at stride 4165, start +32), by stride, and by shuffled
    offsets with initial CRCs; every CRC against the oracle."""
    length, stride = 4133, 4165
    g = torch.Generator(device="cuda").manual_seed(n)
    d = torch.randint(0, 256, (n * stride + 64,), dtype=torch.uint8, device="cuda", generator=g)
    buf = d.cpu().numpy()
    offs = np.arange(n, dtype=np.uint64) * stride + 32
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = _lib.Spans(d.data_ptr() + 32, d.numel() - 32, None, stride, None, length, None, out.data_ptr(), n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, None))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32),
                                  oracle.batch(buf, offs, np.full(n, length, np.uint64)))
    rng = np.random.default_rng(n)
    perm = rng.permutation(n)
    cin = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    got = mc.batch(d, offsets=torch.from_numpy(offs[perm].view(np.int64)).cuda(), length=length,
                   crc_in=torch.from_numpy(cin.view(np.int32)).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32),
                                  oracle.batch(buf, offs[perm], np.full(n, length, np.uint64), cin))


def test_k5_stamp_and_verify_full_epochs(torch):
    """K5 stamps (MODE 2: k_items then k_fix) and verifies (MODE 1) over
    enough 4165-B images for whole 32-step epochs and a partial one: every
    stamped exptime equals the oracle's spill CRC (storage.c:567), the verify
    of the stamped images passes them all, and one flipped byte per 1000
    images is caught exactly."""
    n, nt = 300007, 4165
    g = torch.Generator(device="cuda").manual_seed(11)
    d = torch.randint(0, 256, (n * nt + 64,), dtype=torch.uint8, device="cuda", generator=g)
    im = d[:n * nt].view(n, nt)
    # memcached.h:613-636 header: nbytes 4098 (4096 + CRLF), it_flags ITEM_CAS,
    # nkey 10 -> ITEM_ntotal = 48 + 10 + 1 + 4098 + 8 = 4165; exptime zeroed
    im[:, 28:32] = 0
    im[:, 32:36] = torch.tensor([4098 & 255, 4098 >> 8, 0, 0], dtype=torch.uint8, device="cuda")
    im[:, 38:40] = torch.tensor([2, 0], dtype=torch.uint8, device="cuda")
    im[:, 41] = 10
    offs = np.arange(n, dtype=np.uint64) * nt
    doffs = torch.from_numpy(offs.view(np.int64)).cuda()
    before = d.cpu().numpy()
    want = oracle.batch(before, offs + 32, np.full(n, nt - 32, np.uint64))
    ok, nbad = mc.stamp_items(d, doffs)
    torch.cuda.synchronize()
    assert nbad == 0 and bool(ok.all())
    stamped = im[:, 28:32].contiguous().cpu().numpy().view(np.uint32).reshape(n)
    np.testing.assert_array_equal(stamped, want)
    ok, nbad = mc.verify_items(d, doffs)
    assert nbad == 0 and bool(ok.all())
    victims = np.arange(7, n, 1000)
    im[torch.from_numpy(victims).cuda(), 2000] ^= 0x40
    ok, nbad = mc.verify_items(d, doffs)
    assert nbad == victims.size
    np.testing.assert_array_equal(np.flatnonzero(ok.cpu().numpy() == 0), victims)


def _expected_verdicts(buf, offs, wbuf):
    """The oracle's verdict per image, as the library defines it: the header
    parses to a span inside the buffer and inside the image's wbuf, nkey != 0,
    and the stored exptime equals the spill CRC of that span."""
    ok = np.zeros(offs.size, np.uint8)
    for i, o in enumerate(offs.tolist()):
        if o + 48 > buf.size or buf[o + 41] == 0:
            continue
        nbytes = int.from_bytes(bytes(buf[o + 32:o + 36]), "little")
        if nbytes >= 1 << 31:
            continue
        nt = layout.ntotal_of(buf, o)
        if o + nt > buf.size or o // wbuf != (o + nt - 1) // wbuf:
            continue
        stored = int.from_bytes(bytes(buf[o + 28:o + 32]), "little")
        ok[i] = stored == oracle.item_crc(buf, o)
    return ok


def test_k5_verify_stamp_and_walk_with_fallback(torch):
    """Pages of 4165-B images (the K5 shape) with every kind of damage: a
    flipped length bit (some images then leave the one-block shape -- the
    fallback list and the planned path -- and some their wbuf -- malformed),
    a zeroed key length, a flipped data bit, and a few images of other sizes.
    Verify by offsets and by the device walk, and stamp: exact against the
    oracle, image by image."""
    rng = np.random.default_rng(55)
    wbuf = 1 << 20
    n = 6000
    vals = [4096 if i % 50 else int(rng.integers(200, 9000)) for i in range(n)]
    items = [layout.make_item(b"key%07d" % i, rng.integers(0, 256, v, dtype=np.uint8).tobytes(), cas=i + 1)
             for i, v in enumerate(vals)]
    buf, offs = layout.pack_wbufs(items, wbuf)
    soffs, slens = layout.spans_of(buf, offs)
    layout.store_crcs(buf, offs, oracle.batch(buf, soffs, slens))
    clean = buf.copy()
    victims = rng.choice(n, 300, replace=False)
    for k, v in enumerate(victims.tolist()):
        o = int(offs[v])
        if k % 3 == 0:
            buf[o + 32 + int(rng.integers(0, 2))] ^= 1 << int(rng.integers(0, 8))  # length bit
        elif k % 3 == 1:
            buf[int(soffs[v]) + int(rng.integers(16, slens[v]))] ^= 1 << int(rng.integers(0, 8))  # data bit
        else:
            buf[o + 40] ^= 0x40  # slabs_clsid: in the span, header stays sane
    buf[int(offs[17]) + 41] = 0  # a zeroed key length: malformed
    want = _expected_verdicts(buf, offs, wbuf)
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    for _ in range(2):
        ok, nbad = mc.verify_items(d, do, region_bytes=wbuf)
        np.testing.assert_array_equal(ok.cpu().numpy(), want)
        assert nbad == int((want == 0).sum())
    # the device walk of the same pages: stops where a damaged length sends it
    # (storage.c:950-960); compared with a host walk + the oracle
    w_offs, w_ok, w_bad = mc.verify_pages(d, wbuf)
    h_offs = []
    for w0 in range(0, buf.size, wbuf):
        o = w0
        while o + 48 <= min(w0 + wbuf, buf.size) and buf[o + 41] != 0:
            h_offs.append(o)
            nbytes = int.from_bytes(bytes(buf[o + 32:o + 36]), "little")  # (unsigned, as the kernels)
            o += layout.ntotal_of(buf, o) - int(np.int32(np.uint32(nbytes))) + nbytes
    h_offs = np.asarray(h_offs, np.uint64)
    np.testing.assert_array_equal(w_offs.cpu().numpy().astype(np.uint64), h_offs)
    hw = _expected_verdicts(buf, h_offs, wbuf)
    np.testing.assert_array_equal(w_ok.cpu().numpy(), hw)
    assert w_bad == int((hw == 0).sum())
    # stamp the clean pages with exptime zeroed: every image gets its spill CRC
    z = clean.copy()
    layout.store_crcs(z, offs, np.zeros(n, np.uint32))
    dz = torch.from_numpy(z).cuda()
    ok, nbad = mc.stamp_items(dz, do, region_bytes=wbuf)
    torch.cuda.synchronize()
    assert nbad == 0 and bool(ok.all())
    np.testing.assert_array_equal(dz.cpu().numpy(), clean)


def test_partly_registered_buffer_is_staged_not_read_in_place(torch):
    """A caller that page-locks only part of a buffer (crc32c_host_register of
    the first half of an arena) and passes spans or item images in the other
    half: the library must not read (or stamp) the range in place, which would
    page-fault the GPU; it stages those batches instead.  A fully registered
    buffer still takes the zero-copy path (coalesced by the queue)."""
    import mmap
    rng = np.random.default_rng(77)
    size = 4 << 20
    mm = mmap.mmap(-1, size)  # page-aligned, pageable
    arena = np.frombuffer(mm, dtype=np.uint8)
    arena[:] = rng.integers(0, 256, size, dtype=np.uint8)
    half = size // 2
    _lib.check(_lib.lib.crc32c_host_register(ctypes.c_void_p(arena.ctypes.data), ctypes.c_size_t(half)), "register")
    try:
        # spans on both sides of the registered boundary, through the queue
        n = 64
        lens = rng.integers(1, 60000, n).astype(np.uint32)
        offs = np.array([int(rng.integers(0, size - int(x))) for x in lens], np.uint64)
        offs[:8] = half - 100  # straddling the boundary
        offs[8:16] = size - lens[8:16]  # wholly in the unregistered half
        cin = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        want = oracle.batch(arena, offs, lens, cin)
        l0, s0, j0, q0 = mc.queue_stats()
        out = np.empty(n, np.uint32)
        sp = _lib.Spans(arena.ctypes.data, size, offs.ctypes.data, 0, lens.ctypes.data, 0, cin.ctypes.data,
                        out.ctypes.data, n)
        _lib.check(_lib.lib.crc32c_batch_wait(_submit(sp)), "wait")
        np.testing.assert_array_equal(out, want)
        l1, s1, j1, q1 = mc.queue_stats()
        assert q1 - q0 == 1 and j1 == j0  # run alone (staged), not coalesced in place
        np.testing.assert_array_equal(mc.batch(arena, offsets=offs, lens=lens, crc_in=cin), want)
        # the registered half alone is read in place (coalesced)
        inner = offs[16:][offs[16:] + lens[16:] <= half]
        il = lens[16:][offs[16:] + lens[16:] <= half]
        if inner.size:
            out2 = np.empty(inner.size, np.uint32)
            sp2 = _lib.Spans(arena.ctypes.data, half, inner.ctypes.data, 0, il.ctypes.data, 0, None,
                             out2.ctypes.data, inner.size)
            _lib.check(_lib.lib.crc32c_batch_wait(_submit(sp2)), "wait")
            np.testing.assert_array_equal(out2, oracle.batch(arena, inner, il))
            l2, s2, j2, q2 = mc.queue_stats()
            assert j2 - j1 == 1 and q2 == q1
        # item images packed into a wbuf that straddles the boundary: stamp and verify
        wbuf = 1 << 20
        items_buf, ioffs = _pages(rng, 300, wbuf, 4, max_value=2500)
        lo = half - wbuf // 2
        view = arena[lo:lo + items_buf.size]
        view[:] = items_buf
        layout.store_crcs(view, ioffs, np.zeros(ioffs.size, np.uint32))
        ok, nbad = mc.stamp_items(view, ioffs, region_bytes=wbuf)
        assert nbad == 0 and ok.all()
        np.testing.assert_array_equal(_stored(view, ioffs), _crcs(view, ioffs, 4))
        ok, nbad = mc.verify_items(view, ioffs, region_bytes=wbuf)
        assert nbad == 0 and ok.all()
    finally:
        _lib.check(_lib.lib.crc32c_host_unregister(ctypes.c_void_p(arena.ctypes.data)), "unregister")


@pytest.mark.parametrize("mix", ["fused", "mixed41"])
def test_k5_census_routes_by_shape(torch, mix):
    """Large item batches are routed on the device (k_census): all 4 KiB
    values (the K5 shape) and a mix of 2 KiB and 6.2 KiB values whose average
    image is also ~4.1 KiB (the old host rule's guess sent it to K5).  Verify
    and stamp are exact either way, including a damaged image per 97."""
    rng = np.random.default_rng(91 if mix == "fused" else 92)
    wbuf = 1 << 20
    n = 5000
    vals = [4096] * n if mix == "fused" else [2048 if i % 2 else 6150 for i in range(n)]
    items = [layout.make_item(b"key%07d" % i, rng.integers(0, 256, v, dtype=np.uint8).tobytes(), cas=i + 1)
             for i, v in enumerate(vals)]
    buf, offs = layout.pack_wbufs(items, wbuf)
    if mix == "mixed41":
        assert 4100 <= buf.size / n <= 4300
    soffs, slens = layout.spans_of(buf, offs)
    crcs = oracle.batch(buf, soffs, slens)
    layout.store_crcs(buf, offs, crcs)
    victims = np.arange(5, n, 97)
    for v in victims.tolist():
        buf[int(soffs[v]) + 100] ^= 2
    d = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ok, nbad = mc.verify_items(d, do, region_bytes=wbuf)
    assert nbad == victims.size
    np.testing.assert_array_equal(np.flatnonzero(ok.cpu().numpy() == 0), victims)
    # stamp with exptime zeroed: every image gets the oracle's spill CRC
    z = buf.copy()
    layout.store_crcs(z, offs, np.zeros(n, np.uint32))
    dz = torch.from_numpy(z).cuda()
    ok, nbad = mc.stamp_items(dz, do, region_bytes=wbuf)
    assert nbad == 0 and bool(ok.all())
    np.testing.assert_array_equal(_stored(dz.cpu().numpy(), offs), oracle.batch(z, soffs, slens))


def test_async_device_stamp_returns_before_the_kernels_finish(torch):
    """crc32c_stamp_items with CRC32C_DEVICE | CRC32C_ASYNC and nbad == NULL
    over a K5-sized batch enqueues everything (census, k_items, k_fix and the
    planned fallback with a device-side count) and returns: no read-back in
    the middle.  Queued behind several milliseconds of K1 work, the stream is
    still busy when the call returns; after a sync every stamp is exact."""
    n, nt = 20000, 4165
    g = torch.Generator(device="cuda").manual_seed(12)
    d = torch.randint(0, 256, (n * nt + 64,), dtype=torch.uint8, device="cuda", generator=g)
    im = d[:n * nt].view(n, nt)
    im[:, 28:32] = 0
    im[:, 32:36] = torch.tensor([4098 & 255, 4098 >> 8, 0, 0], dtype=torch.uint8, device="cuda")
    im[:, 38:40] = torch.tensor([2, 0], dtype=torch.uint8, device="cuda")
    im[:, 41] = 10
    im[::7, 32:36] = torch.tensor([0, 8, 0, 0], dtype=torch.uint8, device="cuda")  # nbytes 2048: not one block
    offs = np.arange(n, dtype=np.uint64) * nt
    doffs = torch.from_numpy(offs.view(np.int64)).cuda()
    host = d.cpu().numpy()
    soffs, slens = layout.spans_of(host, offs)
    want = oracle.batch(host, soffs, slens)
    def stamp():
        return _lib.lib.crc32c_stamp_items(ctypes.c_void_p(d.data_ptr()), ctypes.c_uint64(d.numel()),
                                           ctypes.c_uint64(0), ctypes.c_void_p(doffs.data_ptr()), ctypes.c_uint64(n),
                                           None, None, _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC,
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    # (a first call grows the library's scratch -- hipFree synchronises the
    # device -- and must stamp the same)
    _lib.check(stamp(), "async stamp")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_stored(d.cpu().numpy(), offs), want)
    im[:, 28:32] = 0
    big = torch.randint(0, 256, (1 << 30,), dtype=torch.uint8, device="cuda", generator=g)
    kout = torch.empty(1 << 18, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    for _ in range(16):  # ~3 ms of K1 ahead of the stamp on the same stream
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(_lib.Spans(big.data_ptr(), big.numel(), None, 4096, None,
                                                                 4096, None, kout.data_ptr(), 1 << 18)),
                                         _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC, ctypes.c_void_p(st.cuda_stream)))
    rc = stamp()
    busy = not st.query()
    _lib.check(rc, "async stamp")
    torch.cuda.synchronize()
    assert busy, "the async stamp waited for the stream"
    np.testing.assert_array_equal(_stored(d.cpu().numpy(), offs), want)
