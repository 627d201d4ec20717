"""Multi-rank path on CPU: world_size 2 over gloo.

Each rank checksums only its own shard (the product's host scalar CRC here:
there is no GPU on this host; tests/test_gpu_items_queue.py runs two ranks
through the batch path on the GPU), no data is exchanged on the compute path;
the test then gathers the shards to check they tile the batch exactly and
match the oracle.  The C split (crc32c_shard_cuts, used by
crc32c_batch_multi) is checked against shard.plan here too: it is host code.
"""
import os
import socket

import numpy as np
import pytest

from memcached_amd import shard

from . import oracle


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_plan_balances_bytes_and_tiles():
    rng = np.random.default_rng(0)
    lens = (64 * 1.25 ** rng.integers(0, 44, 5000)).astype(np.uint64)
    for world in (1, 2, 3, 4, 8):
        c = shard.plan(lens, world)
        assert c[0] == 0 and c[-1] == lens.size and (np.diff(c) >= 0).all()
        per = [int(lens[c[r]:c[r + 1]].sum()) for r in range(world)]
        assert max(per) - min(per) <= 2 * int(lens.max())
    assert list(shard.plan_equal(8 << 20, 8)) == [i << 20 for i in range(9)]


def test_c_shard_cuts_equal_plan():
    """crc32c_shard_cuts (C, 128-bit prefix) and shard.plan (numpy) give the
    same cut points: Zipf lengths for 1-8 parts, equal lengths, zero-length
    spans, fewer spans than parts, an empty batch."""
    from memcached_amd import crc32c as mc
    rng = np.random.default_rng(7)
    zipf = np.minimum(rng.zipf(1.3, 20000) * 64, 1 << 20).astype(np.uint32)
    cases = [zipf, np.full(1000, 4096, np.uint32), np.zeros(50, np.uint32),
             np.array([5, 0, 0, 7, 1 << 20], np.uint32), np.array([9], np.uint32), np.zeros(0, np.uint32)]
    for lens in cases:
        for parts in range(1, 9):
            got = mc.shard_cuts(lens, parts)
            np.testing.assert_array_equal(got, shard.plan(lens.astype(np.uint64), parts))
            assert got[0] == 0 and got[-1] == lens.size and (np.diff(got) >= 0).all()


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from memcached_amd import crc32c as mc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(1234)  # same batch on every rank
    lens = rng.integers(0, 6000, 700).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    buf = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    c = shard.plan(lens, world)
    mine = [mc.crc32c(0, buf[int(offs[i]):int(offs[i] + lens[i])]) for i in range(c[rank], c[rank + 1])]
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, int(c[rank]), mine))
    dist.destroy_process_group()
    if rank == 0:
        full = [x for _, _, part in sorted(gathered) for x in part]
        want = oracle.batch(buf, offs, lens)
        q.put(full == [int(x) for x in want])


def test_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def _bench_worker(rank, world, port, q):
    import time

    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, _ = bench.dist_setup(world, backend="gloo")
    # rank 1 is slower: the reported time must be the max over ranks
    elapsed, out = bench.timed(lambda k: [time.sleep(0.05 * (1 + r)) for _ in range(k)], 3, w, sync=lambda: None)
    import torch.distributed as dist
    dist.destroy_process_group()
    q.put((r, elapsed))


def test_bench_timing_is_max_over_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(2))
    assert abs(res[0] - res[1]) < 1e-9 and res[0] >= 0.3
