"""Shard plans for multi-GPU batches.

Items are independent, so a batch is split into contiguous index ranges, one
per GPU, balanced by bytes (prefix sum of span lengths), not by count -- Zipf
sized batches put most bytes in a few large items.  No collective is needed on
the data path: each rank checksums its range and writes its slice of out[].
The same split is implemented in C++ by crc32c_batch_multi (crc32c_shim.hip).
"""
from __future__ import annotations

import numpy as np


def plan(lens, world: int):
    """Return world+1 cut points c with rank r owning items [c[r], c[r+1]).

    c[r] is the first item index i whose byte prefix sum(lens[:i]) reaches
    total * r // world, so every rank gets about total / world bytes -- the
    rule of crc32c_shard_cuts (include/crc32c_batch.h), which tests check
    this function against.
    """
    lens = np.asarray(lens, dtype=np.uint64)
    n = lens.size
    if world < 1:
        raise ValueError("world must be >= 1")
    prefix = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)])
    total = int(prefix[-1])
    cuts = [int(np.searchsorted(prefix, np.uint64(total * r // world), side="left")) for r in range(world)]
    return np.asarray(cuts + [n], dtype=np.int64)


def plan_equal(n: int, world: int):
    """Cut points for n equal-size items (BASELINE config 4: 8 Mi items on 8 GPUs)."""
    return np.asarray([n * r // world for r in range(world + 1)], dtype=np.int64)
