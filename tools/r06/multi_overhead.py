"""Per-call cost of crc32c_batch_multi at N = 1 against crc32c_batch on the
same host batch: the hand-off to the persistent device
worker is the difference.  Prints one JSON line per case.

    python tools/r06/multi_overhead.py [REPS]
"""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from memcached_amd import _lib  # noqa: E402

lib = _lib.lib


def timed(fn, reps):
    fn()
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6, min(ts) * 1e6


def case(name, n, pinned, reps):
    nbytes = n * 4096
    if pinned:
        p = lib.crc32c_host_alloc(nbytes)
        assert p, "crc32c_host_alloc"
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    else:
        p = None
        buf = np.empty(nbytes, np.uint8)
    buf[:] = np.random.default_rng(n).integers(0, 256, nbytes, dtype=np.uint8)
    out_a = np.zeros(n, np.uint32)
    out_b = np.zeros(n, np.uint32)
    sa = _lib.Spans(buf.ctypes.data, nbytes, None, 4096, None, 4096, None, out_a.ctypes.data, n)
    sb = _lib.Spans(buf.ctypes.data, nbytes, None, 4096, None, 4096, None, out_b.ctypes.data, n)
    med_a, min_a = timed(lambda: _lib.check(lib.crc32c_batch(ctypes.byref(sa), 0, None)), reps)
    med_b, min_b = timed(lambda: _lib.check(lib.crc32c_batch_multi(ctypes.byref(sb), 1)), reps)
    assert (out_a == out_b).all()
    rec = {"case": name, "items": n, "bytes": nbytes, "pinned": pinned, "reps": reps,
           "batch_us_median": round(med_a, 1), "batch_us_min": round(min_a, 1),
           "multi1_us_median": round(med_b, 1), "multi1_us_min": round(min_b, 1),
           "multi1_minus_batch_us": round(med_b - med_a, 1),
           "batch_GiBps": round(nbytes / med_a / 1e-6 / 2**30, 2), "multi1_GiBps": round(nbytes / med_b / 1e-6 / 2**30, 2)}
    print(json.dumps(rec), flush=True)
    if p:
        lib.crc32c_host_free(p)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    assert lib.crc32c_gpu_count() >= 1
    case("64 x 4 KiB pageable", 64, False, reps)
    case("64 x 4 KiB pinned", 64, True, reps)
    case("4096 x 4 KiB pinned", 4096, True, reps)
    case("65536 x 4 KiB pinned", 65536, True, max(20, reps // 20))


if __name__ == "__main__":
    main()
