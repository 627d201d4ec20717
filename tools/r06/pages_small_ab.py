"""Per-call wall time of crc32c_verify_pages on a few wbufs of mixed items
(fewer than 4096 items: the planned verify, not K5), device-resident, one
thread, synchronous calls.  Prints one JSON line per case.

    MCRC_LIB=ab/X/libmcrc32c.so python tools/r06/pages_small_ab.py
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from memcached_amd import _lib  # noqa: E402


def main():
    out = {"lib": os.environ.get("MCRC_LIB", "in-tree")}
    for wl in ("pagesmix", "mixed41"):
        bench._KEEP.clear()
        vargs, ok, victims, nbytes, cfg = bench.workload_pagesmix(argparse.Namespace(pages=1, workload=wl), 0, 1)
        base, size, region, offs, n, okp = vargs
        for nw in (1, 4, 12):
            nb = nw * region
            cap = nb // 50 + nw
            woffs = torch.empty(cap, dtype=torch.int64, device="cuda")
            wok = torch.empty(cap, dtype=torch.uint8, device="cuda")
            nitems, nbad = ctypes.c_uint64(0), ctypes.c_uint64(0)

            def one():
                _lib.check(_lib.lib.crc32c_verify_pages(base, nb, region, woffs.data_ptr(), wok.data_ptr(), cap,
                                                        ctypes.byref(nitems), ctypes.byref(nbad),
                                                        _lib.CRC32C_DEVICE, None))
            for _ in range(20):
                one()
            ts = []
            for _ in range(60):
                t0 = time.perf_counter()
                one()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print(json.dumps({**out, "workload": wl, "wbufs": nw, "items": nitems.value, "nbad": nbad.value,
                              "median_us": round(ts[len(ts) // 2] * 1e6, 1), "min_us": round(ts[0] * 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
