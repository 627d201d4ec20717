"""Round 5: where K5's verify loses against its span form on the same bytes.

Over the bench's config-5 pages (300 by default) times, event-timed after a
clock settle, the median of REPS calls of:
  verify   crc32c_verify_items (MODE 1: headers parsed, stored CRCs compared)
  stamp    crc32c_stamp_items  (MODE 2)
  spans    crc32c_batch over the same spans [off + 32, off + 4165) given as
           offsets (MODE 0: no header reads; K5 k_lines<0, true>)
One JSON line per mode.
    python tools/r05_k5modes.py [PAGES] [REPS]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from memcached_amd import _lib  # noqa: E402


def main():
    pages = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    vargs, ok, victims, nbytes, cfg = bench.workload_config5(argparse.Namespace(pages=pages), 0, 1)
    base, size, region, offs, n, okp = vargs
    data, offs_t = bench._KEEP[-2], bench._KEEP[-1]
    span_offs = (offs_t + 32).contiguous()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = _lib.Spans(base, size, span_offs.data_ptr(), 0, None, 4133, None, out.data_ptr(), n)
    nbad = ctypes.c_uint64(0)
    st = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(st.cuda_stream)
    calls = {
        "verify": lambda: _lib.check(_lib.lib.crc32c_verify_items(base, size, region, offs, n, okp, ctypes.byref(nbad),
                                                                  _lib.CRC32C_DEVICE, sptr)),
        "stamp": lambda: _lib.check(_lib.lib.crc32c_stamp_items(base, size, region, offs, n, None, ctypes.byref(nbad),
                                                                _lib.CRC32C_DEVICE, sptr)),
        "spans": lambda: _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, sptr)),
    }
    t0 = time.time()
    while time.time() - t0 < 0.3:
        calls["spans"]()
        torch.cuda.synchronize()
    for rnd in range(2):
        for name, fn in calls.items():
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                fn()
                b.record(st)
                b.synchronize()
                ts.append(a.elapsed_time(b))
            ts.sort()
            ms = ts[len(ts) // 2]
            print(json.dumps({"round": rnd, "mode": name, "pages": pages, "ms": round(ms, 4),
                              "hbm_frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
