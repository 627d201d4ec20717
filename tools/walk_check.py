"""Dev check: the bench's config-5 pages (PAGES x 64 MiB), walked on the
device by this library (twice) and by another build (REF_LIB, e.g. the
previous commit's); prints the item counts and, for wbufs whose walks differ,
where they part and the header bytes there.
    python tools/walk_check.py PAGES REF_LIB"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from memcached_amd import _lib  # noqa: E402
import torch  # noqa: E402

pages = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ref = ctypes.CDLL(sys.argv[2]) if len(sys.argv) > 2 else None
bench.workload_config5(argparse.Namespace(pages=pages), 0, 1)
data = bench._KEEP[-2]
wbuf = 4 << 20
nbytes = data.numel()
cap = nbytes // 50 + nbytes // wbuf + 1
offs = torch.empty(cap, dtype=torch.int64, device="cuda")
ok = torch.empty(cap, dtype=torch.uint8, device="cuda")


def walk(lib):
    n, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = lib.crc32c_verify_pages(ctypes.c_void_p(data.data_ptr()), ctypes.c_uint64(nbytes), ctypes.c_uint64(wbuf),
                                 ctypes.c_void_p(offs.data_ptr()), ctypes.c_void_p(ok.data_ptr()),
                                 ctypes.c_uint64(cap), ctypes.byref(n), ctypes.byref(nb), ctypes.c_uint(1),
                                 ctypes.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0, rc
    return offs[:n.value].cpu().numpy().copy(), int(nb.value)


runs = [("cur0",) + walk(_lib.lib), ("cur1",) + walk(_lib.lib)]
if ref is not None:
    runs.append(("ref",) + walk(ref))
host = None
for name, o, nb in runs:
    print(name, "items", o.size, "nbad", nb, flush=True)
base_name, base, _ = runs[-1]
bc = np.bincount((base // wbuf).astype(np.int64), minlength=nbytes // wbuf)
for name, o, nb in runs[:-1]:
    c = np.bincount((o // wbuf).astype(np.int64), minlength=nbytes // wbuf)
    bad = np.nonzero(c != bc)[0]
    print(f"{name} vs {base_name}: {bad.size} wbufs differ", flush=True)
    if host is None and bad.size:
        host = data.cpu().numpy()
    for w in bad[:6]:
        a = o[(o // wbuf) == w] - w * wbuf
        b = base[(base // wbuf) == w] - w * wbuf
        k = next((i for i in range(min(a.size, b.size)) if a[i] != b[i]), min(a.size, b.size))
        print(f"  wbuf {w}: {a.size} vs {b.size} items, part at item {k}: "
              f"{a[k] if k < a.size else None} vs {b[k] if k < b.size else None}", flush=True)
        for x in sorted({int(v) for v in (a[k - 1:k + 1].tolist() + b[k - 1:k + 1].tolist())}):
            h = host[w * wbuf + x: w * wbuf + x + 48]
            print(f"    @{x}: nbytes {int.from_bytes(bytes(h[32:36]), 'little')} flags {h[38]:#x},{h[39]:#x} "
                  f"nkey {h[41]}", flush=True)
