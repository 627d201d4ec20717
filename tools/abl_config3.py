"""Timing-only A/B of span-kernel ablation builds on the config-3 batch.

The batch of bench.py --workload config3 with 8 KiB of slack before the first
span (an ablation that drops the head-piece zero-line selects reads up to
4 KiB before a span, which must stay inside the allocation).  The library is
chosen by MCRC_LIB (memcached_amd/_lib.py).  Prints one JSON line.
    MCRC_LIB=ab/libmcrc32c_X.so python tools/abl_config3.py [steps]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from memcached_amd import _lib  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_device(0)
lens = bench.zipf_lens(1 << 20)
pad = 8192
offs = np.concatenate([[pad + 1], pad + 1 + np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
total = int(offs[-1] + lens[-1] + 16)
g = torch.Generator(device="cuda").manual_seed(3)
data = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.empty(lens.size, dtype=torch.int32, device="cuda")
sp = _lib.Spans(data.data_ptr(), total, d_offs.data_ptr(), 0, d_lens.data_ptr(), 0, None, out.data_ptr(), lens.size)
st = torch.cuda.current_stream()
for _ in range(3):
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC,
                                     ctypes.c_void_p(st.cuda_stream)), "warmup")
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(st)
for _ in range(steps):
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC,
                                     ctypes.c_void_p(st.cuda_stream)), "batch")
b.record(st)
torch.cuda.synchronize()
ms = a.elapsed_time(b) / steps
nbytes = int(lens.astype(np.uint64).sum())
print(json.dumps({"lib": os.path.basename(os.environ.get("MCRC_LIB", "libmcrc32c.so")), "ms": round(ms, 4),
                  "hbm_frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}))
