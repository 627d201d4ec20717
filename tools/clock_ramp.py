"""K1 kernel time per launch over a long sequence (clock ramp after idle).
    python tools/clock_ramp.py [launches]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
torch.cuda.set_device(0)
data, out, spans = bench.make_batch(bench.ITEMS_PER_GPU, 42)
stream = torch.cuda.current_stream()
evs = bench.run_steps(spans, n, stream)
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for a, b in evs]
for i in range(0, n, 20):
    chunk = ms[i:i + 20]
    print(f"launches {i:4d}-{i + len(chunk) - 1:4d}: mean {sum(chunk) / len(chunk):.4f} ms  min {min(chunk):.4f}")
