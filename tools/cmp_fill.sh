#!/bin/bash
# bench.py with splitmix64 vs torch.randint item bytes, alternating on one box
source tools/gpu_guard.sh
O=gpurun_out/${1:-fill}; mkdir -p $O
for i in 1 2; do
  run 300 python bench.py --no-cpu-baseline --fill randint > $O/r$i.json 2>/dev/null
  run 300 python bench.py --no-cpu-baseline --fill splitmix > $O/s$i.json 2>/dev/null
done
echo done
