#!/bin/bash
# Round 5: K1 per byte at 4, 16 and 64 GiB batches (1, 4, 16 Mi x 4 KiB
# items), alternating, to tell whether reading slower per byte at larger
# batches (the mixed pages at 1000 pages) is the memory system's or the span
# kernel's.
#   bash tools/r05_k1_size.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r05k1sz}; R=${2:-2}; mkdir -p $O
for r in $(seq 1 $R); do
  for n in 1048576 4194304 16777216; do
    echo "== round $r items $n" >> $O/k1size.txt
    run 300 python bench.py --items $n --steps 10 --warmup 3 --no-cpu-baseline >> $O/k1size.txt 2>> $O/k1size.err
  done
done
echo done
