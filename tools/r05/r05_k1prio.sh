#!/bin/bash
# Round 5: K1's load issue at raised wave priority (s_setprio 2 around
# each half's four loads; ab/prio) against the shipped K1 (ab/head).
#   bash tools/r05_k1prio.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05kp}; R=${2:-4}; mkdir -p $O
for r in $(seq 1 $R); do
  for n in head prio; do
    echo "== round $r lib $n" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
echo done
