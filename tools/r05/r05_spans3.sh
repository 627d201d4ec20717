#!/bin/bash
# Round 5: the span kernels' pieces layout with the per-half chains
# (half_value: no 80-B spill), nt (ab/hvnt) and default policy (ab/hvdflt),
# against the shipped row layout (ab/head), on the planned-path workloads.
#   bash tools/r05_spans3.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05sp3}; R=${2:-2}; mkdir -p $O
for r in $(seq 1 $R); do
  for n in head hvnt hvdflt; do
    for w in "config3" "pagesmix --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
