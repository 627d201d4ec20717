#!/bin/bash
# Round 5: plan rounds of 4 / 8 GiB (ab/rb4, ab/rb8)
# against no rounds (ab/head), at 1000 and 300 mixed pages and config 3.
#   bash tools/r05_roundbytes.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05rb2}; R=${2:-2}; mkdir -p $O
for r in $(seq 1 $R); do
  for n in head rb4 rb8; do
    for w in "pagesmix --pages 1000" "pagesmix --pages 300" "config3"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
