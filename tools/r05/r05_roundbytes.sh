#!/bin/bash
# Round 5: plan rounds of 1 / 4 GiB (ab/rb1: at most 64 rounds, ab/rb4: 16)
# against 2 GiB (ab/rounds: 32), at 1000 and 300 mixed pages and config 3.
#   bash tools/r05_roundbytes.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05rb}; R=${2:-2}; mkdir -p $O
for r in $(seq 1 $R); do
  for n in rounds rb1 rb4; do
    for w in "pagesmix --pages 1000" "pagesmix --pages 300" "config3"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
