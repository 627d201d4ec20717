#!/bin/bash
# Round 5: the whole-span limit kWholeMax at 256 / 384 / 512 against 1024
# (ab/w256, ab/w384, ab/w512, ab/head): config 3 (Zipf from 64 B) and the
# mixed pages, three rounds.
#   bash tools/r05_wholemax3.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05w3}; R=${2:-3}; mkdir -p $O
for r in $(seq 1 $R); do
  for n in head w512 w384 w256; do
    for w in "config3" "pagesmix --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
