#!/bin/bash
# Round 6: span-kernel variants (ab/<name>, tools/r06/variants.py) against the
# product (ab/cur) on config 3 and the mixed pages, alternating, one box.
#   bash tools/r06/spans_variants_ab.sh OUT ROUNDS "NAMES..."
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_spv}; R=${2:-3}; N=${3:-"cur lbfast u32 remat"}
mkdir -p $O
for r in $(seq 1 $R); do
  for n in $N; do
    for w in "config3 --steps 10 --warmup 2" "pagesmix --pages 1000 --steps 5 --warmup 1"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
