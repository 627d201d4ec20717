#!/bin/bash
# k_count ablations on the mixed pages (wrong results, timing only):
# cnt1 = whole spans' chains skipped, cnt2 = every span chain skipped,
# against walk1 (the same code without the ablation).
#   bash tools/r04_cnt.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for r in $(seq 1 $R); do
  for n in walk1 cnt1 cnt2; do
    echo "== round $r lib $n workload pagesmix" >> $O/ab_cnt.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload pagesmix --pages 300 --steps 5 --warmup 1 >> $O/ab_cnt.txt 2>> $O/ab_cnt.err
  done
done
for n in walk1 cnt1 cnt2; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/ktc_$n -o kt --output-format csv -- python3 bench.py --workload pagesmix --pages 300 --steps 3 --warmup 1 > $O/ktc_$n.log 2>&1
done
echo cnt done
