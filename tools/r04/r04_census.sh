#!/bin/bash
# K5 routing on a batch whose average image is K5's size but whose images are
# not (mixed41: 2 KiB and 6 KiB values in turn): k_census (cur) against every
# batch to the planned path (planned) and every batch to K5 (k5, what the
# old average-size rule chose), then the fused config 5 the same three ways.
#   bash tools/r04_census.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for r in $(seq 1 $R); do
  for n in cur planned k5; do
    for w in mixed41 config5; do
      echo "== round $r lib $n workload $w" >> $O/ab_census.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --pages 300 --steps 5 --warmup 1 >> $O/ab_census.txt 2>> $O/ab_census.err
    done
  done
done
MCRC_LIB=ab/cur/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_mixed41 -o kt --output-format csv -- python3 bench.py --workload mixed41 --pages 300 --steps 3 --warmup 1 > $O/kt_mixed41.log 2>&1
echo done
