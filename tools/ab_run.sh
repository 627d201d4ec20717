#!/bin/bash
# Alternate libraries on one box: for each round, for each ab/NAME, run the
# given bench workloads (each a quoted argument list).
#   bash tools/ab_run.sh OUT ROUNDS "NAME1 NAME2" "--workload config2r --steps 10" ...
source tools/gpu_guard.sh
O=gpurun_out/$1; R=$2; L=$3; shift 3
mkdir -p $O
for r in $(seq 1 $R); do
  for n in $L; do
    for w in "$@"; do
      echo "== round $r lib $n : $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $w --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
