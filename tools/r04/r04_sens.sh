#!/bin/bash
# K1 sensitivity (+VALU / +LDS ablations) and K5 ablations, one box.
#   bash tools/r04_sens.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for r in $(seq 1 $R); do
  for n in base sens1 sens2; do
    echo "== round $r lib $n workload config2" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
bash tools/r04_k5abl.sh $1 $R "base k5a1 k5a2 k5a3 k5rl"
