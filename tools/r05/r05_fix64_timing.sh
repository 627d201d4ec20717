#!/bin/bash
# Round 5, timing only: k_fix rewriting the whole 64-B chunk that holds each
# stamp (read, patch, write; ab/fix64, unguarded against two stamps in one
# chunk, so no tests) against the shipped four byte stores (ab/head).
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/r05f64; mkdir -p $O
for r in 1 2 3; do
  for n in head fix64; do
    echo "== round $r lib $n workload stamp --pages 300" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload stamp --pages 300 --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
for n in head fix64; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload stamp --pages 300 --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$n.json 2> $O/kt_$n.err
done
echo done
