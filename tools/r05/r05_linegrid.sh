#!/bin/bash
# Round 5: the planned path's grid anchored on 128-B lines (every unit block
# whole lines; the span's thread folds up to 127 foreign tail bytes) with the
# span kernels on K1's pieces layout: nt loads (ab/lgnt) and default policy
# (ab/lgdflt), against the shipped build (ab/head).  Full GPU parity with
# lgnt first.
#   bash tools/r05_linegrid.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05lg}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/lgnt/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_lgnt.log 2>&1
tail -1 $O/pytest_lgnt.log
grep -q " passed" $O/pytest_lgnt.log && ! grep -q "failed" $O/pytest_lgnt.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head lgnt lgdflt; do
    for w in "config3" "pagesmix --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
