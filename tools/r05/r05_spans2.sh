#!/bin/bash
# Round 5: the span kernels' pieces layout with the default load policy
# (ab/pdflt) against the previous build (ab/head) on the planned-path
# workloads, after the planned-path GPU tests of pdflt.
#   bash tools/r05_spans2.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05sp2}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/pdflt/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "span or planned or config3 or blocks or small or fuzz or golden or pages or chain" > $O/pytest_pdflt.log 2>&1
tail -1 $O/pytest_pdflt.log
for r in $(seq 1 $R); do
  for n in head pdflt; do
    for w in "config3" "pagesmix --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
