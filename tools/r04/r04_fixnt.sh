#!/bin/bash
# The stamp's k_fix: plain stores (cur), non-temporal stores (ntfix), and no
# k_fix at all (nofix: wrong results, timing only -- what the stores cost
# k_fix and the next k_lines<2>).  Stamp parity with ntfix, A/B, traces.
#   bash tools/r04_fixnt.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/ntfix/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "stamp or k5 or extstore or config1" > $O/pytest_ntfix.log 2>&1
tail -1 $O/pytest_ntfix.log
grep -q " passed" $O/pytest_ntfix.log && ! grep -q "failed" $O/pytest_ntfix.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur ntfix nofix; do
    echo "== round $r lib $n workload stamp" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload stamp --pages 300 --steps 5 --warmup 1 >> $O/ab.txt 2>> $O/ab.err
  done
done
for n in cur ntfix nofix; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload stamp --pages 300 --steps 3 --warmup 1 > $O/kt_$n.log 2>&1
done
echo done
