#!/bin/bash
# Round 6 review item 2: the span kernel on a ring of four half blocks (three
# in flight) against round 5's two whole blocks (HEAD).  The full GPU suite on
# the new kernel first, then ROUNDS alternating rounds of config 3 (1 Mi Zipf
# spans), the mixed pages and config 5 at 1000 pages.
#   bash tools/r06/spans_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_spans}; R=${2:-2}
mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " failed" $O/pytest.log && exit 1
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    for w in "--workload config3" "--workload pagesmix --pages 1000" "--workload config5 --pages 1000"; do
      echo "== round $r lib $n : $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $w --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
