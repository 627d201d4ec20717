#!/bin/bash
# Round 5: plan rounds, second build (empty rounds skipped) against ab/head;
# then a kernel trace of the mixed pages at 1000 pages with each build.
#   bash tools/r05_rounds2.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05rd2}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/rounds/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "planned or config3 or pages or stamp or verify or spans or golden or fuzz" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head rounds; do
    for w in "pagesmix --pages 300" "config3" "config5 --pages 300" "stamp --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
for n in head rounds; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload pagesmix --pages 1000 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_$n.json 2> $O/kt_$n.err
done
echo done
