#!/bin/bash
# Round 5: K5 (k_lines) windows in K1's coalesced non-temporal layout.
# GPU parity of the new build (every K5 / item / page / stamp test), then an
# interleaved A/B against the previous k_lines (ab/k5old = HEAD before the
# change, ab/k5new = the change) on config 5, config 2r and the stamp.
#   bash tools/r05_k5.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k5}; R=${2:-2}; mkdir -p $O
run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k5 or census or async or stamp or items or pages or config1 or extstore or lines or verify" > $O/pytest_k5.log 2>&1
tail -1 $O/pytest_k5.log
grep -q " passed" $O/pytest_k5.log && ! grep -q "failed" $O/pytest_k5.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in k5old k5new; do
    for w in "config5 --pages 300" "config2r" "stamp --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
