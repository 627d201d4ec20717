#!/bin/bash
# Round 5: K5's runs dealt round robin over the waves (ab/rr: run k of wave
# w = images (k W + w) 2 nsr ..., so the waves' windows stay within ~1 GB of
# each other) against each wave's contiguous chunk (ab/head), at 300 and
# 1000 pages (the 1000-page batches ran 3-5 % slower per page).  K5 parity
# tests with ab/rr first.
#   bash tools/r05_k5order.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k5o}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/rr/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "k5 or lines or verify or stamp or config2 or pages" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head rr; do
    for w in "config5 --pages 1000" "config5 --pages 300" "config2r"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
