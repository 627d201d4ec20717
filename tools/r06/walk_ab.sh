#!/bin/bash
# Round 6: K1 by waves per CU, the walk tests on the G = 4 count walk, and a
# same-session A/B of the device walk + verify (HEAD = one guess per lane,
# cur = four in the count pass) on config 5's pages and on the mixed pages.
#   bash tools/r06/walk_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_walk}; R=${2:-2}
mkdir -p $O
run 300 tools/k1_waves 30 > $O/k1_waves.txt 2>&1
run 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_items_queue.py -q -m gpu --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "walk or verify_pages or alignment" > $O/pytest_walk.log 2>&1
tail -1 $O/pytest_walk.log
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    for w in pages pagesmixwalk; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
