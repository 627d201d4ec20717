#!/bin/bash
# Round 6 review item 3: the in-kernel stamp (k_lines<2> stores the CRC and
# ok itself: lnst = non-temporal byte stores, lnc = default-policy byte
# stores) against the shipped k_lines<2> + k_fix (cur), same session.  First
# the stamp tests on each variant (ok flags included), then ROUNDS
# alternating rounds of the 1000-page stamp (the bench requests no ok flags,
# so every variant does the same work: one stamp per image).
#   bash tools/r06/stamp_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/$1; R=${2:-3}
mkdir -p $O
for n in lnst lnc; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 python -u -m pytest tests/test_gpu_items_queue.py tests/test_gpu_parity.py -q \
      -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
      -k "stamp or alignment or k5_verify_stamp" > $O/pytest_$n.log 2>&1
  tail -1 $O/pytest_$n.log
done
for r in $(seq 1 $R); do
  for n in cur lnst lnc; do
    echo "== round $r lib $n" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload stamp --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
echo done
