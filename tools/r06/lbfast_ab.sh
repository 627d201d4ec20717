#!/bin/bash
# Round 6: k_spans' load_block with one address and immediate offsets for
# blocks whose pieces are all real (ab/lbfast) against the product (ab/cur):
# span parity tests on the variant, then config 3 and the mixed pages, alternating.
#   bash tools/r06/lbfast_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_lb}; R=${2:-3}
mkdir -p $O
MCRC_LIB=ab/lbfast/libmcrc32c.so run 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "span or config3 or planned or unaligned or pages or zipf" > $O/pytest_lb.log 2>&1
tail -1 $O/pytest_lb.log
for r in $(seq 1 $R); do
  for n in cur lbfast; do
    for w in "config3 --steps 10 --warmup 2" "pagesmix --pages 1000 --steps 5 --warmup 1"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
