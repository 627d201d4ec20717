#!/bin/bash
# K1 ranges dealt to the waves in a scrambled order (perm) against in wave
# order (cur): K1 parity with perm, headline A/B at 1 and 4 Mi items.
#   bash tools/r04_perm.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/perm/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k1 or fixed or golden or fuzz or config2 or multi or bench" > $O/pytest_perm.log 2>&1
tail -1 $O/pytest_perm.log
grep -q " passed" $O/pytest_perm.log && ! grep -q "failed" $O/pytest_perm.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur perm; do
    echo "== round $r lib $n headline" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    echo "== round $r lib $n headline4mi" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --items 4194304 >> $O/ab.txt 2>> $O/ab.err
  done
done
echo done
