#!/bin/bash
# K1 item order: grid-stride (cur), a contiguous range per wave (k1c), a
# contiguous range per workgroup with its waves interleaved (k1w).
#   bash tools/r04_k1w.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/k1w/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k1 or fixed or golden or fuzz or config2 or multi or bench" > $O/pytest_k1w.log 2>&1
tail -1 $O/pytest_k1w.log
grep -q " passed" $O/pytest_k1w.log && ! grep -q "failed" $O/pytest_k1w.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur k1c k1w; do
    echo "== round $r lib $n headline" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    echo "== round $r lib $n headline4mi" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --items 4194304 >> $O/ab.txt 2>> $O/ab.err
  done
done
echo done
