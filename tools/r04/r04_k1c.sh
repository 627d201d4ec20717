#!/bin/bash
# K1 with each wave on a contiguous range of items (k1c) against the
# grid-stride order (cur): K1 parity with k1c, headline A/B (and 4 Mi items),
# then the K5 routing A/B (tools/r04_census.sh).
#   bash tools/r04_k1c.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/k1c/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k1 or fixed or golden or fuzz or config2 or multi or bench" > $O/pytest_k1c.log 2>&1
tail -1 $O/pytest_k1c.log
grep -q " passed" $O/pytest_k1c.log && ! grep -q "failed" $O/pytest_k1c.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur k1c; do
    echo "== round $r lib $n headline" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    echo "== round $r lib $n headline4mi" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --items 4194304 >> $O/ab.txt 2>> $O/ab.err
  done
done
MCRC_LIB=ab/k1c/libmcrc32c.so run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_k1c -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch_k1c.log 2>&1
bash tools/r04_census.sh $1 2 || exit 1
echo all done
