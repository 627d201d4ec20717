#!/bin/bash
# Round 5: k_small issues its offset / header / block / Z-piece loads before
# the 160 KiB table fill (ab/ksm = the working tree) against the committed
# build (ab/head).  GPU parity first, then the small-call latencies and a
# kernel trace of each build.
#   bash tools/r05_ksmall.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ks}; R=${2:-3}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head ksm; do
    echo "== round $r lib $n workload calls" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload calls >> $O/ab.txt 2>> $O/ab.err
  done
done
for n in head ksm; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload calls > $O/kt_$n.json 2> $O/kt_$n.err
done
echo done
