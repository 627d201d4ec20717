#!/bin/bash
# Round 5: the prefetches past a wave's last K1 group and past each K5 run
# read cache-resident buffers (the table image / the zero slot) instead of
# re-fetching the last window from HBM (ab/ovf = the working tree) against
# the committed build (ab/head).  GPU parity first, then timings and the
# FETCH_SIZE of both K1 builds on the headline batch.
#   bash tools/r05_ovf.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ovf}; R=${2:-3}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head ovf; do
    echo "== round $r lib $n workload headline" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    for w in "config5 --pages 300" "stamp --pages 300" "config2r"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
for n in head ovf; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$n -o f --output-format csv -- python3 bench.py --steps 2 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch_$n.log 2>&1
  MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch5_$n -o f --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch5_$n.log 2>&1
done
echo done
