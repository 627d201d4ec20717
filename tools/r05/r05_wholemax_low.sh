#!/bin/bash
# Round 5: spans of virtual length up to 512 / 768 B all k_count's (its
# wave-cooperative 128-B chunks) instead of up to 1024 (ab/w512, ab/w768
# against ab/head).  Planned-path GPU tests with ab/w512 first.
#   bash tools/r05_wholemax.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05wl}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/w512/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "planned or config3 or pages or stamp or verify or spans or golden or fuzz" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head w512 w768; do
    for w in "config3" "pagesmix --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
