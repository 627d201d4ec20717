#!/bin/bash
# Round 5: the head-fragment limit kFragMax (a head fragment [p, G1) of at
# most this is k_count's, serially in the span's thread) at 0 / 32 / 64
# against 128 (ab/f0, ab/f32, ab/f64, ab/head).  Planned-path GPU tests with
# ab/f0 first.
#   bash tools/r05_fragmax.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05fm}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/f0/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "planned or config3 or pages or stamp or verify or spans or golden or fuzz" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head f0 f32 f64; do
    for w in "config3" "pagesmix --pages 300" "config5 --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
