#!/bin/bash
# Round 5: k_count's grid capped at 2048 / 1024 workgroups (ab/g2048,
# ab/g1024) against 4096 (ab/head).  A K5 fallback list is sized for the
# whole batch, so 4096 mostly-empty workgroups were dispatched per call.
#   bash tools/r05_countgrid.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05cg}; R=${2:-2}; mkdir -p $O
MCRC_LIB=ab/g2048/libmcrc32c.so run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "planned or config3 or pages or stamp or verify or spans" > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head g2048 g1024; do
    for w in "config3" "pagesmix --pages 300" "config5 --pages 300" "stamp --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
