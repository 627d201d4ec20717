#!/bin/bash
# Round 5: K1 with a ring of four half-step buffers (loads three half-steps
# ahead, 12 KiB per wave in flight; ab/k1h = the working tree) against the
# committed K1 (one whole step ahead, 8 KiB; ab/head).  GPU parity first.
#   bash tools/r05_k1h.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k1h}; R=${2:-4}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head k1h; do
    echo "== round $r lib $n" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
echo done
