#!/bin/bash
# k_lines' chunks dealt in a scrambled wave order (k5p) against wave order
# (cur): K5 parity with k5p, A/B on config 2r, config 5 and the stamp.
#   bash tools/r04_k5perm.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/k5p/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "k5 or 4133 or census or async or stamp or verify or pages or items" > $O/pytest_k5p.log 2>&1
tail -1 $O/pytest_k5p.log
grep -q " passed" $O/pytest_k5p.log && ! grep -q "failed" $O/pytest_k5p.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur k5p; do
    for w in config2r config5 stamp; do
      case $w in config2r) a="--workload $w --steps 10 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
