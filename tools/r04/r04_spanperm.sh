#!/bin/bash
# The balanced plan's shares dealt to the span kernel's groups in a scrambled
# order (sp) against in group order (cur): planned-path parity with sp, A/B.
#   bash tools/r04_spanperm.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/sp/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "config3 or spans or verify or pages or overlap or long or fuzz or balance or golden" > $O/pytest_sp.log 2>&1
tail -1 $O/pytest_sp.log
grep -q " passed" $O/pytest_sp.log && ! grep -q "failed" $O/pytest_sp.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur sp; do
    for w in config3 pagesmix; do
      case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
