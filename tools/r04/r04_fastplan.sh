#!/bin/bash
# The planned path with the plan divisions in 32 bits and short block shifts as table steps (fast)
# planned-path parity with fast, A/B on config 3 and the mixed pages, traces.
#   bash tools/r04_fastplan.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
MCRC_LIB=ab/fast/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "config3 or spans or verify or pages or overlap or long or fuzz or balance" > $O/pytest_fast.log 2>&1
tail -1 $O/pytest_fast.log
grep -q " passed" $O/pytest_fast.log && ! grep -q "failed" $O/pytest_fast.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in cur fast; do
    for w in config3 pagesmix; do
      case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab_div.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab_div.txt 2>> $O/ab_div.err
    done
  done
done
for n in cur fast; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/ktd_$n -o kt --output-format csv -- python3 bench.py --workload config3 --steps 5 --warmup 2 > $O/ktd_$n.log 2>&1
done
echo div done
