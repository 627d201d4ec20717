#!/bin/bash
# k_count with wave-cooperative whole spans (whole) against one thread per
# whole span (cur): planned-path parity subset with whole first, then A/B on
# the mixed pages and config 3, and kernel traces.
#   bash tools/r04_whole.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for n in whole; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "golden or config3 or spans or verify or pages or fuzz or stamp or chain" > $O/pytest_$n.log 2>&1
  tail -1 $O/pytest_$n.log
  grep -q " passed" $O/pytest_$n.log && ! grep -q "failed" $O/pytest_$n.log || { echo "tests failed ($n), stopping"; exit 1; }
done
for r in $(seq 1 $R); do
  for n in cur whole; do
    for w in pagesmix config3; do
      case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
for n in cur whole; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload pagesmix --pages 300 --steps 3 --warmup 1 > $O/kt_$n.log 2>&1
done
echo done
