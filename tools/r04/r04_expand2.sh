#!/bin/bash
# The planned path behind a K5 verify (its fallback list, counted on the
# device): cur against cap (plan grids of a device-counted list capped at 256
# workgroups) and inl8 (spans of more than 8 segments expanded by
# k_expand_big); parity subset first, A/B, kernel traces of config 5.
#   bash tools/r04_expand2.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for n in cap inl8; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "config3 or spans or verify or pages or k5 or census or overlap or long" > $O/pytest_$n.log 2>&1
  tail -1 $O/pytest_$n.log
  grep -q " passed" $O/pytest_$n.log && ! grep -q "failed" $O/pytest_$n.log || { echo "tests failed ($n), stopping"; exit 1; }
done
for r in $(seq 1 $R); do
  for n in cur cap inl8; do
    for w in config5 config3 pagesmix; do
      case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
for n in cur cap inl8; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 3 --warmup 1 > $O/kt_$n.log 2>&1
done
echo done
