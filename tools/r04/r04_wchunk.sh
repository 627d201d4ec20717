#!/bin/bash
# k_count's whole-span chunks of 4 (cur), 8 (w8) and 16 (w16) pieces: fewer
# chunks, fewer x^(8n) multiplies, longer lane chains.  Parity, A/B, traces.
#   bash tools/r04_wchunk.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; mkdir -p $O
for n in w8 w16; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x -k "config3 or spans or verify or pages or golden or fuzz or items" > $O/pytest_$n.log 2>&1
  tail -1 $O/pytest_$n.log
  grep -q " passed" $O/pytest_$n.log && ! grep -q "failed" $O/pytest_$n.log || { echo "tests failed ($n), stopping"; exit 1; }
done
for r in $(seq 1 $R); do
  for n in cur w8 w16; do
    for w in pagesmix config3; do
      case $w in config3) a="--workload $w --steps 5 --warmup 2";; *) a="--workload $w --pages 300 --steps 5 --warmup 1";; esac
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py $a >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
for n in cur w8 w16; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload pagesmix --pages 300 --steps 3 --warmup 1 > $O/kt_$n.log 2>&1
done
echo done
