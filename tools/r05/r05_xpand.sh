#!/bin/bash
# Round 5: k_expand writes the inline units of its spans with the whole
# wave (ab/xpand = the working tree) against the committed build (ab/head).
# GPU parity first.
#   bash tools/r05_xpand.sh OUT ROUNDS
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05xp}; R=${2:-2}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
tail -1 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || { echo "tests failed, stopping"; exit 1; }
for r in $(seq 1 $R); do
  for n in head xpand; do
    for w in "config3" "pagesmix --pages 300" "config5 --pages 300"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done

for n in head xpand; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$n.json 2> $O/kt_$n.err
done
echo done
