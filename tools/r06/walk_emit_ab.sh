#!/bin/bash
# Round 6: planned page verifies with the count pass's slots copied and
# k_count reading the headers in parallel (cur) against the emit pass walking
# again and writing k_count's entries (HEAD): the walk / verify_pages GPU
# tests, then a same-session A/B on the mixed pages (planned) and config 5's
# pages (K5 route, unchanged), and a kernel trace of the mixed pages.
#   bash tools/r06/walk_emit_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_emit}; R=${2:-3}
mkdir -p $O
run 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "walk or verify_pages or alignment" > $O/pytest_walk.log 2>&1
tail -1 $O/pytest_walk.log
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    for w in pagesmixwalk pages; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for n in HEAD cur; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python bench.py --workload pagesmixwalk --pages 1000 --steps 5 --no-cpu-baseline > $O/kt_$n.log 2>&1
done
echo done
