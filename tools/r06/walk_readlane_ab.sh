#!/bin/bash
# Round 6: the walk's broadcast of lane m's flag and size by v_readlane
# (scalar walk state, cur) against ds_bpermute (HEAD): walk / verify_pages
# GPU tests, small planned page verifies (per-call wall), and the 1000-page
# walk workloads, alternating.
#   bash tools/r06/walk_readlane_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_rl}; R=${2:-2}
mkdir -p $O
run 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "walk or verify_pages or alignment or planned_rounds" > $O/pytest_walk.log 2>&1
tail -1 $O/pytest_walk.log
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python tools/r06/pages_small_ab.py >> $O/small.jsonl 2>> $O/ab.err
    for w in pagesmixwalk pages; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
