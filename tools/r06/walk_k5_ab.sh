#!/bin/bash
# Round 6: the one-pass walk (K5 inside the walk, k_lines<1, true, true>):
# the walk / verify_pages GPU tests through all three walk modes, a
# same-session A/B of crc32c_verify_pages (walk mode 0 = the two-pass walk,
# 1 = the default: one pass over whole rounds of wbufs for pages of
# one-block items) on config 5's pages (1000 and 300) and the mixed pages,
# config 5's item list as the floor, and a kernel trace of the default.
#   bash tools/r06/walk_k5_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_wk5}; R=${2:-2}
mkdir -p $O
run 900 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "walk or verify_pages or alignment" > $O/pytest_walk.log 2>&1
tail -1 $O/pytest_walk.log
for r in $(seq 1 $R); do
  for p in 1000 300; do
    for m in 0 1; do
      echo "== round $r walk mode $m workload pages $p" >> $O/ab.txt
      run 300 python bench.py --workload pages --walk-mode $m --pages $p --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
  for m in 0 1; do
    echo "== round $r walk mode $m workload pagesmixwalk 1000" >> $O/ab.txt
    run 300 python bench.py --workload pagesmixwalk --walk-mode $m --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
  echo "== round $r workload config5 1000" >> $O/ab.txt
  run 300 python bench.py --workload config5 --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run 300 rocprofv3 --kernel-trace --stats -d $O/prof -o pages --output-format csv -- python bench.py --workload pages --pages 1000 --steps 5 --no-cpu-baseline > $O/prof.log 2>&1
echo done
