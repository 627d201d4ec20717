#!/bin/bash
# Round 6: the speculative page walk (MCRC_WALK_SPEC=1, the default) against
# the two-pass walk (0), same library: the walk / verify_pages GPU tests, then
# config 5's pages (1000, 300) and the mixed pages, alternating, and a kernel
# trace of the speculative run.
#   bash tools/r06/walk_spec_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_spec}; R=${2:-3}
mkdir -p $O
run 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "walk or verify_pages or alignment" > $O/pytest_walk.log 2>&1
tail -1 $O/pytest_walk.log
for r in $(seq 1 $R); do
  for p in 1000 300; do
    for s in 0 1; do
      echo "== round $r spec $s workload pages $p" >> $O/ab.txt
      MCRC_WALK_SPEC=$s run 300 python bench.py --workload pages --pages $p --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
  for s in 0 1; do
    echo "== round $r spec $s workload pagesmixwalk 1000" >> $O/ab.txt
    MCRC_WALK_SPEC=$s run 300 python bench.py --workload pagesmixwalk --pages 1000 --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --workload pages --pages 1000 --steps 3 --warmup 1 --no-cpu-baseline > $O/kt.json 2> $O/kt.err
echo done
