#!/bin/bash
# Round 6: verify_pages by walk mode (0 two-pass, 1 default, 2 one-pass over
# every wbuf) and page count, same session.
#   bash tools/r06/walk_k5_modes.sh OUT ROUNDS "PAGES..." "MODES..."
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_wk5m}; R=${2:-2}; P=${3:-"1000 1024 300"}; M=${4:-"0 2"}
mkdir -p $O
for r in $(seq 1 $R); do
  for p in $P; do
    for m in $M; do
      echo "== round $r walk mode $m workload pages $p" >> $O/ab.txt
      run 300 python bench.py --workload pages --walk-mode $m --pages $p --steps 5 --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
