#!/bin/bash
# Round 6: K5's finish with table operators (cur) against two bitwise
# multiplies per image (HEAD): the full GPU suite on cur, then the K5
# workloads alternating.
#   bash tools/r06/k5_finish_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_k5f}; R=${2:-3}
mkdir -p $O
run 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    for w in "config5 --pages 1000 --steps 5 --warmup 1" "config2r --steps 20 --warmup 5" "stamp --pages 1000 --steps 3 --warmup 1"; do
      echo "== round $r lib $n workload $w" >> $O/ab.txt
      MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --workload $w --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
    done
  done
done
echo done
