#!/bin/bash
# bench.py with one event pair per launch vs one around the timed region, alternating on one box
source tools/gpu_guard.sh
O=gpurun_out/${1:-ev}; mkdir -p $O
run 300 python bench.py --no-cpu-baseline > $O/w.json 2>/dev/null
for i in 1 2; do
  run 300 python bench.py --no-cpu-baseline --events launch > $O/l$i.json 2>/dev/null
  run 300 python bench.py --no-cpu-baseline --events region > $O/g$i.json 2>/dev/null
done
(cd tools && run 300 ./ubench 1048576 50 "m13_ftrue_cifalse" 0 2) > $O/ub.log 2>&1
echo done
