#!/bin/bash
# bench.py K1 vs ubench K1 back to back on one box (clock/power comparison)
source tools/gpu_guard.sh
O=gpurun_out/${1:-cmp}; mkdir -p $O
run 300 python bench.py --no-cpu-baseline > $O/b1.json 2>/dev/null
run 300 python bench.py --no-cpu-baseline > $O/b2.json 2>/dev/null
(cd tools && run 300 ./ubench 1048576 20 "m13_ftrue_cifalse" 0 3) > $O/ub.log 2>&1
run 300 python bench.py --no-cpu-baseline --steps 100 > $O/b3.json 2>/dev/null
echo done
