#!/bin/bash
# headline bench with the previous library (abl/libmcrc32c_prev.so) vs the current one, alternating
source tools/gpu_guard.sh
O=gpurun_out/${1:-abb}; mkdir -p $O
for i in 1 2 3; do
  MCRC_LIB=$PWD/abl/libmcrc32c_prev.so run 300 python bench.py --no-cpu-baseline > $O/prev_$i.json 2>/dev/null
  run 300 python bench.py --no-cpu-baseline > $O/cur_$i.json 2>/dev/null
done
echo done
