#!/bin/bash
# K1 MODE 14: last-prefetch clamp to the batch's last group (old) vs the wave's own last group
source tools/gpu_guard.sh
O=gpurun_out/${1:-clamp}; mkdir -p $O
cd tools
for i in 1 2 3; do
  run 120 ./ubench_oldclamp 1048576 50 "m14_ftrue_cifalse" 0 1 >> ../$O/old.log 2>&1
  run 120 ./ubench 1048576 50 "m14_ftrue_cifalse" 0 1 >> ../$O/new.log 2>&1
done
echo done
