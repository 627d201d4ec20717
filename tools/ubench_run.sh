#!/bin/bash
# ubench variants (tools/ubench, built with -DMCRC_UBENCH_CLOCK): bash tools/ubench_run.sh <outdir> [filter]
source tools/gpu_guard.sh
O=gpurun_out/${1:-ub}; mkdir -p $O
cd tools
run 300 ./ubench 1048576 20 "$2" 0 ${3:-1} > ../$O/ubench.log 2>&1
echo done
