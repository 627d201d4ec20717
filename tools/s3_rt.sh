#!/bin/bash
# HIP runtime trace of the pages workload (300 pages): where the host time goes.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3rt}; mkdir -p $O
run 300 python bench.py --workload pages --pages 300 --steps 5 --warmup 2 > $O/pages_plain.json 2>> $O/err.log
run 300 rocprofv3 --runtime-trace --stats -d $O/rt -o rt --output-format csv -- python3 bench.py --workload pages --steps 3 --warmup 1 --pages 300 > $O/rt_pages.log 2>&1
echo done
