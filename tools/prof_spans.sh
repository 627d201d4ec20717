#!/bin/bash
# Per-kernel split of the span workloads (config 3 / config 5).
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-ps}; mkdir -p $O
run 600 rocprofv3 --kernel-trace --stats -d $O/c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages ${PAGES:-200} --steps 3 --warmup 1 > $O/c5.log 2>&1
run 600 rocprofv3 --kernel-trace --stats -d $O/c3 -o c3 --output-format csv -- python3 bench.py --workload config3 --steps 3 --warmup 1 > $O/c3.log 2>&1
echo done
