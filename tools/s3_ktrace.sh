#!/bin/bash
# Per-kernel durations (rocprofv3 --kernel-trace --stats) of the page workloads
# (stamp, device walk + verify, mixed pages) at 300 pages.
#   bash tools/s3_ktrace.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for w in ${WL:-stamp pages pagesmix}; do
  run 200 rocprofv3 --kernel-trace --stats -d $O/$w -o kt --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --pages 300 > $O/$w.log 2>&1
done
echo done
