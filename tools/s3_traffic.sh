#!/bin/bash
# HBM traffic of the span workloads: separate --pmc passes (FETCH_SIZE, WRITE_SIZE).
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3tr}; mkdir -p $O
for w in config3 config5; do
  run 120 rocprofv3 --pmc FETCH_SIZE -d $O/${w}_fetch -o fetch --output-format csv -- python3 bench.py --workload $w --pages 300 --steps 2 --warmup 1 > $O/${w}_fetch.log 2>&1
  run 120 rocprofv3 --pmc WRITE_SIZE -d $O/${w}_write -o write --output-format csv -- python3 bench.py --workload $w --pages 300 --steps 2 --warmup 1 > $O/${w}_write.log 2>&1
done
echo done
