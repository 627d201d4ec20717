#!/bin/bash
# Evidence for DESIGN: K1 PMC census (headline) and the calls workload's kernel trace.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3ev}; mkdir -p $O
bash tools/r02_pmc.sh ${1:-s3ev}/pmc config2 cur
run 200 rocprofv3 --kernel-trace --stats -d $O/kt_calls -o kt --output-format csv -- python3 bench.py --workload calls > $O/kt_calls.log 2>&1
echo done
