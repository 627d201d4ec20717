#!/bin/bash
# kernel trace of the 1000-page walk + verify and of config 5 (host offsets)
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-pages1000}; mkdir -p $O
run 300 rocprofv3 --kernel-trace -d $O/pages -o pages --output-format csv -- python3 bench.py --workload pages --pages 1000 --steps 3 --warmup 1 > $O/pages.json 2> $O/pages.err
run 300 rocprofv3 --kernel-trace -d $O/c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages 1000 --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err
echo done
