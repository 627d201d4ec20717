#!/bin/bash
# Per-kernel durations (rocprofv3 --kernel-trace --stats) of the span workloads.
#   bash tools/r02_ktrace.sh OUT [lib]
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
lib=; [ -n "$2" ] && lib=$PWD/abl/libmcrc32c_$2.so
for w in config2r config3 config5; do
  MCRC_LIB=$lib run 200 rocprofv3 --kernel-trace --stats -d $O/$w -o kt --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 2 --pages 300 > $O/$w.log 2>&1
done
echo done
