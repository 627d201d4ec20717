#!/bin/bash
# A/B (alternating) of builds on one workload at 300 pages: bash tools/s3_ab3.sh OUT WORKLOAD cur NAME...
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; w=$2; shift 2; mkdir -p $O
for i in 1 2 3; do
  for v in "$@"; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --workload $w --pages 300 --steps 5 --warmup 2 > $O/${v}_${w}_$i.json 2>>$O/err.log
  done
done
echo done
