#!/bin/bash
# K1 headline A/B, alternating builds: bash tools/s3_k1ab.sh OUT cur NAME...
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for i in 1 2 3 4; do
  for v in "$@"; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${v}_k1_$i.json 2>>$O/err.log
  done
done
echo done
