#!/bin/bash
# A/B of library builds on the span workloads (and K1), alternating on one box.
#   bash tools/r02_ab.sh OUT cur NAME...   (NAME = abl/libmcrc32c_NAME.so; cur = the in-tree library)
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for i in 1 2; do
  for v in "$@"; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --workload config2r --steps 10 --warmup 3 > $O/${v}_c2r_$i.json 2>>$O/err.log
    MCRC_LIB=$lib run 300 python bench.py --workload config3 --steps 5 --warmup 2 > $O/${v}_c3_$i.json 2>>$O/err.log
    MCRC_LIB=$lib run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/${v}_c5_$i.json 2>>$O/err.log
  done
done
echo done
