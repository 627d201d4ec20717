#!/bin/bash
# A/B of library builds on the mixed-size pages workload, alternating on one box.
#   bash tools/r02_mix_ab.sh OUT PAGES cur NAME...   (NAME = abl/libmcrc32c_NAME.so)
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; P=$2; shift 2; mkdir -p $O
for i in 1 2; do
  for v in "$@"; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --workload pagesmix --pages $P --steps 5 --warmup 2 > $O/${v}_mix_$i.json 2>>$O/err.log
  done
done
echo done
