#!/bin/bash
# span-kernel ablations at one span length (config2r --span-len L): time + VALU
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; L=$2; shift 2; mkdir -p $O
for v in "$@"; do
  lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
  MCRC_LIB=$lib run 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/${v}_a -o a --output-format csv -- python3 bench.py --workload config2r --span-len $L --steps 2 --warmup 1 > $O/${v}_a.log 2>&1
  MCRC_LIB=$lib run 120 python bench.py --workload config2r --span-len $L --steps 10 --warmup 3 > $O/${v}.json 2>>$O/err.log
done
echo done
