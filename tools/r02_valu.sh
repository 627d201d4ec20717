#!/bin/bash
# VALU / LDS instruction counts and time of the span kernel per library (config2r).
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; W=$2; shift 2; mkdir -p $O
for v in "$@"; do
  lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
  MCRC_LIB=$lib run 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/${v}_a -o a --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --pages 100 > $O/${v}_a.log 2>&1
  MCRC_LIB=$lib run 120 python bench.py --workload $W --steps 10 --warmup 3 --pages 300 > $O/${v}.json 2>>$O/err.log
done
echo done
