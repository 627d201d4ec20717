#!/bin/bash
# GPU tests, then the per-call latency workload, alternating with abl/libmcrc32c_$2.so.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2 3; do
  for v in cur $2; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --workload calls > $O/${v}_calls_$i.json 2>>$O/err.log
  done
done
echo done
