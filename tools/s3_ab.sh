#!/bin/bash
# GPU tests, then A/B (alternating) of this build against abl/libmcrc32c_$2.so
# on the page workloads at 300 pages.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  for v in cur $2; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    for w in ${WL:-config5 stamp pages}; do
      MCRC_LIB=$lib run 300 python bench.py --workload $w --pages 300 --steps 5 --warmup 2 > $O/${v}_${w}_$i.json 2>>$O/err.log
    done
  done
done
echo done
