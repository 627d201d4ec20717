#!/bin/bash
# GPU tests, then A/B (alternating) of this build against abl/libmcrc32c_$2.so:
# headline K1, per-call latency, config 2 variant, config 3, config 5 (300 pages).
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2 3; do
  for v in cur $2; do
    lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
    MCRC_LIB=$lib run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${v}_k1_$i.json 2>>$O/err.log
    MCRC_LIB=$lib run 300 python bench.py --workload calls > $O/${v}_calls_$i.json 2>>$O/err.log
    MCRC_LIB=$lib run 300 python bench.py --workload config2r --steps 10 --warmup 3 > $O/${v}_c2r_$i.json 2>>$O/err.log
    MCRC_LIB=$lib run 300 python bench.py --workload config3 --steps 5 --warmup 2 > $O/${v}_c3_$i.json 2>>$O/err.log
    MCRC_LIB=$lib run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/${v}_c5_$i.json 2>>$O/err.log
  done
done
echo done
