#!/bin/bash
# Span kernels: GPU parity tests, then the span workloads for the current
# library and the previous one (abl/libmcrc32c_prev.so) alternating.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed\|error" $O/pytest_gpu.log || { echo "tests failed"; exit 1; }
for i in 1 2; do
  for v in cur prev; do
    lib=; [ $v = prev ] && lib=$PWD/abl/libmcrc32c_prev.so
    MCRC_LIB=$lib run 300 python bench.py --workload config2r --steps 10 --warmup 3 > $O/${v}_c2r_$i.json 2>/dev/null
    MCRC_LIB=$lib run 300 python bench.py --workload config3 --steps 5 --warmup 2 > $O/${v}_c3_$i.json 2>/dev/null
    MCRC_LIB=$lib run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/${v}_c5_$i.json 2>/dev/null
  done
done
echo done
