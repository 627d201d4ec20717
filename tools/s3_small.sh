#!/bin/bash
# k_small workgroup size: GPU tests, then the calls workload per spans-per-workgroup.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3small}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  for p in 32 16 8 4 2; do
    MCRC_SMALL_SPANS=$p run 300 python bench.py --workload calls > $O/calls_p${p}_$i.json 2>>$O/err.log
  done
  run 300 python bench.py --workload calls > $O/calls_def_$i.json 2>>$O/err.log
done
echo done
