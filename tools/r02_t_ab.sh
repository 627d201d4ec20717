#!/bin/bash
# GPU tests, then an A/B of the in-tree library against abl/libmcrc32c_NAME.so.
#   bash tools/r02_t_ab.sh OUT NAME
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
bash tools/r02_ab.sh $1 cur $2
