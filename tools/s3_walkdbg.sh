#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3wd}; mkdir -p $O
run 300 python -u -m pytest tests -x -q -m gpu -k "walk or pages" --timeout 300 --timeout-method thread > $O/pytest_walk.log 2>&1
echo done
