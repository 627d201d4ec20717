#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3wd}; mkdir -p $O
run 300 python -u -m pytest tests -x -q -m gpu -k "bench_layout" --timeout 300 --timeout-method thread > $O/pytest_bl.log 2>&1
MCRC_LIB=$PWD/abl/libmcrc32c_broken.so run 300 python -u -m pytest tests -q -m gpu -k "bench_layout" --timeout 300 --timeout-method thread > $O/pytest_bl_broken.log 2>&1
echo done
