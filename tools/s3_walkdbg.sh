#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3wd}; mkdir -p $O
run 300 python tools/walk_check.py 300 $PWD/abl/libmcrc32c_head.so > $O/wc300.log 2>&1
run 300 python tools/walk_check.py 1000 $PWD/abl/libmcrc32c_head.so > $O/wc1000.log 2>&1
run 300 python tools/walk_check.py 300 $PWD/abl/libmcrc32c_head.so > $O/wc300b.log 2>&1
echo done
