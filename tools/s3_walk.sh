#!/bin/bash
# Two-pass wave walk: GPU tests, the pages workload (1000 pages), its kernel split.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3walk}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 300 python tools/walk_check.py 1000 $PWD/abl/libmcrc32c_head.so > $O/wc1000.log 2>&1
run 300 python bench.py --workload pages --pages 1000 --steps 3 --warmup 1 > $O/pages.json 2> $O/pages.err
MCRC_LIB=$PWD/abl/libmcrc32c_head.so run 300 python bench.py --workload pages --pages 1000 --steps 3 --warmup 1 > $O/pages_head.json 2>> $O/pages.err
run 200 rocprofv3 --kernel-trace --stats -d $O/kt_pages -o kt --output-format csv -- python3 bench.py --workload pages --steps 3 --warmup 1 --pages 300 > $O/kt_pages.log 2>&1
echo done
