#!/bin/bash
# Full-size parity tests (config 3, bench pages) and the config-3 bench line.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-s3fs}; mkdir -p $O
run 600 python -u -m pytest tests -x -v -m gpu -k "config3_full or bench_layout" --timeout 300 --timeout-method thread > $O/pytest_fs.log 2>&1
run 300 python bench.py --workload config3 --steps 5 --warmup 2 > $O/c3.json 2> $O/c3.err
echo done
