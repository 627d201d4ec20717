#!/bin/bash
# GPU tests + the headline bench with the driver's arguments.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r02b}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench_d.json 2> $O/bench.err
run 300 python bench.py --steps 20 --warmup 5 --settle-ms 0 --no-cpu-baseline > $O/bench_d0.json 2>> $O/bench.err
echo done
