#!/bin/bash
# Quick state check on a fresh box: GPU tests, bench (default and the driver's
# --steps 20 --warmup 5), span workloads.
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r02a}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 300 python bench.py > $O/bench.json 2> $O/bench.err
run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_d.json 2>> $O/bench.err
run 300 python bench.py --workload config3 --steps 5 --warmup 2 > $O/c3.json 2>> $O/bench.err
run 300 python bench.py --workload config2r --steps 10 --warmup 3 > $O/c2r.json 2>> $O/bench.err
run 300 python bench.py --workload config5 --pages 300 --steps 5 --warmup 2 > $O/c5.json 2>> $O/bench.err
echo done
