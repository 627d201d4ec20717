#!/bin/bash
# One GPU session: parity tests (every failure listed), smoke, the headline
# bench with the driver's arguments, the per-call and multi-device workloads.
#   bash tools/gpu_check.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-check}; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
run 300 python bench.py --workload calls > $O/calls.json 2> $O/calls.err
run 300 python bench.py --workload multi --gpus 1 --steps 20 --warmup 5 > $O/multi.json 2> $O/multi.err
echo done
