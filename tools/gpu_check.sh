#!/bin/bash
# One GPU session: parity tests, smoke, bench (each step under its own limit).
source tools/gpu_guard.sh
O=gpurun_out/${1:-check}; mkdir -p $O
run 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1
run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 600 python bench.py > $O/bench.json 2> $O/bench.err
echo done
