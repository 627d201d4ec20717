#!/bin/bash
# parity tests, then the span workloads for the in-tree library vs abl/ variants
source tools/gpu_guard.sh
O=gpurun_out/${1:-ab}; mkdir -p $O; shift
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
grep -q "passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed"; exit 1; }
bash tools/ablate_spans.sh run ${O#gpurun_out/} "$@"
