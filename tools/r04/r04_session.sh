#!/bin/bash
# Full GPU parity of the current library, then the A/B of tools/r04_ab.sh.
#   bash tools/r04_session.sh OUT ROUNDS "libs" "workloads"
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
run 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -x > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
bash tools/r04_ab.sh $1 "$2" "$3" "$4"
