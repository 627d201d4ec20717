#!/bin/bash
# GPU tests, then the device page walk + verify (pages workload) with the
# previous library (abl/libmcrc32c_prev.so) vs the current one, alternating
source tools/gpu_guard.sh
O=gpurun_out/${1:-abwalk}; mkdir -p $O
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
grep -q "passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
for i in 1 2; do
  MCRC_LIB=$PWD/abl/libmcrc32c_prev.so run 300 python bench.py --workload pages --pages ${PAGES:-1000} --steps 3 --warmup 1 > $O/prev_pages_$i.json 2>/dev/null
  run 300 python bench.py --workload pages --pages ${PAGES:-1000} --steps 3 --warmup 1 > $O/cur_pages_$i.json 2>/dev/null
done
echo done
