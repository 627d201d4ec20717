#!/bin/bash
# kernel split of the pages workload (device walk + verify), previous vs current library
source tools/gpu_guard.sh
export TMPDIR=/tmp
run 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${1:-profwalk}_pytest.log 2>&1
grep -q "passed" gpurun_out/${1:-profwalk}_pytest.log && ! grep -q "failed" gpurun_out/${1:-profwalk}_pytest.log || { echo "tests failed"; exit 1; }
O=gpurun_out/${1:-profwalk}; mkdir -p $O
MCRC_LIB=$PWD/abl/libmcrc32c_prev.so run 300 rocprofv3 --kernel-trace --stats -d $O/prev -o prev --output-format csv -- python3 bench.py --workload pages --pages 300 --steps 3 --warmup 1 > $O/prev.json 2> $O/prev.err
run 300 rocprofv3 --kernel-trace --stats -d $O/cur -o cur --output-format csv -- python3 bench.py --workload pages --pages 300 --steps 3 --warmup 1 > $O/cur.json 2> $O/cur.err
echo done
