#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r03b}; mkdir -p $O
run 600 python -u -m pytest tests/test_gpu_items_queue.py tests/test_integration.py -v -s -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_new.log 2>&1
run 600 bash tools/queue_runs.sh $O/queue.txt
run 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_hazard.hip -o /tmp/walk_hazard && run 300 /tmp/walk_hazard 300 3 > $O/walk_hazard.txt 2>&1
echo done
