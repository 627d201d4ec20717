#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c}; mkdir -p $O
run 600 bash tools/queue_runs.sh $O/queue.txt
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_hazard.hip -o /tmp/walk_hazard && run 300 /tmp/walk_hazard 300 3 > $O/walk_hazard.txt 2>&1
run 1200 bash tools/profile_round.sh r03c/prof
echo done
