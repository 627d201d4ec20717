#!/bin/bash
source tools/gpu_guard.sh
O=gpurun_out/${1:-r03d}; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_hazard.hip -o /tmp/walk_hazard && run 300 /tmp/walk_hazard 300 2 > $O/walk_hazard.txt 2>&1
echo done
