#!/bin/bash
# The walk experiment of DESIGN.md section 3 (SGPR vs VGPR walk state, wait
# states, co-resident workgroups) on one GPU.
#   bash tools/walk_hazard.sh OUT [PAGES] [REPS]
source tools/gpu_guard.sh
O=gpurun_out/${1:-walk}; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_hazard.hip -o /tmp/walk_hazard &&
    run 400 /tmp/walk_hazard ${2:-300} ${3:-2} > $O/walk_hazard.txt 2>&1
