#!/bin/bash
# The reduced 24-VGPR walk reproducer (tools/walk_vgpr_repro.hip) on one GPU.
#   bash tools/walk_vgpr_repro.sh OUT [PAGES] [REPS]
source tools/gpu_guard.sh
O=gpurun_out/${1:-walkrepro}; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I memcached_amd/csrc tools/walk_vgpr_repro.hip -o /tmp/walk_vgpr_repro &&
    run 300 /tmp/walk_vgpr_repro ${2:-300} ${3:-2} > $O/walk_vgpr_repro.txt 2>&1
