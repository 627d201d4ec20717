#!/bin/bash
# The 64-bit shift / top-VGPR experiment (tools/shift64_top_vgpr.hip) on one
# GPU, after checking on the CPU that each kernel takes the amount from the
# register and allocation its name says.
#   bash tools/shift64_top_vgpr.sh OUT [PAGES]
source tools/gpu_guard.sh
O=gpurun_out/${1:-shift64}; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/shift64_top_vgpr.hip --cuda-device-only -S -o $O/shift64_top_vgpr.s &&
    python3 tools/shift64_asm_check.py $O/shift64_top_vgpr.s > $O/asm_check.txt &&
    hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/shift64_top_vgpr.hip -o /tmp/shift64_top_vgpr &&
    run 300 /tmp/shift64_top_vgpr ${2:-300} > $O/shift64_top_vgpr.txt 2>&1
