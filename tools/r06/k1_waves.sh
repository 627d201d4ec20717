#!/bin/bash
# Round 6: K1 / register / LDS-DMA streams by waves per CU (tools/k1_waves.hip)
#   bash tools/r06/k1_waves.sh OUT
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_k1w}; mkdir -p $O
run 300 tools/k1_waves 30 > $O/k1_waves.txt 2>&1
