#!/bin/bash
# Round 6: K1 half-step ring depth (tools/k1_ring), then the span-kernel
# suite + A/B (tools/r06/spans_ab.sh).
#   bash tools/r06/combo1.sh OUT ROUNDS
source tools/gpu_guard.sh
mkdir -p gpurun_out/$1
run 300 tools/k1_ring 30 > gpurun_out/$1/k1_ring.txt 2>&1
bash tools/r06/spans_ab.sh $1 ${2:-2}
