#!/bin/bash
# Round 6: effective clock of K1 against the plain register stream
# (GRBM_GUI_ACTIVE cycles / kernel duration per dispatch), one PMC pass with
# the kernel trace, over tools/k1_waves 3 (no settle at REPS <= 1; REPS 3
# settles 300 ms first).
#   bash tools/r06/k1_clock.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_clock}; mkdir -p $O
run 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES -d $O/pmc -o pmc --output-format csv -- tools/k1_waves 3 > $O/k1_waves_pmc.txt 2>&1
