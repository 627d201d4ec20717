#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/p4; mkdir -p $O
for V in 4_l32_c64_r2_m1 4_l32_c64_r2_m3 4_l32_c64_r2_m0 4_l32_c64_r2_m5; do
run 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/pa_$V -o pa --output-format csv -- ./tools/ubench 1048576 3 $V 1024 > $O/pa_$V.log 2>&1
done
echo done
