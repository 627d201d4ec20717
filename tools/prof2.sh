#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/p2; mkdir -p $O
cd tools
run 300 ./ubench 1048576 10 > ../$O/ablate.log 2>&1
for V in 4_l32_c32_r4_m0 1_l64_c32_r2_m0; do
run 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d ../$O/pa_$V -o pa --output-format csv -- ./ubench 1048576 2 $V 1024 > ../$O/pa_$V.log 2>&1
run 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL -d ../$O/pb_$V -o pb --output-format csv -- ./ubench 1048576 2 $V 1024 > ../$O/pb_$V.log 2>&1
run 200 rocprofv3 --kernel-trace --stats -d ../$O/kt_$V -o kt --output-format csv -- ./ubench 1048576 5 $V 1024 > ../$O/kt_$V.log 2>&1
done
echo done
