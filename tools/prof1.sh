#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/p1; mkdir -p $O
cd tools
run 60 rocprofv3 -L > ../$O/counters.txt 2>&1
run 120 ./ubench 32768 200 "crc ch32 r2" 1024 > ../$O/l2res.log 2>&1
run 120 ./ubench 32768 200 "crc ch64 r1" 1024 >> ../$O/l2res.log 2>&1
run 120 ./ubench 32768 200 "crc ch16 r4" 1024 >> ../$O/l2res.log 2>&1
run 120 ./ubench 32768 200 "load ch32 r2" 1024 >> ../$O/l2res.log 2>&1
run 200 rocprofv3 --kernel-trace --stats -d ../$O/kt -o kt --output-format csv -- ./ubench 1048576 5 "crc ch32 r2" 1024 > ../$O/kt.log 2>&1
run 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d ../$O/pa -o pa --output-format csv -- ./ubench 1048576 2 "crc ch32 r2" 1024 > ../$O/pa.log 2>&1
run 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL -d ../$O/pb -o pb --output-format csv -- ./ubench 1048576 2 "crc ch32 r2" 1024 > ../$O/pb.log 2>&1
run 200 rocprofv3 --pmc FETCH_SIZE -d ../$O/pc -o pc --output-format csv -- ./ubench 1048576 2 "crc ch32 r2" 1024 > ../$O/pc.log 2>&1
echo done
