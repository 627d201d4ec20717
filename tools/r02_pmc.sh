#!/bin/bash
# PMC instruction census of the span kernel: cur vs given ablation libs.
#   bash tools/r02_pmc.sh OUT WORKLOAD lib...   (lib: cur or abl name)
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/$1; W=$2; shift 2; mkdir -p $O
for v in "$@"; do
  lib=$PWD/abl/libmcrc32c_$v.so; [ $v = cur ] && lib=
  MCRC_LIB=$lib run 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/${v}_a -o a --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --pages 100 > $O/${v}_a.log 2>&1
  MCRC_LIB=$lib run 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/${v}_b -o b --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --pages 100 > $O/${v}_b.log 2>&1
done
echo done
