#!/bin/bash
# PMC census of the final K1 (headline shape), two passes of SQ counters.
#   bash tools/r04_k1pmc.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_k1pmc}; mkdir -p $O
a="--steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline"
run 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_a -o a --output-format csv -- python3 bench.py $a > $O/pmc_a.log 2>&1
run 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/pmc_b -o b --output-format csv -- python3 bench.py $a > $O/pmc_b.log 2>&1
echo done
