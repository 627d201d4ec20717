#!/bin/bash
# PMC census of the planned path's kernels (k_count, k_spans, k_expand) on
# config 3 and the mixed pages: two passes of SQ counters each.
#   bash tools/r04_pmc_count.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_pmc_count}; mkdir -p $O
for w in config3 pagesmix; do
  a="--workload $w --steps 2 --warmup 1 --settle-ms 0"; [ $w = pagesmix ] && a="$a --pages 100"
  run 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${w}_a -o a --output-format csv -- python3 bench.py $a > $O/pmc_${w}_a.log 2>&1
  run 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/pmc_${w}_b -o b --output-format csv -- python3 bench.py $a > $O/pmc_${w}_b.log 2>&1
done

echo done
