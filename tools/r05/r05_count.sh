#!/bin/bash
# Round 5: per-batch kernel split (kernel trace) and k_count's PMC census on
# mixed pages and config 3, working-tree build.
#   bash tools/r05_count.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05cnt}; mkdir -p $O
for w in pagesmix config3; do
  run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$w -o kt --output-format csv -- python3 bench.py --workload $w --pages 300 --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$w.json 2> $O/kt_$w.err
  run 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${w}_a -o a --output-format csv -- python3 bench.py --workload $w --pages 300 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${w}_a.log 2>&1
  run 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/pmc_${w}_b -o b --output-format csv -- python3 bench.py --workload $w --pages 300 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${w}_b.log 2>&1
done
echo done
