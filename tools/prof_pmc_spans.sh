#!/bin/bash
# PMC counters: K1 (config 2) vs the span kernel on 4133-B spans (config2r).
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}; mkdir -p $O
for w in ${WL:-config2 config2r}; do
  run 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $O/${w}_a -o a --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $O/${w}_a.log 2>&1
  run 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD -d $O/${w}_b -o b --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $O/${w}_b.log 2>&1
done
echo done
