#!/bin/bash
# Round 5: per-batch kernel split and the span kernel's PMC census, config 3,
# shipped build (ab/head) against the line grid with nt pieces (ab/lgnt).
#   bash tools/r05_lgtrace.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05lgt}; mkdir -p $O
for n in head lgnt; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o kt --output-format csv -- python3 bench.py --workload config3 --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_$n.json 2> $O/kt_$n.err
  MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${n}_a -o a --output-format csv -- python3 bench.py --workload config3 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${n}_a.log 2>&1
  MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/pmc_${n}_b -o b --output-format csv -- python3 bench.py --workload config3 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_${n}_b.log 2>&1
  MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$n -o f --output-format csv -- python3 bench.py --workload config3 --steps 2 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/fetch_$n.log 2>&1
done
echo done
