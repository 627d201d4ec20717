#!/bin/bash
source tools/gpu_guard.sh
O=gpurun_out/${1:-x1}; mkdir -p $O
run 600 python bench.py --workload config3 --steps 10 --warmup 2 > $O/config3.json 2> $O/config3.err
run 600 python bench.py --workload config5 --pages ${PAGES:-1000} --steps 5 --warmup 1 > $O/config5.json 2> $O/config5.err
run 600 python bench.py --workload config2r --steps 10 --warmup 2 > $O/config2r.json 2> $O/config2r.err
run 600 python bench.py --workload pagesmix --pages ${PAGES:-1000} --steps 5 --warmup 1 > $O/pagesmix.json 2> $O/pagesmix.err
run 600 python bench.py --workload pages --pages ${PAGES:-1000} --steps 3 --warmup 1 > $O/pages.json 2> $O/pages.err
run 600 python bench.py --workload stamp --pages ${PAGES:-1000} --steps 3 --warmup 1 > $O/stamp.json 2> $O/stamp.err
run 600 python bench.py --workload host --steps 5 --warmup 1 > $O/host.json 2> $O/host.err
run 600 python bench.py --workload calls > $O/calls.json 2> $O/calls.err
run 300 python bench.py --workload multi --gpus 1 --steps 20 --warmup 5 > $O/multi.json 2> $O/multi.err
# PMC instruction census of the span kernels (VALU / LDS per wave-step, wait
# cycles), one pass per counter group (tools/pmctab.py reads them)
export TMPDIR=/tmp
for w in config3 config2r; do
  run 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${w}_a -o a --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 > $O/pmc_${w}_a.log 2>&1
  run 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d $O/pmc_${w}_b -o b --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 > $O/pmc_${w}_b.log 2>&1
done
echo done
