#!/bin/bash
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/p3; mkdir -p $O
run 300 ./tools/ubench 1048576 20 4_l32_c64_r2_m0 1024 > $O/ubench.log 2>&1
run 300 python bench.py --steps 50 --no-cpu-baseline > $O/bench50.json 2>$O/bench50.err
run 300 ./tools/ubench 1048576 20 4_l32_c64_r2_m0 1024 >> $O/ubench.log 2>&1
run 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py --steps 20 --no-cpu-baseline > $O/kt.log 2>&1
run 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/pa -o pa --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pa.log 2>&1
run 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/pu -o pu --output-format csv -- ./tools/ubench 1048576 5 4_l32_c64_r2_m0 1024 > $O/pu.log 2>&1
run 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o pf --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pf.log 2>&1
run 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o pw --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pw.log 2>&1
echo done
