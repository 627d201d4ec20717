#!/bin/bash
# Final-build span evidence: config 3 HBM traffic with the balanced plan
# (FETCH_SIZE and WRITE_SIZE in separate passes) and the kernel split of the
# mixed pages.
#   bash tools/final_spans.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-fspans}; mkdir -p $O
run 120 rocprofv3 --pmc FETCH_SIZE -d $O/config3_fetch -o fetch --output-format csv -- python3 bench.py --workload config3 --steps 2 --warmup 1 > $O/config3_fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE -d $O/config3_write -o write --output-format csv -- python3 bench.py --workload config3 --steps 2 --warmup 1 > $O/config3_write.log 2>&1
run 300 rocprofv3 --kernel-trace --stats -d $O/kt_mix -o mix --output-format csv -- python3 bench.py --workload pagesmix --pages 300 --steps 3 --warmup 1 > $O/kt_mix.json 2> $O/kt_mix.err
echo done
