#!/bin/bash
# Round 6: dynamic instruction mix per byte, K1 (headline) against the span
# kernel (config 3) and K5 (config 5): one --pmc pass per workload.
#   bash tools/r06/insts_pmc.sh OUT
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_insts}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM_WR"
run 120 rocprofv3 --pmc $C -d $O/k1 -o k1 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/k1.log 2>&1
run 300 rocprofv3 --pmc $C -d $O/c3 -o c3 --output-format csv -- python3 bench.py --workload config3 --steps 2 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/c3.log 2>&1
run 300 rocprofv3 --pmc $C -d $O/c5 -o c5 --output-format csv -- python3 bench.py --workload config5 --pages 300 --steps 2 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/c5.log 2>&1
echo done
