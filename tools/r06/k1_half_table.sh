#!/bin/bash
# Round 6: what an LDS-DMA K1 would pay first -- K1 with a half-replicated
# table image (two-way bank conflicts on every lookup; ab/k1half) against the
# product (ab/cur): headline A/B, alternating, and one PMC pass each.
#   bash tools/r06/k1_half_table.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_k1half}; R=${2:-3}
mkdir -p $O
for r in $(seq 1 $R); do
  for n in cur k1half; do
    echo "== round $r lib $n" >> $O/ab.txt
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python bench.py --no-cpu-baseline >> $O/ab.txt 2>> $O/ab.err
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for n in cur k1half; do
  MCRC_LIB=ab/$n/libmcrc32c.so run 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$n -o pmc --output-format csv -- python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/pmc_$n.log 2>&1
done
echo done
