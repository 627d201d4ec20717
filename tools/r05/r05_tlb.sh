#!/bin/bash
# Round 5: address-translation counters of the mixed pages at 300 and 1000
# pages (the span kernel reads 7-8 % slower per byte at 1000 pages).
#   bash tools/r05_tlb.sh OUT
source tools/gpu_guard.sh
export TMPDIR=/tmp
O=gpurun_out/${1:-r05tlb}; mkdir -p $O
run 120 rocprofv3 --list-avail > $O/avail.txt 2>&1
grep -i -E "UTCL|TLB|TRANSLATION" $O/avail.txt | head -40 > $O/avail_tlb.txt
for p in 300 1000; do
  run 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum -d $O/tlb_$p -o p --output-format csv -- python3 bench.py --workload pagesmix --pages $p --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline > $O/tlb_$p.log 2>&1
done
echo done
