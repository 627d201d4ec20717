#!/bin/bash
# Round 6: small planned page verifies (< 4096 items), HEAD vs cur, alternating.
#   bash tools/r06/pages_small_ab.sh OUT ROUNDS
source tools/gpu_guard.sh
O=gpurun_out/${1:-r06_psmall}; R=${2:-2}
mkdir -p $O
for r in $(seq 1 $R); do
  for n in HEAD cur; do
    MCRC_LIB=ab/$n/libmcrc32c.so run 300 python tools/r06/pages_small_ab.py >> $O/ab.jsonl 2>> $O/ab.err
  done
done
echo done
